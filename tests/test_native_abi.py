"""The C-ABI library loads and exports every symbol include/hockey.h declares (no GPU needed, no
compute calls), and the ctypes structures match the header's layout."""
import ctypes
import os
import re

import pytest

from conftest import ROOT


def _declared():
    src = open(os.path.join(ROOT, "include", "hockey.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hk_[a-z0-9_]+)\s*\(", src)))


def test_header_declares_boundary():
    names = _declared()
    for required in ("hk_create", "hk_destroy", "hk_reset", "hk_step", "hk_get_state", "hk_set_state",
                     "hk_observe", "hk_last_error"):
        assert required in names


def test_library_exports_every_declared_symbol():
    from hockey_amd import _native as N

    if not os.path.exists(N.LIB_PATH):
        N.build()
    L = ctypes.CDLL(N.LIB_PATH)
    missing = [n for n in _declared() if not hasattr(L, n)]
    assert not missing, missing
    assert set(_declared()) == set(N.EXPORTS)
    lib = N.lib()
    assert b"gfx950" in lib.hk_version()


def test_ctypes_struct_layout_matches_header(tmp_path):
    """Sizes and field offsets of hk_config / hk_step_io as the C compiler lays them out from the header."""
    import subprocess

    from hockey_amd import _native as N

    probes = {"Config": ("hk_config", [f for f, _ in N.Config._fields_]),
              "StepIO": ("hk_step_io", [f for f, _ in N.StepIO._fields_])}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hockey.h"', "int main(void) {"]
    for cname, fields in probes.values():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f in fields:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    want = dict(line.split() for line in subprocess.check_output([str(exe)], text=True).splitlines())
    for pyname, (cname, fields) in probes.items():
        S = getattr(N, pyname)
        assert ctypes.sizeof(S) == int(want[cname]), cname
        for f in fields:
            assert getattr(S, f).offset == int(want[f"{cname}.{f}"]), (cname, f)


def test_product_has_no_cpu_fallback(monkeypatch, tmp_path):
    """Missing native library -> loud failure, never a silent Python/oracle path."""
    from hockey_amd import _native as N

    monkeypatch.setattr(N, "LIB_PATH", str(tmp_path / "missing.so"))
    monkeypatch.setattr(N, "_lib", None)
    with pytest.raises(N.HockeyNativeError):
        N.lib()


def test_product_never_imports_the_oracle():
    pkg = os.path.join(ROOT, "hockey-env_amd")
    for dirpath, _, files in os.walk(pkg):
        for f in files:
            if f.endswith((".py", ".cpp", ".hip", ".h")):
                text = open(os.path.join(dirpath, f), errors="replace").read()
                assert "hk_oracle" not in text and "import oracle" not in text, f


def test_source_hash_matches_makefile_recipe():
    """bench.py's counter provenance: hockey_amd._native.source_hash() hashes exactly the Makefile's HASHSRC
    list (SRC, HDR, Makefile) in its order, so it equals the .srchash sidecar make writes next to the library."""
    import hashlib
    import subprocess

    from hockey_amd import _native as N

    mk = open(os.path.join(N.CSRC, "Makefile")).read()

    def var(name):
        return re.search(rf"^{name} = (.*)$", mk, flags=re.M).group(1).split()

    assert re.search(r"^HASHSRC = \$\(SRC\) \$\(HDR\) Makefile$", mk, flags=re.M)
    assert var("SRC") + var("HDR") + ["Makefile"] == N.HASH_SOURCES
    cat = b"".join(open(os.path.join(N.CSRC, f), "rb").read() for f in N.HASH_SOURCES)
    assert N.source_hash() == hashlib.sha256(cat).hexdigest()[:12]
    out = subprocess.check_output(f"cat {' '.join(N.HASH_SOURCES)} | sha256sum | cut -c1-12", shell=True,
                                  cwd=N.CSRC, text=True).strip()
    assert out == N.source_hash()


def test_facade_action_staging_matches_numpy_clip():
    """hockey_env._stage_actions (the facade's per-step action staging) stores exactly
    float32(np.clip(np.asarray(action, float64)[0:4], -1, 1)) (hockey_env.py:659, 875-886) for every input kind,
    including NaN, infinities, -0.0 and values that round across +-1 in float32."""
    import numpy as np

    from hockey_amd.hockey_env import _stage_actions

    rng = np.random.default_rng(0)
    cases = [rng.uniform(-3, 3, 4).astype(np.float32), rng.uniform(-3, 3, 8), rng.uniform(-1, 1, 6).astype(np.float16),
             [0.5, -2.0, float("nan"), -0.0], np.array([np.inf, -np.inf, -0.0, 0.99999999], np.float64),
             (1.0000001, -1.0000001, 0.3, 0.2), [1, 2, 3, 4], np.array([1, 2, -3, 0], np.int64),
             np.array([[0.1, 0.2, 0.3, 0.4]]).reshape(4)]
    for c in cases:
        got = np.full(8, 7.0, np.float32)
        _stage_actions(got, c)
        want = np.clip(np.asarray(c, np.float64)[0:4], -1, 1).astype(np.float32)
        assert got[:4].view(np.uint32).tolist() == want.view(np.uint32).tolist(), (c, got, want)
        assert got[4:].view(np.uint32).tolist() == [0, 0, 0, 0]


def test_facade_phase_increment_is_the_reference_draw():
    """HockeyEnv_BasicOpponent.step draws 0.2 * np.random.random(): the same doubles, from the same global stream,
    as the reference's np.random.uniform(0, 0.2) (hockey_env.py:796)."""
    import numpy as np

    np.random.seed(1234)
    want = [np.random.uniform(0, 0.2) for _ in range(20000)]
    np.random.seed(1234)
    got = [0.2 * np.random.random() for _ in range(20000)]
    assert np.array(got).view(np.uint64).tolist() == np.array(want).view(np.uint64).tolist()


def _declared_learner():
    src = open(os.path.join(ROOT, "include", "hockey_learner.h")).read()
    src = re.sub(r"/\*.*?\*/", "", src, flags=re.S)
    return sorted(set(re.findall(r"\b(hkl_[a-z0-9_]+)\s*\(", src)))


def test_learner_library_exports_every_declared_symbol():
    """libhockey_learner.so (the fused TD3 learner, include/hockey_learner.h) loads without a GPU and exports every
    declared entry point; the ctypes binding lists the same set."""
    from hockey_amd import learner_hip as LH

    if not os.path.exists(LH.LIB_PATH):
        import subprocess
        subprocess.check_call(["make", "-s", "-C", os.path.join(ROOT, "hockey-env_amd", "csrc"), "learner"])
    L = ctypes.CDLL(LH.LIB_PATH)
    missing = [n for n in _declared_learner() if not hasattr(L, n)]
    assert not missing, missing
    assert set(_declared_learner()) == set(LH.EXPORTS)
    assert LH.lib().hkl_pack_floats() == LH.PACK_FLOATS


def test_learner_ctypes_struct_layout_matches_header(tmp_path):
    """Sizes and field offsets of the learner's ABI structs as the C compiler lays them out from the header."""
    import subprocess

    from hockey_amd import learner_hip as LH

    probes = {"Net": "hkl_net", "CriticIO": "hkl_critic_io", "ActorIO": "hkl_actor_io", "Seg": "hkl_seg",
              "AdamIO": "hkl_adam_io", "WgJob": "hkl_wgrad_job", "SampleIO": "hkl_sample_io"}
    lines = ['#include <stdio.h>', '#include <stddef.h>', '#include "hockey_learner.h"', "int main(void) {"]
    for py, cname in probes.items():
        lines.append(f'  printf("{cname} %zu\\n", sizeof({cname}));')
        for f, _ in getattr(LH, py)._fields_:
            lines.append(f'  printf("{cname}.{f} %zu\\n", offsetof({cname}, {f}));')
    lines += ["  return 0;", "}"]
    src = tmp_path / "layout.c"
    src.write_text("\n".join(lines))
    exe = tmp_path / "layout"
    subprocess.check_call(["gcc", "-I", os.path.join(ROOT, "include"), "-o", str(exe), str(src)])
    want = dict(line.split() for line in subprocess.check_output([str(exe)], text=True).splitlines())
    for py, cname in probes.items():
        S = getattr(LH, py)
        assert ctypes.sizeof(S) == int(want[cname]), cname
        for f, _ in S._fields_:
            assert getattr(S, f).offset == int(want[f"{cname}.{f}"]), (cname, f)


def test_learner_adam_rejects_incomplete_io_before_any_launch():
    """hkl_adam validates its pointers on the host (no GPU needed): loss partials without a destination, or a folded
    soft update without target twins, return HKL_E_INVALID instead of launching a kernel that would write through a
    null pointer."""
    from hockey_amd import learner_hip as LH

    L = LH.lib()
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    io = LH.AdamIO()
    io.seg[0] = LH.Seg(p, p, p, p, 1, 8, 8, 1, 8, p)
    io.n_seg = 1
    io.loss_src = p  # loss partials, but no loss_sum / loss_count
    assert L.hkl_adam(ctypes.byref(io), None) == 1
    io.loss_src = None
    io.polyak = 1
    io.seg[0].target = None  # soft update asked, no target twin
    assert L.hkl_adam(ctypes.byref(io), None) == 1
    io.n_seg = 0
    assert L.hkl_adam(ctypes.byref(io), None) == 1


def test_abi_rejects_invalid_arguments_before_any_launch():
    """Every entry point checks its arguments on the host and fails with HK_E_INVALID and a message naming itself
    (include/hockey.h: 0 or a negative HK_E* code, hk_last_error() describes it) -- the status-code contract the
    reference's Python callers get as exceptions.  No GPU needed: nothing here reaches a HIP call, except a
    well-formed hk_create, which on a host without a gfx950 device must fail with HK_E_DEVICE and leave *out NULL."""
    from hockey_amd import _native as N

    L = N.lib()
    E_INVALID, E_DEVICE = -1, -4

    def cfg(**kw):
        c = N.Config()
        c.keep_mode, c.mode, c.auto_reset, c.vel_ref_semantics, c.seed, c.arena_offset, c.diag_flags = 1, 0, 0, 0, 0, 0, 0
        c.policy[0] = c.policy[1] = 0
        for k, v in kw.items():
            if k == "policy":
                c.policy[0], c.policy[1] = v
            else:
                setattr(c, k, v)
        return c

    def err():
        return L.hk_last_error().decode()

    out = ctypes.c_void_p(1234)
    assert L.hk_create(0, 64, ctypes.byref(cfg()), None) == E_INVALID and "out is NULL" in err()
    for n in (0, -5, (1 << 30) + 1):
        assert L.hk_create(0, n, ctypes.byref(cfg()), ctypes.byref(out)) == E_INVALID, n
        assert "bad n_arenas" in err() and out.value is None
    assert L.hk_create(0, 64, None, ctypes.byref(out)) == E_INVALID and "cfg is NULL" in err()
    for bad, msg in ((dict(mode=3), "bad mode"), (dict(mode=-1), "bad mode"), (dict(policy=(9, 0)), "bad policy"),
                     (dict(policy=(0, -2)), "bad policy"), (dict(diag_flags=1 << 7), "unknown diag_flags")):
        assert L.hk_create(0, 64, ctypes.byref(cfg(**bad)), ctypes.byref(out)) == E_INVALID, bad
        assert msg in err(), (bad, err())

    io = N.StepIO()
    buf = (ctypes.c_float * 64)()
    p = ctypes.cast(buf, ctypes.c_void_p)
    cnt = (ctypes.c_int64 * 16)()
    i64 = ctypes.c_int64()
    calls = {"hk_set_policy": lambda: L.hk_set_policy(None, 0, 0),
             "hk_reset": lambda: L.hk_reset(None, None, None, None, None, None),
             "hk_step": lambda: L.hk_step(None, ctypes.byref(io), None),
             "hk_rollout": lambda: L.hk_rollout(None, 4, ctypes.byref(io), None),
             "hk_step_host": lambda: L.hk_step_host(None, p, p, 0, p, None),
             "hk_get_state": lambda: L.hk_get_state(None, p, p, None),
             "hk_set_state": lambda: L.hk_set_state(None, p, p, None, None),
             "hk_observe": lambda: L.hk_observe(None, p, p, None),
             "hk_info": lambda: L.hk_info(None, p, p, p, p, None),
             "hk_opponent_phase": lambda: L.hk_opponent_phase(None, p, p, None),
             "hk_opponent_phase3": lambda: L.hk_opponent_phase3(None, p, p, None),
             "hk_counters": lambda: L.hk_counters(None, cnt, None),
             "hk_reset_counters": lambda: L.hk_reset_counters(None, None),
             "hk_bytes_per_step": lambda: L.hk_bytes_per_step(None, ctypes.byref(i64), ctypes.byref(i64))}
    for name, call in calls.items():
        assert call() == E_INVALID, name
        assert err().startswith(name + ":") and "NULL" in err(), (name, err())
    assert L.hk_num_arenas(None) == 0
    L.hk_destroy(None)  # a no-op, as free(NULL)

    rc = L.hk_create(0, 64, ctypes.byref(cfg()), ctypes.byref(out))
    if rc == 0:  # a gfx950 device is present: the well-formed call succeeds
        L.hk_destroy(out)
    else:
        assert rc == E_DEVICE and out.value is None, (rc, err())
        assert "device" in err()
