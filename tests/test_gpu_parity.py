"""GPU parity: the gfx950 kernels (through the C ABI) vs the CPU oracle and the golden vectors.

Bar (BASELINE north_star: "match ... within a stated fp32 tolerance on fixed seeds"): the stated
tolerance is ZERO -- every float32 obs / state / force and every float32-rounded reward / info value is
bit-identical to the oracle, step after step (kernel and oracle share IEEE op order, no FMA contraction,
correctly rounded div/sqrt, deterministic sin/cos).  Reward / info are compared against the oracle's
float64 value rounded to float32 (the kernel's output dtype).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

torch = pytest.importorskip("torch")

from hockey_amd import _native as N  # noqa: E402
from hockey_amd.placement import np_random, placement  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _gpu():
    assert torch.cuda.is_available(), "GPU tests need the MI355X (gfx950)"
    assert "gfx950" in torch.cuda.get_device_properties(0).gcnArchName


def _vec(n, keep=True, mode=0, **kw):
    from hockey_amd.vec_env import VecHockeyEnv
    return VecHockeyEnv(n, keep_mode=keep, mode=mode, device="cuda:0", **kw)


def _np(t):
    return t.detach().cpu().numpy()


def _f32(x):
    return np.asarray(x, np.float64).astype(np.float32)


# --------------------------------------------------------------------------------------------- goldens
def test_g1_reset_obs_through_kernel(golden):
    g1 = golden("g1_reset.npz")
    for mode in (0, 1, 2):
        idx = np.nonzero(g1["mode"] == mode)[0]
        params = np.zeros((len(idx), 6), np.float32)
        for k, i in enumerate(idx):
            rng, _ = np_random(int(g1["seed"][i]))
            params[k], _ = placement(mode, bool(g1["one_starts"][i]), rng)
        env = _vec(len(idx), mode=mode)
        env.reset_params(params)
        obs, _ = env.observe()
        assert np.array_equal(_np(obs).astype(np.float64), g1["obs"][idx])
        st, aux = env.get_state()
        assert np.array_equal(_np(st), g1["state"][idx])
        env.close()


def test_g2_step_laws_through_kernel(golden):
    g2 = golden("g2_step_presolve.npz")
    bad = {}
    for keep in (True, False):
        for mode in (0, 1, 2):
            idx = np.nonzero((g2["keep_mode"] == int(keep)) & (g2["mode"] == mode))[0]
            if len(idx) == 0:
                continue
            n = len(idx)
            env = _vec(n, keep=keep, mode=mode)
            env.reset_params(np.tile(np.array([8, 4, 3, 4, 0, 0], np.float32), (n, 1)))
            env.set_state(g2["state"][idx], g2["aux"][idx])
            dbg = torch.zeros((n, N.DEBUG_DIM), dtype=torch.float32, device="cuda:0")
            res = env.step(g2["action"][idx], with_agent_two=True, debug=dbg, skip_physics=True)
            st, aux = env.get_state()
            d = _np(dbg)
            got = {"force": d[:, 0:6].reshape(n, 3, 2), "torque": d[:, 6:8], "ldamp": d[:, 8:11],
                   "adamp": d[:, 11:13], "state_after": _np(st), "has_after": _np(aux)[:, 0:3],
                   "obs": _np(res.obs).astype(np.float64), "obs2": _np(res.obs2).astype(np.float64),
                   "done": _np(res.done).astype(np.int32)}
            for f, v in got.items():
                ok = np.all(v.reshape(n, -1) == g2[f][idx].reshape(n, -1), axis=1)
                if not ok.all():
                    bad.setdefault(f, []).extend(idx[~ok][:3].tolist())
            for f, t in (("reward", res.reward), ("reward2", res.reward2), ("info", res.info),
                         ("info2", res.info2)):
                ok = np.all((_np(t).reshape(n, -1) == _f32(g2[f][idx]).reshape(n, -1)), axis=1)
                if not ok.all():
                    bad.setdefault(f, []).extend(idx[~ok][:3].tolist())
            env.close()
    assert not bad, bad


# --------------------------------------------------------------------------------------------- physics
def _oracle_worlds(oracle, n, keep, mode, params, max_t):
    ws = []
    for i in range(n):
        w = oracle.OracleWorld(keep, mode)
        w.reset(params[i], max_t)
        ws.append(w)
    return ws


def _lockstep(oracle, mode, n, steps, seed, policy_mix=True):
    """Step GPU and oracle arenas with identical actions; return the first divergence or None."""
    keep = True
    env = _vec(n, keep=keep, mode=mode)
    params = np.zeros((n, 6), np.float32)
    for i in range(n):
        rng, _ = np_random(seed * 100_000 + i)
        params[i], max_t = placement(mode, bool(i % 2), rng)
    env.reset_params(params)
    ws = _oracle_worlds(oracle, n, keep, mode, params, max_t)
    rng = np.random.default_rng(seed)
    phases = rng.uniform(0, np.pi, (n, 2))
    obs = np.stack([w.obs() for w in ws]).astype(np.float64)
    obs2 = np.stack([w.obs_two() for w in ws]).astype(np.float64)
    n_toi = 0
    for t in range(steps):
        acts = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
        if policy_mix:  # half the arenas play strong-vs-strong BasicOpponent (contacts, shots, goals)
            for i in range(0, n, 2):
                a1, phases[i, 0] = oracle.basic_opponent(0, 1, phases[i, 0], 0.1, obs[i])
                a2, phases[i, 1] = oracle.basic_opponent(0, 1, phases[i, 1], 0.1, obs2[i])
                acts[i] = np.concatenate([a1, a2]).astype(np.float32)
        res = env.step(acts, with_agent_two=True)
        g_obs, g_r, g_d, g_info = _np(res.obs), _np(res.reward), _np(res.done), _np(res.info)
        g_obs2, g_r2 = _np(res.obs2), _np(res.reward2)
        for i, w in enumerate(ws):
            o, r, d, info, _ = w.step(acts[i])
            n_toi += w.stats()[1]
            o2 = w.obs_two()
            i2, r2 = w.info_two()
            checks = (("obs", np.array_equal(g_obs[i], o)), ("obs2", np.array_equal(g_obs2[i], o2)),
                      ("reward", g_r[i] == np.float32(r)), ("reward2", g_r2[i] == np.float32(r2)),
                      ("done", bool(g_d[i]) == d), ("info", np.array_equal(g_info[i], _f32(info))))
            for name, ok in checks:
                if not ok:
                    return {"step": t, "arena": i, "field": name, "gpu_obs": g_obs[i].tolist(), "cpu_obs": o.tolist()}
            obs[i], obs2[i] = o, o2
    st, _ = env.get_state()
    for i, w in enumerate(ws):
        assert np.array_equal(_np(st)[i], w.get_raw()[0]), i
    env.close()
    return {"n_toi": n_toi}


@pytest.mark.parametrize("mode,seed", [(0, 1), (0, 2), (1, 3), (2, 4)])
def test_physics_lockstep_bit_exact(oracle, mode, seed):
    out = _lockstep(oracle, mode, n=128, steps=260, seed=seed)
    assert "field" not in out, out
    if mode == 0:
        assert out["n_toi"] > 0  # continuous collision paths were exercised


def test_fused_basic_opponent_matches_oracle(oracle):
    """policy='strong'/'weak' inside the kernel == BasicOpponent.act on the same obs, phase and increment."""
    n, steps = 96, 120
    env = _vec(n, policies=("strong", "weak"))
    params = np.zeros((n, 6), np.float32)
    for i in range(n):
        rng, _ = np_random(500 + i)
        params[i], max_t = placement(0, bool(i % 2), rng)
    env.reset_params(params)
    rng = np.random.default_rng(11)
    phases = rng.uniform(0, np.pi, (n, 2))
    env.opponent_phase(phases)
    ws = _oracle_worlds(oracle, n, True, 0, params, max_t)
    for t in range(steps):
        inc = rng.uniform(0, 0.2, (n, 2))
        res = env.step(None, opp_inc=inc, record_actions=True)
        ga, go = _np(res.actions), _np(res.obs)
        for i, w in enumerate(ws):
            a1, phases[i, 0] = oracle.basic_opponent(0, 1, phases[i, 0], inc[i, 0], w.obs().astype(np.float64))
            a2, phases[i, 1] = oracle.basic_opponent(1, 1, phases[i, 1], inc[i, 1], w.obs_two().astype(np.float64))
            a = np.concatenate([a1, a2]).astype(np.float32)
            assert np.array_equal(ga[i], a), (t, i, ga[i], a)
            o, *_ = w.step(a)
            assert np.array_equal(go[i], o), (t, i)
    gph = _np(env.opponent_phase())
    assert np.array_equal(gph, phases)
    env.close()


# --------------------------------------------------------------------------------------------- scale
def test_full_size_random_rollout_properties():
    """65 536 arenas (BASELINE config size), device random policy + auto reset: size-independent
    properties -- finite state, mirror symmetry obs2 == mirror(obs), sticky/auto-reset bookkeeping,
    no island-capacity overflow, goals on both sides."""
    n, steps = 65536, 300
    env = _vec(n, policies=("random", "random"), auto_reset=True, seed=123)
    env.reset()
    for _ in range(steps):
        res = env.step(None, with_agent_two=True)
    torch.cuda.synchronize()
    o, o2 = _np(res.obs), _np(res.obs2)
    assert np.isfinite(o).all()
    assert np.array_equal(o2[:, 0:2], -o[:, 6:8]) and np.array_equal(o2[:, 12:16], -o[:, 12:16])
    assert np.array_equal(o2[:, 2], o[:, 8]) and np.array_equal(o2[:, 16], o[:, 17])
    c = env.counters()
    assert c[N.CNT_STEPS] == n * steps
    assert c[N.CNT_OVERFLOW] == 0
    assert c[N.CNT_EPISODES] > 0 and c[N.CNT_GOALS_P1] > 0 and c[N.CNT_GOALS_P2] > 0
    assert c[N.CNT_EPISODES] >= c[N.CNT_GOALS_P1] + c[N.CNT_GOALS_P2]
    st, aux = env.get_state()
    assert (_np(aux)[:, 2] <= 251).all()  # time never exceeds max_t + 1 with auto reset
    env.close()


def test_shard_invariance():
    """An arena's trajectory depends on its GLOBAL id only: the shard [256, 512) run alone with
    arena_offset=256 equals the same arenas inside a 512-arena run (multi-GPU sharding contract)."""
    full = _vec(512, policies=("random", "strong"), auto_reset=True, seed=9)
    part = _vec(256, policies=("random", "strong"), auto_reset=True, seed=9, arena_offset=256)
    for _ in range(200):
        full.step(None)
        part.step(None)
    sf, af = full.get_state()
    sp, ap = part.get_state()
    assert np.array_equal(_np(sf)[256:], _np(sp)) and np.array_equal(_np(af)[256:], _np(ap))


def test_facades_drop_in(golden):
    from hockey_amd.hockey_env import HockeyEnv, HockeyEnv_BasicOpponent, make

    g1 = golden("g1_reset.npz")
    env = HockeyEnv()
    obs, info = env.reset(seed=42)
    row = np.nonzero((g1["mode"] == 0) & (g1["seed"] == 42) & (g1["one_starts"] == 0))[0][0]
    assert np.array_equal(obs, g1["obs"][row]) and info["winner"] == 0 and env.one_starts is False
    o2 = env.obs_agent_two()
    assert np.array_equal(o2[0:2], -obs[6:8])
    for _ in range(5):
        obs, r, d, t, info = env.step(np.zeros(8))
    assert obs.shape == (18,) and isinstance(r, float) and t is False and set(info) >= {"winner"}
    assert env.time == 5
    one = make("Hockey-One-v0")
    assert isinstance(one, HockeyEnv_BasicOpponent) and one.action_space.shape == (4,)
    one.reset(seed=1)
    for _ in range(10):
        obs, r, d, _, info = one.step(np.array([0.5, 0.0, 0.0, 0.0]))
    assert np.isfinite(obs).all()
    with pytest.raises(TypeError):
        env.reset(mode=1)  # reference quirk


@pytest.mark.gpu
@pytest.mark.parametrize("n", [512, 37])
def test_rollout_equals_repeated_steps(n):
    """hk_rollout(K) == K hk_step calls, bit for bit: per-step outputs, final state and counters
    (fused opponents + auto-reset, and external actions).  512 arenas write their observation rows as staged
    16-B stores of whole waves; 37 (one partial wave) takes the per-lane stores."""
    import torch

    k = 37
    for pol in (("strong", "weak"), ("external", "strong")):
        a = _vec(n, policies=pol, auto_reset=True, seed=11)
        b = _vec(n, policies=pol, auto_reset=True, seed=11)
        acts = None
        if pol[0] == "external":
            acts = torch.rand((k, n, 8), device="cuda:0") * 2 - 1
        ro = a.rollout(k, actions=acts, with_agent_two=True, record_actions=True)
        for t in range(k):
            r = b.step(None if acts is None else acts[t], with_agent_two=True, record_actions=True)
            for name in ("obs", "reward", "done", "info", "obs2", "reward2", "info2", "actions"):
                assert torch.equal(getattr(ro, name)[t], getattr(r, name)), (pol, t, name)
        sa, xa = a.get_state()
        sb, xb = b.get_state()
        assert torch.equal(sa, sb) and torch.equal(xa, xb)
        assert np.array_equal(a.counters()[:7], b.counters()[:7])
        a.close()
        b.close()


# --------------------------------------------------------------------------------------------- batched contract
from vec_lockstep import first_mismatch  # noqa: E402

_RES_FIELDS = ("obs", "obs2", "reward", "reward2", "done", "info", "info2", "actions", "final_obs")


def _res_np(res, t=None):
    out = {}
    for f in _RES_FIELDS:
        v = getattr(res, f)
        if v is not None:
            out[f] = _np(v if t is None else v[t])
    return out


def _bench_path_lockstep(oracle, n, steps, mode, policies, seed, offset=0, diag_flags=0, keep_mode=True,
                         vel_ref=False, external=False):
    """GPU (hk_step for the first half, hk_rollout for the rest) vs the oracle's batched context.  external:
    U(-1.2, 1.2) joint actions (clipped in both) for the external players."""
    env = _vec(n, keep=keep_mode, mode=mode, policies=policies, auto_reset=True, seed=seed, arena_offset=offset,
               diag_flags=diag_flags, vel_ref_semantics=vel_ref)
    ov = oracle.OracleVec(n, keep_mode=keep_mode, mode=mode, policies=policies, auto_reset=True, seed=seed,
                          arena_offset=offset, vel_ref=vel_ref)
    rng = np.random.default_rng(seed)
    acts = rng.uniform(-1.2, 1.2, (steps, n, 8)).astype(np.float32) if external else None
    half = steps // 2
    for t in range(half):
        a = None if acts is None else acts[t]
        got = _res_np(env.step(a, with_agent_two=True, record_actions=True, final_obs=True))
        bad = first_mismatch(t, got, ov.step(a, with_agent_two=True, final_obs=True))
        if bad:
            return bad
    ro = env.rollout(steps - half, actions=None if acts is None else torch.as_tensor(acts[half:], device="cuda:0"),
                     with_agent_two=True, record_actions=True, final_obs=True)
    for t in range(steps - half):
        a = None if acts is None else acts[half + t]
        bad = first_mismatch(half + t, _res_np(ro, t), ov.step(a, with_agent_two=True, final_obs=True))
        if bad:
            return bad
    st, aux = env.get_state()
    ost, oaux = ov.get_state()
    assert np.array_equal(_np(st), ost) and np.array_equal(_np(aux), oaux)
    assert np.array_equal(_np(env.opponent_phase()), ov.phase())
    c, oc = env.counters(), ov.counters()
    assert np.array_equal(c[:5], oc[:5]), (c[:7], oc[:7])
    env.close()
    return {"counters": c}


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_keep_mode_false_with_physics_lockstep_vs_oracle(oracle, mode):
    """Hockey-v0 with keep_mode=False (hockey_env.py:91): player 2's action at index 3 (:663), no hold / shoot
    (:668-680), world.Step running -- external random actions against the fused BasicOpponent(keep_mode=False),
    then bot vs bot, bit-exact through hk_step and hk_rollout in every mode."""
    out = _bench_path_lockstep(oracle, 128, 300, mode, ("external", "strong"), seed=60 + mode, keep_mode=False,
                               external=True)
    assert "field" not in out, out
    out = _bench_path_lockstep(oracle, 128, 300, mode, ("weak", "strong"), seed=63 + mode, keep_mode=False)
    assert "field" not in out, out
    assert out["counters"][N.CNT_EPISODES] > 0


def test_live_velocity_semantics_with_physics_lockstep_vs_oracle(oracle):
    """vel_ref_semantics=1 (live-reference velocity getters in _check_boundaries,
    hockey_env.py:425-432) with world.Step running, bit-exact against the oracle."""
    out = _bench_path_lockstep(oracle, 128, 300, 0, ("external", "external"), seed=66, vel_ref=True, external=True)
    assert "field" not in out, out
    out = _bench_path_lockstep(oracle, 256, 400, 0, ("strong", "strong"), seed=67, vel_ref=True)
    assert "field" not in out, out
    assert out["counters"][N.CNT_TOI] > 0


@pytest.mark.parametrize("mode,steps", [(0, 600), (1, 300), (2, 300)])
def test_bench_path_lockstep_vs_oracle(oracle, mode, steps):
    """THE benchmarked workload -- strong-vs-strong BasicOpponent fused in the kernel, in-kernel Philox
    phase increments (opp_inc NULL), auto-reset with device Philox placement -- bit-exact against the
    oracle's independent restatement, through hk_step and hk_rollout, in all three modes (every arena
    rolls over at least twice; TRAIN_SHOOTING / TRAIN_DEFENSE device resets included)."""
    n = 256
    out = _bench_path_lockstep(oracle, n, steps, mode, ("strong", "strong"), seed=40 + mode)
    assert "field" not in out, out
    assert out["counters"][N.CNT_EPISODES] >= 2 * n
    assert out["counters"][N.CNT_TOI] > 0


def test_random_policies_lockstep_vs_oracle(oracle):
    """C2/C4's random-vs-random Philox actions (and a weak opponent) on a shard with a global offset."""
    out = _bench_path_lockstep(oracle, 256, 400, 0, ("random", "random"), seed=3, offset=77_000)
    assert "field" not in out, out
    out = _bench_path_lockstep(oracle, 128, 300, 1, ("random", "weak"), seed=4, offset=5)
    assert "field" not in out, out


def test_per_step_opponent_mix_lockstep_vs_oracle(oracle):
    """C5's opponent mix (rl/training/opponent_manager.py:62-91): player 2's policy drawn per arena and step
    from {external (self-play actions), weak bot, strong bot} through hk_step_io.policy2, each bot with its
    own phase -- bit-exact against the oracle over episodes with auto-reset."""
    n, steps = 256, 400
    env = _vec(n, mode=0, policies=("external", "external"), auto_reset=True, seed=31)
    ov = oracle.OracleVec(n, mode=0, policies=("external", "external"), auto_reset=True, seed=31)
    rng = np.random.default_rng(31)
    for t in range(steps):
        a = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
        p2 = rng.choice(np.array([0, 2, 3], np.uint8), n)
        got = _res_np(env.step(a, with_agent_two=True, record_actions=True, final_obs=True,
                               policy2=torch.as_tensor(p2, device="cuda:0")))
        want = ov.step(a, with_agent_two=True, final_obs=True, policy2=p2)
        bad = first_mismatch(t, got, want)
        assert bad is None, bad
    st, aux = env.get_state()
    ost, oaux = ov.get_state()
    assert np.array_equal(st.cpu().numpy(), ost) and np.array_equal(aux.cpu().numpy(), oaux)
    assert env.counters()[N.CNT_EPISODES] > 0
    env.close()


def test_large_island_path_on_gpu_vs_oracle(oracle):
    """HK_DIAG_LARGE_ISLANDS: every island / TOI mini-island solved on the HBM slot file (the path islands
    beyond the register slots take in production) -- bit-exact on gfx950 too."""
    out = _bench_path_lockstep(oracle, 128, 300, 0, ("strong", "strong"), seed=8, diag_flags=N.DIAG_LARGE_ISLANDS)
    assert "field" not in out, out
    assert out["counters"][N.CNT_TOI] > 0


def test_autoreset_external_policy_transitions(oracle):
    """auto_reset with an external player: obs after a done step is the NEW episode's first state (so the
    next action is chosen from it), final_obs holds the terminal observation."""
    n, steps = 128, 300
    env = _vec(n, mode=2, policies=("external", "strong"), auto_reset=True, seed=12)
    ov = oracle.OracleVec(n, mode=2, policies=("external", "strong"), auto_reset=True, seed=12)
    rng = np.random.default_rng(0)
    resets = 0
    for t in range(steps):
        a = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
        got = _res_np(env.step(a, with_agent_two=True, record_actions=True, final_obs=True))
        want = ov.step(a, with_agent_two=True, final_obs=True)
        assert first_mismatch(t, got, want) is None
        d = got["done"].astype(bool)
        resets += int(d.sum())
        assert np.array_equal(got["obs"][~d], got["final_obs"][~d])
        if d.any():  # a fresh TRAIN_DEFENSE placement: player 1 at (2, 4) at rest, time 0
            assert np.all(got["obs"][d, 0:6] == np.array([-3, 0, 0, 0, 0, 0], np.float32))
    assert resets > n
    env.close()


def test_c4_shard_131072_arenas(oracle):
    """BASELINE C4's per-GPU shard: 131 072 arenas (random vs random, auto-reset).  Checks: counters and
    finiteness at full size, 1 x 131 072 == 2 x 65 536 shard contexts with global offsets bit for bit, and
    three 256-arena blocks (start, middle, end) equal, at every step, to the oracle run with the same global ids."""
    n, steps, seed = 131072, 300, 2024
    full = _vec(n, policies=("random", "random"), auto_reset=True, seed=seed, arena_offset=n)  # rank 1 of C4
    halves = [_vec(n // 2, policies=("random", "random"), auto_reset=True, seed=seed, arena_offset=n + k * n // 2)
              for k in range(2)]
    blocks = (0, n // 2 - 128, n - 256)
    ovs = [oracle.OracleVec(256, policies=("random", "random"), auto_reset=True, seed=seed, arena_offset=n + b)
           for b in blocks]
    for t in range(steps):
        res = full.step(None, with_agent_two=True, final_obs=True)
        for h in halves:
            h.step(None)
        for b, ov in zip(blocks, ovs):  # every step's outputs of the three blocks (sliced on the device)
            want = ov.step(with_agent_two=True, final_obs=True)
            sl = {f: _np(getattr(res, f)[b:b + 256]) for f in ("obs", "obs2", "reward", "reward2", "done", "info",
                                                                  "info2", "final_obs")}
            bad = first_mismatch(t, sl, want, fields=tuple(sl))
            assert bad is None, (b, bad)
    torch.cuda.synchronize()
    st, aux = full.get_state()
    st, aux = _np(st), _np(aux)
    assert np.isfinite(st).all()
    for k, h in enumerate(halves):
        hs, ha = h.get_state()
        assert np.array_equal(st[k * n // 2:(k + 1) * n // 2], _np(hs))
        assert np.array_equal(aux[k * n // 2:(k + 1) * n // 2], _np(ha))
    for b, ov in zip(blocks, ovs):
        ost, oaux = ov.get_state()
        assert np.array_equal(st[b:b + 256], ost) and np.array_equal(aux[b:b + 256], oaux)
    c = full.counters()
    assert c[N.CNT_STEPS] == n * steps and c[N.CNT_OVERFLOW] == 0
    assert c[N.CNT_EPISODES] > 0 and c[N.CNT_GOALS_P1] > 0 and c[N.CNT_GOALS_P2] > 0
    ch = sum(h.counters() for h in halves)
    assert np.array_equal(c[:7], ch[:7])
    for e in [full, *halves]:
        e.close()


def test_policy2_validation_and_phase_rows():
    """hk_step rejects a policy2 override without io.actions (an override may pick EXTERNAL); an id that is
    not an HK_POLICY_* is counted in HK_CNT_BAD_POLICY and that player acts with zeros, never as a bot; and
    hk_opponent_phase3 reads / writes all three phase rows ([N,3])."""
    n = 128
    env = _vec(n, policies=("strong", "strong"), auto_reset=True, seed=5)
    p2 = torch.full((n,), 2, dtype=torch.uint8, device="cuda:0")
    with pytest.raises(N.HockeyNativeError, match="policy2"):
        env.step(None, policy2=p2)
    ph = torch.rand((n, 3), dtype=torch.float64, device="cuda:0") * 3
    env.opponent_phase(ph, rows=3)
    assert torch.equal(env.opponent_phase(rows=3), ph)
    assert torch.equal(env.opponent_phase(), ph[:, :2])
    acts = torch.zeros((n, 8), device="cuda:0")
    p2[: n // 2] = 7  # invalid ids
    env.reset_counters()
    res = env.step(acts, policy2=p2, record_actions=True)
    a = _np(res.actions)
    assert np.all(a[: n // 2, 4:8] == 0)  # zeros, not a bot
    assert np.any(a[n // 2:, 4:8] != 0)   # the weak bot acts where the id is valid
    c = env.counters()
    assert c[N.CNT_BAD_POLICY] == n // 2 and c[N.CNT_STEPS] == n
    ph2 = _np(env.opponent_phase(rows=3))
    ph0 = _np(ph)
    assert np.array_equal(ph2[: n // 2, 1:], ph0[: n // 2, 1:])  # no bot walked player 2's rows there
    assert np.all(ph2[n // 2:, 2] != ph0[n // 2:, 2]) and np.array_equal(ph2[n // 2:, 1], ph0[n // 2:, 1])
    env.close()


@pytest.mark.parametrize("n", [1, 37, 100])
def test_partial_wave_lockstep_vs_oracle(oracle, n):
    """Contexts whose last wave is partial (1, 37, 100 arenas): the wave-cooperative TOI and narrow-phase
    drains deal their work to the ACTIVE lanes only -- bit-exact against the oracle on the TOI-heavy
    strong-vs-strong workload with device auto-reset."""
    out = _bench_path_lockstep(oracle, n, 300, 0, ("strong", "strong"), seed=70 + n)
    assert "field" not in out, out
    out = _bench_path_lockstep(oracle, n, 200, 2, ("external", "weak"), seed=80 + n, external=True)
    assert "field" not in out, out


def test_rejected_calls_leave_the_context_intact():
    """Every argument check on a live context fails with HK_E_INVALID before it launches anything (a missing
    io.actions for an external player, n_steps < 1, hk_step_host on a multi-arena context, a bad player / policy id,
    a missing counters buffer), and the context then steps on exactly as a twin that never saw the bad calls:
    bit-identical obs, reward, done and state after 40 steps."""
    import ctypes

    n = 100
    env, twin = (_vec(n, policies=("external", "strong"), auto_reset=True, seed=11) for _ in range(2))
    L = env.L
    io = N.StepIO()
    io.obs = env.obs_buf.data_ptr()
    assert L.hk_step(env._ctx, ctypes.byref(io), env._stream()) == -1 and b"io->actions is NULL" in L.hk_last_error()
    acts = torch.rand((n, 8), device="cuda:0") * 2 - 1
    io.actions = acts.data_ptr()
    for k in (0, -3):
        assert L.hk_rollout(env._ctx, k, ctypes.byref(io), env._stream()) == -1 and b"n_steps" in L.hk_last_error()
    host = (ctypes.c_float * 64)()
    hp = ctypes.cast(host, ctypes.c_void_p)
    assert L.hk_step_host(env._ctx, hp, hp, 0, hp, None) == -1 and b"single-arena" in L.hk_last_error()
    for player, pol in ((2, 0), (-1, 0), (1, 99)):
        assert L.hk_set_policy(env._ctx, player, pol) == -1 and b"hk_set_policy" in L.hk_last_error()
    assert L.hk_counters(env._ctx, None, env._stream()) == -1
    g = torch.Generator(device="cuda:0").manual_seed(3)
    for _ in range(40):
        a = torch.rand((n, 8), device="cuda:0", generator=g) * 2 - 1
        r1, r2 = env.step(a), twin.step(a)
        for f in ("obs", "reward", "done", "info"):
            assert torch.equal(getattr(r1, f), getattr(r2, f)), f
    s1, s2 = env.get_state(), twin.get_state()
    for x, y in zip(s1, s2):
        assert torch.equal(x, y)
    env.close()
    twin.close()


def _digest_torch(res):
    """Order-sensitive 64-bit digest of a step's obs / reward / done / info (wrapping int64 arithmetic)."""
    tot = torch.zeros((), dtype=torch.int64, device="cuda:0")
    for t in (res.obs, res.reward, res.done, res.info):
        bits = (t.view(torch.int32) if t.dtype == torch.float32 else t.to(torch.int32)).reshape(-1).to(torch.int64)
        w = (torch.arange(bits.numel(), device="cuda:0", dtype=torch.int64) * 2654435761 + 1) % (1 << 31)
        tot = tot * 1000003 + (bits * w).sum()
    return int(tot.item())


def _digest_np(out):
    tot = np.int64(0)
    with np.errstate(over="ignore"):
        for k in ("obs", "reward", "done", "info"):
            a = out[k]
            bits = (a.view(np.int32) if a.dtype == np.float32 else a.astype(np.int32)).reshape(-1).astype(np.int64)
            w = (np.arange(bits.size, dtype=np.int64) * 2654435761 + 1) % (1 << 31)
            tot = tot * np.int64(1000003) + (bits * w).sum(dtype=np.int64)
    return int(tot)


def test_benchmarked_trajectories_bit_exact_at_full_size(oracle):
    """bench.py's own workload at its own size -- 65 536 arenas, strong vs strong fused, auto-reset, seed 0,
    env.reset(), the 1 000-step pre-roll as hk_rollout launches without outputs, then 500 hk_step launches with
    obs / reward / done / info -- against the oracle's batched context stepped alongside: every step's outputs
    equal (a 64-bit digest of all 65 536 rows per step, the full arrays at the last step), and the final state,
    phases and counters equal.  The throughput figure is measured on exactly these trajectories."""
    import bench

    n, pre, steps = 65536, 1000, 500
    env = _vec(n, policies=("strong", "strong"), auto_reset=True, seed=0)
    env.reset()
    ov = oracle.OracleVec(n, policies=("strong", "strong"), auto_reset=True, seed=0)
    ov.reset(one_starts=env.one_starts.astype(np.uint8))
    bench.preroll(env, pre, N)
    for _ in range(pre):
        ov.step()
    for t in range(steps):
        res = env.step()
        want = ov.step()
        assert _digest_torch(res) == _digest_np(want), f"step {pre + t}"
    for k in ("obs", "reward", "done", "info"):
        assert np.array_equal(_np(getattr(res, k)), want[k]), k
    st, aux = env.get_state()
    ost, oaux = ov.get_state()
    assert np.array_equal(_np(st), ost) and np.array_equal(_np(aux), oaux)
    assert np.array_equal(_np(env.opponent_phase()), ov.phase())
    c, oc = env.counters(), ov.counters()
    assert np.array_equal(c[:5], oc[:5]), (c[:7], oc[:7])
    assert c[N.CNT_EPISODES] > n and c[N.CNT_TOI] > 0
    env.close()
    ov.close()


def test_packed_int_words_round_trip_and_range_checks():
    """r06 packs an arena's 12 int words into 6 (hk_kernels.h PW_*): every value in range round-trips through
    hk_set_state / hk_get_state, hk_step keeps the oracle's time / has_puck / winner semantics (the lockstep tests), and
    out-of-range aux / max_t rows of the selected arenas are rejected with HK_E_INVALID before anything runs."""
    from hockey_amd._native import HockeyNativeError
    from hockey_amd.vec_env import VecHockeyEnv

    n = 8
    env = VecHockeyEnv(n, device="cuda:0")
    env.reset(seeds=list(range(n)))
    st, aux = env.get_state()
    want = torch.tensor([[0, 0, 0, 0, 0], [15, 0, 251, 1, 1], [0, 15, 7, 1, -1], [255, 255, 123456789, 0, 0],
                         [3, 4, 2**31 - 1, 1, 1], [1, 2, 3, 0, -1], [0, 0, 0, 1, 0], [9, 0, 80, 0, 1]],
                        dtype=torch.int32, device="cuda:0")
    env.set_state(aux=want)
    _, got = env.get_state()
    assert torch.equal(got, want)
    for bad in ([256, 0, 0, 0, 0], [0, -1, 0, 0, 0], [0, 0, 0, 2, 0], [0, 0, 0, 0, 2], [0, 0, 0, 0, -2]):
        rows = want.clone()
        rows[5] = torch.tensor(bad, dtype=torch.int32)
        with pytest.raises(HockeyNativeError):
            env.set_state(aux=rows)
        mask = torch.ones(n, dtype=torch.uint8)
        mask[5] = 0
        env.set_state(aux=rows, mask=mask)  # the bad row is not selected: accepted
    _, got = env.get_state()
    assert torch.equal(got, want)
    params = torch.zeros((n, 6), dtype=torch.float32)
    params[:, 0], params[:, 1], params[:, 2], params[:, 3] = 8.0, 4.0, 3.5, 4.0
    env.reset_params(params, max_t=torch.full((n,), 65535, dtype=torch.int32))
    with pytest.raises(HockeyNativeError):
        env.reset_params(params, max_t=torch.full((n,), 65536, dtype=torch.int32))
    with pytest.raises(HockeyNativeError):
        env.reset_params(params, max_t=torch.full((n,), -1, dtype=torch.int32))
    env.close()
