"""The kernel's per-arena source (hk_step.h -> hk_arena.h / hk_solver.h / hk_geom.h), compiled for the host
CPU by tests/hostcheck.py, held bit-for-bit to the oracle -- on the CPU, without a GPU.

This catches logic errors in the device code before a GPU run; the GPU parity tests (test_gpu_parity.py)
then hold the gfx950 binary of the same source to the same oracle.  The harness is test infrastructure
(never loaded by the product package).
"""
import os

import numpy as np
import pytest

from hockey_amd.placement import np_random, placement

from hostcheck import HostVec, velocity_diag


def _f32(x):
    return np.asarray(x, np.float64).astype(np.float32)


def _lockstep(oracle, mode, n, steps, seed, **env_kw):
    keep = True
    env = HostVec(n, keep_mode=keep, mode=mode, **env_kw)
    params = np.zeros((n, 6), np.float32)
    for i in range(n):
        rng, _ = np_random(seed * 100_000 + i)
        params[i], max_t = placement(mode, bool(i % 2), rng)
    env.reset_params(params)
    ws = []
    for i in range(n):
        w = oracle.OracleWorld(keep, mode)
        w.reset(params[i], max_t)
        ws.append(w)
    rng = np.random.default_rng(seed)
    phases = rng.uniform(0, np.pi, (n, 2))
    obs = np.stack([w.obs() for w in ws]).astype(np.float64)
    obs2 = np.stack([w.obs_two() for w in ws]).astype(np.float64)
    n_toi = 0
    for t in range(steps):
        acts = rng.uniform(-1, 1, (n, 8)).astype(np.float32)
        for i in range(0, n, 2):  # half the arenas: strong-vs-strong BasicOpponent (contacts, shots, goals)
            a1, phases[i, 0] = oracle.basic_opponent(0, 1, phases[i, 0], 0.1, obs[i])
            a2, phases[i, 1] = oracle.basic_opponent(0, 1, phases[i, 1], 0.1, obs2[i])
            acts[i] = np.concatenate([a1, a2]).astype(np.float32)
        res = env.step(acts, with_agent_two=True)
        for i, w in enumerate(ws):
            o, r, d, info, _ = w.step(acts[i])
            n_toi += w.stats()[1]
            o2 = w.obs_two()
            i2, r2 = w.info_two()
            checks = (("obs", np.array_equal(res.obs[i], o)), ("obs2", np.array_equal(res.obs2[i], o2)),
                      ("reward", res.reward[i] == np.float32(r)), ("reward2", res.reward2[i] == np.float32(r2)),
                      ("done", bool(res.done[i]) == d), ("info", np.array_equal(res.info[i], _f32(info))))
            for name, ok in checks:
                if not ok:
                    return {"step": t, "arena": i, "field": name}
            obs[i], obs2[i] = o, o2
    st, _ = env.get_state()
    for i, w in enumerate(ws):
        assert np.array_equal(st[i], w.get_raw()[0]), i
    out = {"n_toi": n_toi, "counters": env.counters()}
    env.close()
    return out


@pytest.mark.parametrize("mode,seed", [(0, 1), (1, 3), (2, 4)])
def test_kernel_source_lockstep_vs_oracle(oracle, mode, seed):
    out = _lockstep(oracle, mode, n=48, steps=200, seed=seed)
    assert "field" not in out, out
    if mode == 0:
        assert out["n_toi"] > 0


def test_large_island_solver_vs_oracle(oracle):
    """diag_flags=HK_DIAG_LARGE_ISLANDS routes every island / TOI solve through the HBM slot file (HbmSlots,
    the path of islands with more contacts than the register slots) -- it must be bit-identical as well."""
    out = _lockstep(oracle, 1, n=32, steps=150, seed=3, diag_flags=1)
    assert "field" not in out, out
    assert out["counters"][6] > 0  # large-island solves were taken


def test_fused_opponents_autoreset_run(oracle):
    """Fused strong/weak BasicOpponent with device auto-reset: counters consistent, no overflow."""
    env = HostVec(256, policies=("strong", "weak"), auto_reset=True, seed=7)
    for _ in range(300):
        env.step(None)
    c = env.counters()
    assert c[0] == 256 * 300 and c[5] == 0
    assert c[1] > 0 and c[2] + c[3] <= c[1]


# ------------------------------------------------------------------------------------------------ batched contract
from vec_lockstep import first_mismatch  # noqa: E402


def _vec_lockstep(oracle, n, steps, mode, policies, seed, external=False, offset=0, mix=False, keep_mode=True,
                  vel_ref=False):
    """The kernel source (host build) vs the oracle's batched context on the hk_step contract: fused
    policies with Philox increments (opp_inc NULL), device auto-reset with episode counters.  mix: player 2's
    policy is drawn per arena and step from {external, weak, strong} (hk_step_io.policy2)."""
    env = HostVec(n, keep_mode=keep_mode, mode=mode, policies=policies, auto_reset=True, seed=seed,
                  arena_offset=offset, vel_ref=vel_ref)
    ov = oracle.OracleVec(n, keep_mode=keep_mode, mode=mode, policies=policies, auto_reset=True, seed=seed,
                          arena_offset=offset, vel_ref=vel_ref)
    rng = np.random.default_rng(seed)
    for t in range(steps):
        acts = rng.uniform(-1.2, 1.2, (n, 8)).astype(np.float32) if external else None
        p2 = rng.choice(np.array([0, 2, 3], np.uint8), n) if mix else None
        got = vars(env.step(acts, with_agent_two=True, record_actions=True, final_obs=True, policy2=p2))
        want = ov.step(acts, with_agent_two=True, final_obs=True, policy2=p2)
        bad = first_mismatch(t, got, want)
        if bad:
            return bad
    st, aux = env.get_state()
    ost, oaux = ov.get_state()
    assert np.array_equal(st, ost) and np.array_equal(aux, oaux)
    c, oc = env.counters().astype(np.int64), ov.counters()
    assert np.array_equal(c[:5], oc[:5]), (c[:7], oc[:7])  # steps, episodes, goals p1 / p2, TOI events
    return {"counters": c}


@pytest.mark.parametrize("mode,steps", [(0, 560), (1, 200), (2, 200)])
def test_bench_path_vs_oracle_vec(oracle, mode, steps):
    """The benchmarked workload (strong vs strong, in-kernel Philox phase increments, auto-reset with device
    placement): every arena rolls over at least twice in every mode."""
    out = _vec_lockstep(oracle, 64, steps, mode, ("strong", "strong"), seed=5 + mode)
    assert "field" not in out, out
    assert out["counters"][1] >= 2 * 64


def test_random_and_external_policies_vs_oracle_vec(oracle):
    out = _vec_lockstep(oracle, 48, 300, 0, ("random", "weak"), seed=21, offset=1000)
    assert "field" not in out, out
    out = _vec_lockstep(oracle, 48, 300, 2, ("external", "strong"), seed=22, external=True)
    assert "field" not in out, out


def test_per_step_opponent_mix_vs_oracle_vec(oracle):
    """Player 2's opponent drawn per arena and step (hk_step_io.policy2, rl/training/opponent_manager.py:62-91):
    external (self-play actions), weak bot and strong bot, each bot with its own phase."""
    out = _vec_lockstep(oracle, 48, 300, 0, ("external", "external"), seed=23, external=True, mix=True)
    assert "field" not in out, out
    out = _vec_lockstep(oracle, 32, 200, 1, ("strong", "weak"), seed=24, external=True, mix=True)
    assert "field" not in out, out


def test_island_retirement_and_slot_swaps_vs_oracle(oracle):
    """Islands of one lane retire one by one inside the shared velocity loop (hk_solver.h vgen / vtwo), and
    the live contacts are swapped into the one- and two-contact slots: both paths run in a bit-exact lockstep
    of the strong-vs-strong workload against the oracle (which solves island by island, like Box2D)."""
    velocity_diag()
    out = _vec_lockstep(oracle, 256, 400, 0, ("strong", "strong"), seed=31)
    assert "field" not in out, out
    d = velocity_diag()
    assert d[0] > 0 and d[1] > 0, d


@pytest.mark.parametrize("mode", [0, 1, 2])
def test_keep_mode_false_with_physics_vs_oracle_vec(oracle, mode):
    """Hockey-v0 with keep_mode=False (hockey_env.py:91): 6-dim joint action, player 2's action at index 3
    (:663), no hold / shoot (:668-680) -- with world.Step running, external random actions and the fused
    BasicOpponent(keep_mode=False) in every mode."""
    out = _vec_lockstep(oracle, 48, 260, mode, ("external", "strong"), seed=41 + mode, external=True,
                        keep_mode=False)
    assert "field" not in out, out
    out = _vec_lockstep(oracle, 48, 200, mode, ("weak", "strong"), seed=44 + mode, keep_mode=False)
    assert "field" not in out, out


def test_live_velocity_semantics_with_physics_vs_oracle_vec(oracle):
    """SURVEY App. B Q1 live-reference velocity getters (vel_ref_semantics=1, hockey_env.py:425-432) with
    world.Step running: random external actions (boundary hits) and the strong-vs-strong workload."""
    out = _vec_lockstep(oracle, 48, 300, 0, ("external", "external"), seed=47, external=True, vel_ref=True)
    assert "field" not in out, out
    out = _vec_lockstep(oracle, 48, 300, 1, ("strong", "strong"), seed=48, vel_ref=True)
    assert "field" not in out, out


def test_step_record_matches_outputs_and_state(oracle):
    """hk_step_io.record (the single-env facade's one-copy step result): float64 info / info2 / rewards whose
    float32 roundings are the step's float outputs (oracle-checked), and has_puck / time / done / winner equal
    to the state after the step -- over a strong-vs-strong run with goals and holds."""
    n = 64
    env = HostVec(n, policies=("strong", "strong"), auto_reset=False, seed=9)
    ov = oracle.OracleVec(n, policies=("strong", "strong"), auto_reset=False, seed=9)
    held = 0
    for t in range(300):
        got = env.step(None, with_agent_two=True, record=True)
        want = ov.step(with_agent_two=True)
        rec = got.record
        assert first_mismatch(t, {"info": rec[:, 0:4].astype(np.float32), "info2": rec[:, 4:8].astype(np.float32),
                                  "reward": rec[:, 8].astype(np.float32), "reward2": rec[:, 9].astype(np.float32)},
                              want, fields=("info", "info2", "reward", "reward2")) is None
        _, aux = env.get_state()
        assert np.array_equal(rec[:, 10:15].astype(np.int32), aux), t
        assert np.array_equal(rec[:, 13].astype(np.uint8), got.done) and np.all(rec[:, 15] == 0)
        held += int((aux[:, 0] > 0).sum())
    assert aux[:, 3].sum() > 0 and held > 0  # goals and holds happened



def test_shape_families_vs_oracle(oracle):
    """The tail's shape-specialised velocity loops (r06, hk_solver.h): the S2 two-contact chunk (contact 1's body B
    aliased to contact 0's body A, contact 1 static-A) and the S3 three-contact family (wall-puck, player-puck,
    wall-player with the two dynamic bodies in locals) both run in a bit-exact lockstep of the strong-vs-strong
    bench workload against the oracle.  (The host build runs one lane at a time, so the one-contact riders of those
    loops run on the GPU only: tests/test_gpu_parity.py.)"""
    velocity_diag()
    out = _vec_lockstep(oracle, 1024, 400, 0, ("strong", "strong"), seed=41)
    assert "field" not in out, out
    d = velocity_diag()
    assert d[2] > 0 and d[3] > 0, d
