"""§8 row f3: the C5 loop's opponent machinery (hockey_amd/opponents.py) against the reference's
rl/training/opponent_manager.py:62-91, self_play.py:20-68 and curricula.py.  CPU tests pin the schedule,
the per-step draw probabilities, the pool and its difficulty scores; the GPU test runs the mixed loop on
65 536 arenas (tests/test_td3.py) and the per-arena policy override is pinned bit-exactly against the oracle
(test_gpu_parity.py / test_hostcheck_parity.py)."""
import math

import numpy as np
import pytest
import torch

from hockey_amd import _native as N
from hockey_amd.evaluate import Actor
from hockey_amd.opponents import CURRICULA, OpponentMix, SelfPlayPool


def test_curriculum_rows_follow_progress():
    mix = OpponentMix(8, "stage3", device="cpu")
    # first row whose threshold exceeds the progress (opponent_manager._update_single)
    for progress, want in ((0.0, (0.30, 0.70, 0.00)), (0.149, (0.30, 0.70, 0.00)), (0.15, (0.60, 0.30, 0.10)),
                           (0.69, (0.60, 0.30, 0.10)), (0.7, (0.35, 0.35, 0.30)), (0.999, (0.35, 0.35, 0.30))):
        mix.update_schedule(progress)
        assert (mix.p_strong, mix.p_weak, mix.p_self) == want
    assert CURRICULA["ablation"] == CURRICULA["stage2"]


def test_self_play_pool_snapshots_scores_and_cap():
    actor = Actor()
    pool = SelfPlayPool(interval=3, pool_size=2, seed=0)
    assert pool.sample() is None
    for _ in range(2):
        pool.step(actor)
    assert len(pool) == 0
    pool.step(actor)  # episode 3: snapshot
    assert len(pool) == 1 and pool.scores == [1.0]
    assert all(not p.requires_grad for p in pool.pool[0].parameters())
    with torch.no_grad():
        actor.fc3.bias.add_(1.0)
    x = torch.randn(3, 18)
    assert not torch.equal(pool.pool[0](x), actor(x))  # a frozen copy, not a reference
    pool.step(actor, episodes=7)  # crosses two boundaries: one snapshot (same weights)
    pool.step(actor, episodes=3)
    assert len(pool) == 2  # capped, oldest dropped
    # difficulty: x1.2 per non-win, x0.95 per win, clipped to [0.1, 10]
    pool.update_difficulty(0, wins=0, others=2)
    assert math.isclose(pool.scores[0], 1.44)
    pool.update_difficulty(0, wins=1, others=0)
    assert math.isclose(pool.scores[0], 1.44 * 0.95)
    pool.update_difficulty(1, wins=0, others=100)
    assert pool.scores[1] == 10.0
    pool.update_difficulty(1, wins=10_000, others=0)
    assert pool.scores[1] == 0.1
    # sampling follows the scores
    pool.scores = [9.0, 1.0]
    draws = np.array([pool.sample() for _ in range(4000)])
    assert abs((draws == 0).mean() - 0.9) < 0.03


def test_per_step_draw_probabilities():
    n = 200_000
    mix = OpponentMix(n, [(1.0, 0.35, 0.35, 0.30)], device="cpu", seed=1)
    obs2 = torch.zeros(n, 18)
    p2, act, idx = mix.select(obs2)  # empty pool: no self-play, strong below P(strong), weak otherwise
    assert idx is None and act is None
    assert abs((p2 == N.POLICY_BASIC_STRONG).float().mean() - 0.35) < 0.01
    assert set(p2.unique().tolist()) == {N.POLICY_BASIC_STRONG, N.POLICY_BASIC_WEAK}
    mix.pool.add_snapshot(Actor())
    p2, act, idx = mix.select(torch.randn(n, 18))
    sp = p2 == N.POLICY_EXTERNAL
    assert idx == 0 and abs(sp.float().mean() - 0.30) < 0.01
    assert abs((p2 == N.POLICY_BASIC_STRONG).float().mean() - 0.70 * 0.35) < 0.01
    assert act.shape == (n, 4) and torch.all(act[~sp] == 0) and torch.any(act[sp] != 0)
    # outcomes of self-play arenas' done steps fold into the snapshot's score once per round
    done = torch.zeros(n, dtype=torch.uint8)
    reward = torch.zeros(n)
    first = torch.nonzero(sp)[:3, 0]
    done[first] = 1
    reward[first[0]] = 10.0
    mix.register_outcomes(done, reward)
    counts = mix.end_round()
    assert math.isclose(mix.pool.scores[0], 0.95 * 1.2 * 1.2)
    assert counts["self_play"] == int(sp.sum()) and sum(counts.values()) == 2 * n


def _ref_update_difficulty(score, win):
    """rl/training/self_play.py:45-55, one outcome at a time (restated)."""
    score = score * 1.2 if win == 0 else score * 0.95
    return float(np.clip(score, 0.1, 10.0))


def test_difficulty_clips_after_every_outcome_like_the_reference():
    """Saturation: 20 non-wins then 30 wins -> 10 * 0.95^30 = 2.146 in the reference (clipped at 10 on the way
    up), not 1.2^20 * 0.95^30 = 8.2; the per-step tallies reproduce any outcome sequence whose steps hold
    their non-wins before their wins."""
    pool = SelfPlayPool(interval=1, pool_size=1, seed=0)
    pool.add_snapshot(Actor())
    pool.update_difficulty(0, wins=0, others=20)
    pool.update_difficulty(0, wins=30, others=0)
    assert math.isclose(pool.scores[0], 10 * 0.95 ** 30)
    rng = np.random.default_rng(3)
    for _ in range(20):
        pool.scores = [float(rng.uniform(0.1, 10))]
        ref = pool.scores[0]
        for _ in range(40):  # steps
            w, o = (int(x) for x in rng.integers(0, 25, 2))
            for win in [0] * o + [1] * w:
                ref = _ref_update_difficulty(ref, win)
            pool.update_difficulty(0, wins=w, others=o)
            assert math.isclose(pool.scores[0], ref, rel_tol=1e-9), (pool.scores[0], ref)


def test_round_outcomes_fold_step_by_step():
    n = 64
    mix = OpponentMix(n, [(1.0, 0.0, 0.0, 1.0)], device="cpu", seed=2)
    mix.pool.add_snapshot(Actor())
    ref = 1.0
    for t in range(30):
        mix.select(torch.zeros(n, 18))
        done = torch.zeros(n, dtype=torch.uint8)
        reward = torch.zeros(n)
        k = 8 if t < 10 else 3  # many non-wins early (saturate at 10), wins later
        done[:k] = 1
        if t >= 10:
            reward[:2] = 10.0
        mix.register_outcomes(done, reward)
        wins = int(((done != 0) & (reward > 0)).sum())
        for win in [0] * (k - wins) + [1] * wins:
            ref = _ref_update_difficulty(ref, win)
    mix.end_round()
    assert math.isclose(mix.pool.scores[0], ref, rel_tol=1e-9)
