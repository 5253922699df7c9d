"""Behavioural pins for the Box2D-2.3 restatement (the part with no per-trajectory reference).

Box2D / box2d-py are third-party, unpinned and absent, so per-step trajectory parity
with real Box2D is "parity unpinned".  What the reference DOES record is Hockey-Env.ipynb's
"Check side consistency" study: 1000 strong-vs-strong BasicOpponent games (NORMAL mode, <=500 steps,
break on done) -> 150 911 steps (150.9 / game), winner counts {+1: 319, 0: 368, -1: 313}, and summed
agent-1 reward -4360.24 (Hockey-Env.ipynb:999, :2088-2154).  We replay that protocol with seeded resets
and a seeded phase stream and require agreement within sampling error.
"""
import numpy as np
import pytest

from hockey_amd.placement import np_random, placement


def _play(oracle, n_games, seed=0):
    """The notebook protocol: one env reused across games (alternating puck side), two long-lived strong
    BasicOpponents whose phases run on across games.  Per-game records for study_zscores."""
    w = oracle.OracleWorld(True, 0)
    one = True
    mirror = np.random.RandomState(seed)
    ph1, ph2 = mirror.uniform(0, np.pi), mirror.uniform(0, np.pi)
    rec = {"winner": [], "length": [], "return": [], "return2": [], "obs_sum": []}
    toi = 0
    for g in range(n_games):
        one = not one
        rng, _ = np_random(10_000 * seed + g)
        p, mt = placement(0, one, rng)
        w.reset(p, mt)
        obs, obs2 = w.obs().astype(np.float64), w.obs_two().astype(np.float64)
        ret = ret2 = 0.0
        osum = np.zeros(18)
        for t in range(500):
            a1, ph1 = oracle.basic_opponent(0, 1, ph1, mirror.uniform(0, 0.2), obs)
            a2, ph2 = oracle.basic_opponent(0, 1, ph2, mirror.uniform(0, 0.2), obs2)
            o, r, d, info, _ = w.step(np.concatenate([a1, a2]).astype(np.float32))
            toi += w.stats()[1]
            ret += r
            ret2 += w.info_two()[1]
            osum += o
            obs, obs2 = o.astype(np.float64), w.obs_two().astype(np.float64)
            assert np.all(np.isfinite(o))
            if d:
                break
        rec["winner"].append(int(info[0]))
        rec["length"].append(t + 1)
        rec["return"].append(ret)
        rec["return2"].append(ret2)
        rec["obs_sum"].append(osum)
    return {k: np.array(v) for k, v in rec.items()}, toi


def test_side_consistency_statistics(oracle):
    """1000 games each side: outcome split, steps per game and both agents' reward per game within 3 combined
    standard errors of the notebook's 1000 games; obs means jointly (chi-square, 18 dof, below its 0.1 % point)."""
    from hockey_amd.evaluate import study_zscores

    per_game, toi = _play(oracle, 1000)
    zs = study_zscores(per_game)
    for key in ("win", "draw", "loss", "steps_per_game", "reward_per_game", "reward2_per_game"):
        assert abs(zs[key]["z"]) < 3.0, (key, zs[key])
    assert sum(o["z"] ** 2 for o in zs["obs_mean"]) < 42.3, [round(o["z"], 2) for o in zs["obs_mean"]]
    assert abs(per_game["winner"].mean()) < 0.1  # symmetric game (reference 0.006)
    assert toi > 0  # continuous collision is exercised


def test_sticky_done_and_time_limit(oracle):
    """done is sticky and the +-10 repeats after a goal; the time limit is checked before time += 1
    (hockey_env.py:521-527, 685-693)."""
    w = oracle.OracleWorld(True, 0)
    w.reset(np.array([8, 4, 3, 4, 0, 0], np.float32), 250)
    zero = np.zeros(8, np.float32)
    for t in range(251):
        _, r, d, _, _ = w.step(zero)
        assert d == (t >= 250), t
    _, r, d, info, _ = w.step(zero)
    assert d and info[0] == 0


def test_goal_scored_and_sticky_reward(oracle):
    """A puck shot into the right goal fires BeginContact(goal_player_2) -> winner +1, reward +10 on every
    later step (no auto reset in reference semantics)."""
    w = oracle.OracleWorld(True, 0)
    w.reset(np.array([8, 4, 8.9, 4.0, 0, 0], np.float32), 250)
    st, aux = w.get_raw()
    st[15] = 20.0  # puck vx towards the right goal
    w.set_raw(st, aux)
    # move player 2 out of the way
    st[6:8] = [8.0, 6.5]
    w.set_raw(st, aux)
    zero = np.zeros(8, np.float32)
    winners = []
    for _ in range(30):
        _, r, d, info, _ = w.step(zero)
        winners.append((d, info[0], r))
    done_idx = [i for i, x in enumerate(winners) if x[0]]
    assert done_idx, winners
    k = done_idx[0]
    assert winners[k][1] == 1 and winners[k][2] >= 9.0
    assert all(x[0] and x[2] >= 9.0 for x in winners[k:])


def test_possession_hold_and_shot(oracle):
    """Puck touching player 1 with vx < 0.1 -> has_puck1 = 15, the puck is carried for 14 steps and shot
    at the 15th (hockey_env.py:63-67, 668-674)."""
    w = oracle.OracleWorld(True, 0)
    w.reset(np.array([8, 4, 2.35, 4.0, 0, 0], np.float32), 250)
    st, aux = w.get_raw()
    st[15] = -1.0
    w.set_raw(st, aux)
    zero = np.zeros(8, np.float32)
    has = []
    for _ in range(20):
        o, _, _, _, _ = w.step(zero)
        has.append(int(o[16]))
    assert 15 in has
    k = has.index(15)
    assert has[k:k + 14] == list(range(15, 1, -1))
    assert has[k + 14] == 0  # shot fired when the counter reached 1
    o, _, _, _, _ = w.step(zero)
    assert o[14] > 10.0  # the 60 m/s shot left the racket towards +x


@pytest.mark.parametrize("mode", [1, 2])
def test_training_modes_run(oracle, mode):
    w = oracle.OracleWorld(True, mode)
    rng, _ = np_random(7)
    p, mt = placement(mode, True, rng)
    w.reset(p, mt)
    assert mt == 80
    r = np.random.default_rng(0)
    for t in range(81):
        o, _, d, _, _ = w.step(r.uniform(-1, 1, 8).astype(np.float32))
        assert np.all(np.isfinite(o))
    assert d
