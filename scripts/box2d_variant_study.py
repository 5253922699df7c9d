"""Which Box2D-restatement choices move the statistical residual? (SURVEY §8 rows a7 / c)

The oracle's Box2D 2.3 restatement can only be pinned statistically, against Hockey-Env.ipynb:940-2154 (1000
strong-vs-strong BasicOpponent games).  The pinned restatement sits at draw z ~ -2.1 and steps/game z ~ -1.6.
This study re-runs the notebook protocol on the CPU oracle (oracle/hk_oracle.c, batched context, OpenMP) under
variants of the choices the restatement had to make, and reports z-scores per variant:

  base          the restatement the kernel is pinned to (canonical pair order, block solver, sleep on, copy Q1)
  reverse       every contact-order-dependent loop walks the pair table backwards (Box2D's real order follows
                contact creation: b2ContactManager::AddPair prepends to the world and body edge lists)
  no_block      2-point manifolds solve point by point (g_blockSolve = false)
  no_sleep      islands never sleep
  live_q1       SURVEY App. B Q1 live-reference velocity getters in _check_boundaries
  iters_8_3     world.Step(dt, 8, 3) instead of (dt, 180, 60): a positive control (a solver change the study
                must resolve)

Protocol (hockey_amd.evaluate.basic_vs_basic_study, restated on the oracle): ``games`` arenas, one game each,
placement of game i as reset(seed=seed + i) on a reused env (puck side alternating), both BasicOpponent phases
uniform in [0, 2 pi) (long-lived opponents), Philox phase increments, up to 251 steps with the game ending at
done.  Test infrastructure only (CPU, no GPU).

Usage: python scripts/box2d_variant_study.py [games] [seed] > profiles/r03/box2d_variant_study.json
"""
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from hockey_amd.evaluate import reset_params, study_zscores  # noqa: E402

VARIANTS = {"base": (0, False), "reverse": (O.VAR_REVERSE, False), "no_block": (O.VAR_NO_BLOCK, False),
            "no_sleep": (O.VAR_NO_SLEEP, False), "live_q1": (0, True), "iters_8_3": (O.VAR_ITERS_8_3, False)}


def oracle_study(games, seed, params, max_t, vel_ref):
    ov = O.OracleVec(games, policies=("strong", "strong"), auto_reset=False, seed=seed, vel_ref=vel_ref)
    ov.reset(params=params, max_t=np.full(games, max_t, np.int32))
    ov.phase(np.random.default_rng(seed).uniform(0, 2 * np.pi, (games, 2)))
    live = np.ones(games, bool)
    ret = np.zeros(games)
    ret2 = np.zeros(games)
    length = np.zeros(games, np.int64)
    winner = np.zeros(games, np.float32)
    obs_sum = np.zeros((games, 18))
    for _ in range(max_t + 1):
        out = ov.step(with_agent_two=True)
        lv = live.astype(np.float64)
        ret += lv * out["reward"]
        ret2 += lv * out["reward2"]
        obs_sum += lv[:, None] * out["obs"]
        length += live
        d = out["done"].astype(bool)
        winner = np.where(live & d, out["info"][:, 0], winner)
        live &= ~d
        if not live.any():
            break
    ov.close()
    return {"winner": winner, "length": length, "return": ret, "return2": ret2, "obs_sum": obs_sum}


def main():
    games = int(sys.argv[1]) if len(sys.argv) > 1 else 20000
    seed = int(sys.argv[2]) if len(sys.argv) > 2 else 0
    params, max_t, _ = reset_params(games, seed)
    out = {"games": games, "seed": seed, "protocol": __doc__.split("Protocol")[1].split("Usage")[0].strip(),
           "variants": {}}
    for name, (flags, vel_ref) in VARIANTS.items():
        O.set_variant(flags)
        t0 = time.time()
        zs = study_zscores(oracle_study(games, seed, params, max_t, vel_ref))
        O.set_variant(0)
        obs_z = [o["z"] for o in zs["obs_mean"]]
        zs["obs_mean_chi2_18"] = float(sum(x * x for x in obs_z))
        zs["seconds"] = time.time() - t0
        out["variants"][name] = zs
        print(name, {k: (round(v["value"], 4), round(v["z"], 2)) for k, v in zs.items() if isinstance(v, dict)},
              "chi2", round(zs["obs_mean_chi2_18"], 1), f"{zs['seconds']:.0f}s", file=sys.stderr, flush=True)
    base = out["variants"]["base"]
    # variant minus base, in units of the combined standard error the z-scores use
    out["shift_vs_base"] = {name: {k: round(v[k]["z"] - base[k]["z"], 3) for k in
                                   ("win", "draw", "loss", "steps_per_game", "reward_per_game")}
                            for name, v in out["variants"].items() if name != "base"}
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
