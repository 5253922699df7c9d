"""Power of the behavioural pins on world.Step (SURVEY §8 rows a7 / c).

The checkpoint pin (tests/test_gpu_checkpoints.py) holds the simulator to the 20 win rates the reference recorded for
its 12 shipped actors.  Green there only means something if wrong physics turns it red.  This study runs the SAME
protocol and the SAME acceptance rule (hockey_amd.evaluate.checkpoint_pins / recorded_rate_z / pin_acceptance) on the
CPU oracle (oracle/hk_oracle.c, which the kernel equals bit for bit) for the pinned restatement and for variants:

  base          the restatement the kernel is pinned to
  reverse, no_block, no_sleep, live_q1
                restatement choices Box2D's real behaviour may differ in (contact order, block solver, sleeping,
                SURVEY App. B Q1 velocity getters)
  iters_8_3     world.Step(dt, 8, 3) instead of (dt, 180, 60)
  rest_thresh0  WRONG: b2_velocityThreshold 0 instead of 1 m/s
  arith_fric    WRONG: b2MixFriction arithmetic instead of geometric mean
  no_toi        WRONG: b2World::SolveTOI skipped
  rest_min      WRONG: b2MixRestitution min instead of max

Protocol per recorded rate (rl/utils/evaluator.py:10-35 and hockey_amd.evaluate.checkpoint_pins): the actor plays
R replicas of the reference's 100 evaluation placements (reset seeds run_seed + i) against the fused BasicOpponent
(oracle policy "weak" / "strong"), opponent phases uniform on [0, 2 pi), greedy actions from the actor evaluated
with torch on the CPU, up to 251 steps; per-placement win frequencies give recorded_rate_z.  Common random numbers:
every variant uses the same placements, phases and Philox phase-increment streams.

Usage: python scripts/pin_power_study.py [--replicas 64] [--variants base,no_toi,...] --out profiles/r05/pin_power.json
Test infrastructure only (CPU, no GPU).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle")]

import torch  # noqa: E402

import oracle as O  # noqa: E402
from hockey_amd.evaluate import Actor, pin_acceptance, recorded_rate_z, reset_params  # noqa: E402

FIXTURE = os.path.join(ROOT, "tests", "golden", "checkpoint_actors.npz")
VARIANTS = {"base": (0, False), "reverse": (O.VAR_REVERSE, False), "no_block": (O.VAR_NO_BLOCK, False),
            "no_sleep": (O.VAR_NO_SLEEP, False), "live_q1": (0, True), "iters_8_3": (O.VAR_ITERS_8_3, False),
            "rest_thresh0": (O.VAR_REST_THRESH0, False), "arith_fric": (O.VAR_ARITH_FRIC, False),
            "no_toi": (O.VAR_NO_TOI, False), "rest_min": (O.VAR_REST_MIN, False)}
WRONG = ("rest_thresh0", "arith_fric", "no_toi", "rest_min")


def load_actors(path=FIXTURE):
    z = np.load(path)
    meta = json.loads(str(z["meta"]))
    actors = []
    for k in range(len(meta["checkpoints"])):
        a = Actor()
        with torch.no_grad():
            for name, p in a.named_parameters():
                p.copy_(torch.from_numpy(z[f"{k}/{name.replace('.', '_')}"]))
        actors.append(a.eval())
    return meta, actors


@torch.no_grad()
def oracle_eval(actor, episodes, seed, weak, replicas, phase_seed, vel_ref=False):
    """hockey_amd.evaluate.evaluate(..., replicas, per_episode=True) on the oracle: winner [R, E] (+1 / 0 / -1) and
    the mean game length."""
    n = episodes * replicas
    ov = O.OracleVec(n, policies=("external", "weak" if weak else "strong"), auto_reset=False, seed=seed,
                     vel_ref=vel_ref)
    params, max_t, _ = reset_params(episodes, seed)
    ov.reset(params=np.tile(params, (replicas, 1)), max_t=np.full(n, max_t, np.int32))
    ov.phase(np.random.default_rng(phase_seed).uniform(0, 2 * np.pi, (n, 2)))
    obs, _ = ov.observe()
    live = np.ones(n, bool)
    winner = np.zeros(n, np.float32)
    length = np.zeros(n, np.int64)
    act = np.zeros((n, 8), np.float32)
    for _ in range(max_t + 1):
        act[:, :4] = actor(torch.from_numpy(obs)).numpy()
        out = ov.step(act)
        length += live
        d = out["done"].astype(bool)
        winner = np.where(live & d, out["info"][:, 0], winner)
        live &= ~d
        obs = out["obs"]
        if not live.any():
            break
    ov.close()
    return winner.reshape(replicas, episodes).astype(np.int8), float(length.mean())


def pins(meta, actors, replicas, vel_ref=False):
    """hockey_amd.evaluate.checkpoint_pins on the oracle (same phase seeds, same row fields)."""
    rows = []
    for k, ck in enumerate(meta["checkpoints"]):
        for opp, rec in (("strong", ck["wr_strong"]), ("weak", ck["wr_weak"])):
            if rec is None:
                continue
            w, mean_len = oracle_eval(actors[k], ck["eval_episodes"], ck["eval_seed"], opp == "weak", replicas,
                                      1000 + 2 * k + (opp == "weak"), vel_ref)
            row = recorded_rate_z(w, rec)
            score = ck["score"]
            row.update(checkpoint=ck["name"], kind=ck["kind"], opponent=opp, eval_index=ck["eval_index"],
                       n_evals=ck["n_evals"], selected=ck["kind"] == "best" and (score in ("min", "winrates")
                                                                                 or score == opp),
                       mean_length=mean_len)
            rows.append(row)
    return rows


def detectable_shift(rows):
    """The smallest uniform shift delta (win-rate points, simulator minus recorded) of every free rate that takes the
    free chi^2 of ``rows`` to the acceptance rule's 0.1 % critical value: the resolution of the pin as a whole."""
    from scipy import stats

    free = [r for r in rows if not r["selected"]]
    crit = stats.chi2.ppf(0.999, len(free))
    out = {}
    for sign in (1, -1):
        lo, hi = 0.0, 1.0
        for _ in range(60):
            mid = 0.5 * (lo + hi)
            chi2 = sum(((r["recorded"] - (r["estimate"] + sign * mid)) / r["se"]) ** 2 for r in free)
            lo, hi = (lo, mid) if chi2 >= crit else (mid, hi)
        out["up" if sign > 0 else "down"] = round(100 * hi, 2)
    return out


def summarize(out):
    """Per variant: pass / fail, free chi^2, the stage-1 best strong z, and the paired shift of the 20 simulated
    rates against base (common random numbers: same placements, phases and Philox streams), in win-rate points."""
    base = out["variants"].get("base")
    table = {}
    for name, v in out["variants"].items():
        t = {"wrong_physics": v["wrong_physics"], "passed": v["acceptance"]["passed"],
             "free_chi2": round(v["acceptance"]["free_chi2"], 2), "stage1_best_strong_z": round(v["stage1_best_strong_z"], 2),
             "max_abs_z": round(max(abs(r["z"]) for r in v["rows"]), 2)}
        if base:
            d = np.array([100 * (r["estimate"] - b["estimate"]) for r, b in zip(v["rows"], base["rows"])])
            t.update(shift_mean_pts=round(float(d.mean()), 2), shift_rms_pts=round(float(np.sqrt((d ** 2).mean())), 2),
                     shift_max_abs_pts=round(float(np.abs(d).max()), 2))
        table[name] = t
    if base:
        table["_pin_resolution_pts"] = detectable_shift(base["rows"])
    return table


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--replicas", type=int, default=64)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--threads", type=int, default=0)
    ap.add_argument("--out", default=None)
    ap.add_argument("--summarize", action="store_true", help="only recompute the summary of an existing --out")
    args = ap.parse_args()
    if args.summarize:
        with open(args.out) as f:
            out = json.load(f)
        out["summary"] = summarize(out)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
        for name, t in out["summary"].items():
            print(name, t)
        return
    if args.threads:
        torch.set_num_threads(args.threads)
    meta, actors = load_actors()
    out = {"replicas": args.replicas, "protocol": __doc__.split("Protocol")[1].split("Usage")[0].strip(),
           "variants": {}}
    if args.out and os.path.exists(args.out):
        with open(args.out) as f:
            prev = json.load(f)
        if prev.get("replicas") == args.replicas:
            out["variants"] = prev.get("variants", {})
    for name in args.variants.split(","):
        flags, vel_ref = VARIANTS[name]
        O.set_variant(flags)
        t0 = time.time()
        rows = pins(meta, actors, args.replicas, vel_ref)
        O.set_variant(0)
        acc = pin_acceptance(rows)
        stage1 = next(r for r in rows if r["checkpoint"].startswith("pretrained/stage_1:best") and
                      r["opponent"] == "strong")
        out["variants"][name] = {"wrong_physics": name in WRONG, "acceptance": acc,
                                 "stage1_best_strong_z": stage1["z"], "seconds": round(time.time() - t0, 1),
                                 "rows": [{k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()}
                                          for r in rows]}
        print(f"{name:13s} passed={acc['passed']!s:5s} free chi2 {acc['free_chi2']:7.1f} (p {acc['free_chi2_p']:.2g}) "
              f"stage1 strong z {stage1['z']:+.2f} violations {acc['violations_free'] + acc['violations_selected']} "
              f"{time.time() - t0:.0f}s", file=sys.stderr, flush=True)
        if args.out:
            with open(args.out, "w") as f:
                json.dump(out, f, indent=1)
    out["summary"] = summarize(out)
    if args.out:
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    else:
        print(json.dumps(out, indent=1))
    for name, t in out["summary"].items():
        print(name, t, file=sys.stderr)


if __name__ == "__main__":
    main()
