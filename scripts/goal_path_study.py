"""Does how goals are scored explain the one-sided parity residual? (SURVEY §8 rows a7 / a8 / c.)

Several independent residuals say the restated rink is slightly more decisive than the reference's Box2D one: the
notebook's 1 000 strong-vs-strong games have fewer draws and shorter games than the oracle predicts (draw z ~ -2,
steps/game z ~ -1.2), and trained policies score 2-8 points above the report against the bots.  The r03 / r05
variant studies never varied the goal path itself.  This study does, on the CPU oracle (which the kernel equals bit
for bit), with switches of hk_oracle.c hko_set_variant:

  base          the restatement the kernel is pinned to
  skin_plus     the goal sensor fires one polygon skin (b2_polygonRadius = 1 cm) early: core distance < 10 eps + skin
                (hockey_env.py:321-343; Box2D's b2TestOverlap is distance-with-radii < 10 eps)
  skin_minus    the sensor polygon's skin is dropped: core distance < puck radius + 10 eps, a skin deeper
  swept         the sensor overlap is tested along the puck's last sweep (17 positions) instead of at its end
                position: what Box2D does NOT do (no TOI for sensors), so a fast shot that crosses
                the goal mouth between two steps scores here and tunnels there
  core_overlap  an extreme control, not a candidate: radii ignored, the goal counts only once the puck's centre is
                inside the goal polygon (a puck radius deeper); shows the direction and size of a threshold change
  keep_com      _keep_puck (hockey_env.py:618-620) puts the held puck at the player's centre of mass instead of its
                body origin, so Box2D's push-out of the overlapping puck starts elsewhere

Per variant: (1) the notebook protocol (Hockey-Env.ipynb:940-2154, scripts/box2d_variant_study.oracle_study:
``games`` strong-vs-strong games, common random numbers across variants) with z-scores against the notebook's
recorded outcome split, steps per game, rewards and obs means; (2) the checkpoint pin (scripts/pin_power_study:
the reference's 12 shipped actors x 100 placements x R replicas against the fused bots, the acceptance rule of
tests/test_gpu_checkpoints.py), with the paired shift of the 20 simulated rates against base.  The question is
which variant, if any, moves draw z by >= 1 and the free rates by >= 1 point.  Nothing is tuned: the pinned
restatement stays the base.

Usage: python scripts/goal_path_study.py [--games 100000] [--replicas 64] --out profiles/r06/goal_path_study.json
Test infrastructure only (CPU, no GPU).
"""
import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [os.path.join(ROOT, "scripts"), os.path.join(ROOT, "hockey-env_amd"), os.path.join(ROOT, "oracle")]

import oracle as O  # noqa: E402
from box2d_variant_study import oracle_study  # noqa: E402
from hockey_amd.evaluate import pin_acceptance, reset_params, study_zscores  # noqa: E402
from pin_power_study import load_actors, pins  # noqa: E402

VARIANTS = {"base": 0, "skin_plus": O.VAR_SENSOR_SKIN_PLUS, "skin_minus": O.VAR_SENSOR_SKIN_MINUS,
            "swept": O.VAR_SENSOR_SWEPT, "keep_com": O.VAR_KEEP_COM, "core_overlap": O.VAR_SENSOR_CORE}
KEYS = ("win", "draw", "loss", "steps_per_game", "reward_per_game")


def run_variant(name, flags, games, seed, replicas, meta, actors):
    O.set_variant(flags)
    try:
        t0 = time.time()
        params, max_t, _ = reset_params(games, seed)
        zs = study_zscores(oracle_study(games, seed, params, max_t, False))
        zs["obs_mean_chi2_18"] = float(sum(o["z"] ** 2 for o in zs["obs_mean"]))
        t1 = time.time()
        rows = pins(meta, actors, replicas) if replicas > 0 else []
        acc = pin_acceptance(rows) if rows else None
    finally:
        O.set_variant(0)
    out = {"flags": flags, "notebook": zs, "notebook_seconds": round(t1 - t0, 1),
           "pin_seconds": round(time.time() - t1, 1)}
    if rows:
        stage1 = next(r for r in rows if r["checkpoint"].startswith("pretrained/stage_1:best")
                      and r["opponent"] == "strong")
        out.update(acceptance=acc, stage1_best_strong_z=stage1["z"],
                   rows=[{k: (round(v, 5) if isinstance(v, float) else v) for k, v in r.items()} for r in rows])
    return out


def summarize(out):
    base = out["variants"]["base"]
    table = {}
    for name, v in out["variants"].items():
        nb = v["notebook"]
        t = {k: round(nb[k]["z"], 2) for k in KEYS}
        t["obs_chi2_18"] = round(nb["obs_mean_chi2_18"], 1)
        if name != "base":
            t["delta_z"] = {k: round(nb[k]["z"] - base["notebook"][k]["z"], 3) for k in KEYS}
        if "rows" in v:
            t["pin_passed"] = v["acceptance"]["passed"]
            t["pin_free_chi2"] = round(v["acceptance"]["free_chi2"], 2)
            t["stage1_best_strong_z"] = round(v["stage1_best_strong_z"], 2)
            if name != "base" and "rows" in base:
                free = [(r, b) for r, b in zip(v["rows"], base["rows"]) if not b["selected"]]
                d_all = np.array([100 * (r["estimate"] - b["estimate"]) for r, b in zip(v["rows"], base["rows"])])
                d_free = np.array([100 * (r["estimate"] - b["estimate"]) for r, b in free])
                t["rate_shift_pts"] = {"all_mean": round(float(d_all.mean()), 2),
                                       "free_mean": round(float(d_free.mean()), 2),
                                       "free_rms": round(float(np.sqrt((d_free ** 2).mean())), 2)}
                t["moves_draw_z_by_1"] = abs(t["delta_z"]["draw"]) >= 1.0
                t["moves_free_rates_by_1pt"] = abs(t["rate_shift_pts"]["free_mean"]) >= 1.0
        table[name] = t
    return table


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--games", type=int, default=100_000)
    ap.add_argument("--seed", type=int, default=0)
    ap.add_argument("--replicas", type=int, default=64)
    ap.add_argument("--variants", default=",".join(VARIANTS))
    ap.add_argument("--out", required=True)
    args = ap.parse_args()
    meta, actors = load_actors()
    out = {"games": args.games, "seed": args.seed, "replicas": args.replicas,
           "protocol": __doc__.split("Per variant:")[1].split("Usage")[0].strip(), "variants": {}}
    if os.path.exists(args.out):
        with open(args.out) as f:
            prev = json.load(f)
        if (prev.get("games"), prev.get("replicas")) == (args.games, args.replicas):
            out["variants"] = prev.get("variants", {})
    for name in args.variants.split(","):
        v = run_variant(name, VARIANTS[name], args.games, args.seed, args.replicas, meta, actors)
        out["variants"][name] = v
        nb = v["notebook"]
        print(f"{name:10s} " + " ".join(f"{k} z {nb[k]['z']:+.2f}" for k in KEYS)
              + (f" | pin {v['acceptance']['passed']} chi2 {v['acceptance']['free_chi2']:.1f}" if "rows" in v else "")
              + f" | {v['notebook_seconds']:.0f}+{v['pin_seconds']:.0f} s", file=sys.stderr, flush=True)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
    if "base" in out["variants"]:
        out["summary"] = summarize(out)
        with open(args.out, "w") as f:
            json.dump(out, f, indent=1)
        for name, t in out["summary"].items():
            print(name, t, file=sys.stderr)


if __name__ == "__main__":
    main()
