"""GPU TD3 loop vs the reference's own loop on the same restated physics, per protocol.

Inputs: runs of scripts/noise_study.py (the GPU loop, hockey_amd.td3.train) and of scripts/reference_loop_study.py
(the reference's rl/ code on the C oracle, CPU), both with a ``final_eval`` block (the best checkpoint re-evaluated
on 1 000 fresh placements per bot).  For each (protocol, noise) present in both: mean +- std (ddof 1) of the final
win rates and returns of each loop, Welch's t between the loops with its two-sided p, the Mann-Whitney U p, and the
mean evaluation score min(WR_strong, WR_weak) of each loop at every 1 000 episodes (the learning curve).  Win rates
in percent.  Also the number of runs of each loop whose evaluations reach WR_weak >= 0.9, with Fisher's exact p.

Usage: python scripts/reference_loop_compare.py --gpu profiles/r05/noise_runs --ref profiles/r05/reference_loop_stage2 \
           > profiles/r05/reference_loop_stage2_comparison.json
"""
import argparse
import glob
import json
import os

import numpy as np
from scipy import stats

KEYS = (("wr_weak", 100.0), ("wr_strong", 100.0), ("r_weak", 1.0), ("r_strong", 1.0))


def key_of(r):
    proto = r.get("protocol", "scratch")
    if proto == "sp_per":
        return proto, f"per{int(r.get('per', False))}_sp{int(r.get('self_play', False))}"
    return proto, r["noise"]


def load(d, ref):
    runs = {}
    for f in sorted(glob.glob(os.path.join(d, "*.json"))):
        r = json.load(open(f))
        if "final_eval" not in r or "evals" not in r:
            continue
        if ref and r.get("protocol") == "sp_per":
            r["per"], r["self_play"] = False, False  # reference_loop_study runs the baseline row only
        runs.setdefault(key_of(r), []).append(r)
    return runs


def curve(rs, every=1000):
    out = {}
    for r in rs:
        for e in r["evals"]:
            if e["episode"] % every == 0:
                out.setdefault(e["episode"], []).append(e["score"])
    return {ep: round(float(np.mean(v)), 3) for ep, v in sorted(out.items())}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpu", required=True)
    ap.add_argument("--ref", required=True)
    args = ap.parse_args()
    gpu, ref = load(args.gpu, False), load(args.ref, True)
    out = {"source": "scripts/reference_loop_compare.py", "gpu_dir": args.gpu, "ref_dir": args.ref, "cells": {}}
    for k in sorted(set(gpu) & set(ref)):
        g, r = gpu[k], ref[k]
        cell = {"gpu_seeds": [x["seed"] for x in g], "ref_seeds": [x["seed"] for x in r]}
        for key, scale in KEYS:
            a = np.array([x["final_eval"][key] * scale for x in g])
            b = np.array([x["final_eval"][key] * scale for x in r])
            t = stats.ttest_ind(a, b, equal_var=False) if len(a) > 1 and len(b) > 1 else None
            cell[key] = {"gpu": [round(float(a.mean()), 2), round(float(a.std(ddof=1)), 2) if len(a) > 1 else 0.0],
                         "ref": [round(float(b.mean()), 2), round(float(b.std(ddof=1)), 2) if len(b) > 1 else 0.0],
                         "gpu_values": [round(float(v), 2) for v in a], "ref_values": [round(float(v), 2) for v in b],
                         "welch_t": None if t is None else round(float(t.statistic), 2),
                         "welch_p": None if t is None else round(float(t.pvalue), 3),
                         "mann_whitney_p": round(float(stats.mannwhitneyu(a, b).pvalue), 3)}
        cell["score_curve"] = {"gpu": curve(g), "ref": curve(r)}
        # runs whose evaluations reach WR_weak >= 0.9 at some point (the stage-1 "learned" mark), Fisher exact p
        hit = lambda rs: sum(any(e["wr_weak"] >= 0.9 for e in x["evals"]) for x in rs)  # noqa: E731
        hg, hr = hit(g), hit(r)
        cell["reach_wr_weak_0.9"] = {"gpu": [hg, len(g)], "ref": [hr, len(r)],
                                     "fisher_p": round(float(stats.fisher_exact([[hg, len(g) - hg],
                                                                                [hr, len(r) - hr]]).pvalue), 3)}
        cell["best_episode"] = {"gpu": [x["best"]["episode"] for x in g], "ref": [x["best"]["episode"] for x in r]}
        out["cells"]["/".join(k)] = cell
    print(json.dumps(out, indent=1))
    for name, c in out["cells"].items():
        print(name, " ".join(f"{k} gpu {c[k]['gpu'][0]}+-{c[k]['gpu'][1]} ref {c[k]['ref'][0]}+-{c[k]['ref'][1]} "
                             f"(p {c[k]['welch_p']})" for k, _ in KEYS), file=__import__("sys").stderr)


if __name__ == "__main__":
    main()
