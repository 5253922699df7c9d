"""Where the reference's one recorded stage-1 curve sits among our seeded runs.

Reads the per-seed learning curves of scripts/td3_stage1_pin.py -- 20 arenas (profiles/r03/stage1_pin_n20_s*.json),
4 arenas (profiles/r03/stage1_pin_n4_s*.json) and ONE arena, the reference's own round structure of one episode
then 32 updates (profiles/r04/stage1_pin_n1_s*.json, scripts/gpu_r04b.sh, 18 minutes per seed, so 2 600-5 400
episodes) -- and, at every 1 000 episodes, compares the mean WR_weak of the last three evaluations (ep-400 .. ep)
per seed with the same window of the reference's recorded curve (pretrained/stage_1 metrics, carried in every curve
file as ``reference_wr_weak``).  Writes profiles/r04/stage1_seed_study.json.
Usage: python scripts/stage1_seed_study.py"""
import glob
import json
import os
import statistics as st

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
STUDIES = ((20, "profiles/r03/stage1_pin_n20_s*.json"), (4, "profiles/r03/stage1_pin_n4_s*.json"),
           (1, "profiles/r04/stage1_pin_n1_s*.json"))


def window(curve, ep):
    return st.mean(curve[e] for e in range(ep - 400, ep + 1, 200))


def main():
    ref = None
    out = {"what": __doc__.split("\n\n")[0], "window": "mean WR_weak of the evaluations at ep-400, ep-200, ep",
           "studies": {}}
    for n, pat in STUDIES:
        curves = {}
        for f in sorted(glob.glob(os.path.join(ROOT, pat))):
            if "summary" in f:
                continue
            d = json.load(open(f))
            ref = ref or {200 * (i + 1): v for i, v in enumerate(d["reference_wr_weak"])}
            curves[d["seed"]] = {e["episode"]: e["wr_weak"] for e in d["evals"]}
        rows = []
        for ep in range(1000, 10001, 1000):
            vals = {s: window(c, ep) for s, c in curves.items() if ep in c}
            if not vals:
                continue
            r = window(ref, ep)
            v = list(vals.values())
            rows.append({"episode": ep, "reference": round(r, 4), "seeds": len(v), "mean": round(st.mean(v), 4),
                         "min": round(min(v), 4), "max": round(max(v), 4),
                         "seeds_below_reference": sum(x < r for x in v)})
        out["studies"][f"{n}_arenas"] = {"episodes_reached": {s: max(c) for s, c in curves.items()}, "rows": rows}
        print(f"{n} arena(s)")
        for row in rows:
            print(f"  {row['episode']:5d}: reference {row['reference']:.2f}  seeds {row['mean']:.2f} "
                  f"[{row['min']:.2f}, {row['max']:.2f}]  {row['seeds_below_reference']}/{row['seeds']} below")
    with open(os.path.join(ROOT, "profiles", "r04", "stage1_seed_study.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
