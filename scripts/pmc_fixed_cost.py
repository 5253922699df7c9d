"""Split hk::step_kernel's PMC traffic into a per-arena part and a fixed per-launch part (scripts/gpu_r04t.sh:
FETCH_SIZE / WRITE_SIZE at several arena counts of the same workload).  A least-squares line bytes = fixed +
per_arena * N per counter; FETCH_SIZE doubled (gfx950 correction, MI355X_MICROARCH.md).
Usage: python scripts/pmc_fixed_cost.py DIR [OUT.json]"""
import csv
import glob
import json
import os
import re
import sys


def per_launch(d, counter):
    vals = []
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if "step_kernel<false>" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]) * 1024.0)
    return (sum(vals) / len(vals), len(vals)) if vals else (None, 0)


def fit(xs, ys):
    n = len(xs)
    mx, my = sum(xs) / n, sum(ys) / n
    sxx = sum((x - mx) ** 2 for x in xs)
    slope = sum((x - mx) * (y - my) for x, y in zip(xs, ys)) / sxx
    return my - slope * mx, slope


def main():
    d = sys.argv[1]
    rows = {}
    for sub in sorted(glob.glob(os.path.join(d, "n*_*"))):
        m = re.match(r"n(\d+)_(FETCH_SIZE|WRITE_SIZE)$", os.path.basename(sub))
        if not m or not os.path.isdir(sub):
            continue
        n, c = int(m.group(1)), m.group(2)
        v, k = per_launch(sub, c)
        if v is None:
            continue
        rows.setdefault(n, {})[c] = {"bytes_per_launch": v * (2.0 if c == "FETCH_SIZE" else 1.0), "launches": k}
    out = {"what": "hk::step_kernel PMC bytes per launch vs arena count (FETCH_SIZE x2); fit bytes = fixed + "
                   "per_arena * N", "points": {str(n): r for n, r in sorted(rows.items())}, "fit": {}}
    for c in ("FETCH_SIZE", "WRITE_SIZE"):
        pts = [(n, r[c]["bytes_per_launch"]) for n, r in sorted(rows.items()) if c in r]
        if len(pts) >= 2:
            fixed, slope = fit([p[0] for p in pts], [p[1] for p in pts])
            out["fit"][c] = {"fixed_bytes_per_launch": fixed, "bytes_per_arena": slope,
                             "residuals": [y - (fixed + slope * x) for x, y in pts]}
        for n, y in pts:
            print(f"{c:10s} N={n:6d}  {y / 1e6:8.3f} MB/launch  {y / n:8.1f} B/arena")
    for c, f in out["fit"].items():
        print(f"{c:10s} fixed {f['fixed_bytes_per_launch'] / 1e6:.3f} MB/launch, {f['bytes_per_arena']:.1f} B/arena")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
