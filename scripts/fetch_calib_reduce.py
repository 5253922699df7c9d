"""Reduce the FETCH_SIZE / WRITE_SIZE passes of scripts/micro/fetch_calib.hip (scripts/gpu_fetch_calib.sh): for each
calibration kernel, the counter per launch divided by the bytes the kernel is known to move, i.e. the factor that
turns the counter into bytes for that access width.  Writes profiles/r04/fetch_calib.json.
Usage: python scripts/fetch_calib_reduce.py DIR   (DIR holds pmc_FETCH_SIZE/, pmc_WRITE_SIZE/ and known.txt)"""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def counter_by_kernel(d, counter):
    vals = {}
    for fn in glob.glob(os.path.join(d, f"pmc_{counter}", "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                if row.get("Counter_Name") != counter:
                    continue
                name = row["Kernel_Name"].split("(")[0].split()[-1]
                vals.setdefault(name, []).append(float(row["Counter_Value"]) * 1024.0)  # KiB -> B
    return {k: sum(v[1:]) / max(1, len(v) - 1) for k, v in vals.items()}  # first launch dropped (cold)


def main():
    d = sys.argv[1]
    known = {}
    for line in open(os.path.join(d, "known.txt")):
        k, r, w = line.split()
        known[k] = (int(r), int(w))
    fetch, write = counter_by_kernel(d, "FETCH_SIZE"), counter_by_kernel(d, "WRITE_SIZE")
    out = {"what": "FETCH_SIZE / WRITE_SIZE bytes per launch over the known bytes, per access pattern "
                   "(scripts/micro/fetch_calib.hip; first launch of each kernel dropped)", "kernels": {}}
    for k, (r, w) in known.items():
        f, wr = fetch.get(k), write.get(k)
        out["kernels"][k] = {"known_read": r, "known_write": w, "fetch_size_bytes": f, "write_size_bytes": wr,
                             "fetch_per_written_byte": f / w if f is not None and w else None,
                             "fetch_over_known": f / r if f is not None and r else None,
                             "write_over_known": wr / w if wr is not None and w else None}
        print(f"{k:12s} read {r:10d} FETCH {f if f is None else round(f):>10}  ratio "
              f"{out['kernels'][k]['fetch_over_known']}  | write {w:10d} WRITE {wr if wr is None else round(wr):>10}  "
              f"ratio {out['kernels'][k]['write_over_known']}  | FETCH per byte written "
              f"{out['kernels'][k]['fetch_per_written_byte']}")
    os.makedirs(os.path.join(ROOT, "profiles", "r04"), exist_ok=True)
    with open(os.path.join(ROOT, "profiles", "r04", "fetch_calib.json"), "w") as f:
        json.dump(out, f, indent=1)


if __name__ == "__main__":
    main()
