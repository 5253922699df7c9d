"""Reduce the rocprofv3 PMC passes of scripts/pmc.sh to per-launch HBM bytes of hk::step_kernel and
write profiles/pmc_summary.json (read by bench.py for roofline.traffic).

FETCH_SIZE / WRITE_SIZE are KiB per dispatch.  MI355X_MICROARCH.md (HBM [CDNA4]): on gfx950 FETCH_SIZE
reports 1/2 of the bytes of wide coalesced reads -> doubled here; WRITE_SIZE is exact."""
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
from hockey_amd._native import built_hash, source_hash  # noqa: E402  (pure Python: no GPU, no library load)


def per_launch(counter):
    files = glob.glob(os.path.join(ROOT, "gpurun_out", f"pmc_{counter}", "**", "*counter_collection.csv"),
                      recursive=True)
    vals = []
    for fn in files:
        with open(fn) as f:
            for row in csv.DictReader(f):
                if "step_kernel<false>" in row.get("Kernel_Name", "") and row.get("Counter_Name") == counter:
                    vals.append(float(row["Counter_Value"]))
    if not vals:
        sys.exit(f"no {counter} rows for step_kernel in {files}")
    return sum(vals) / len(vals), len(vals)


if __name__ == "__main__":
    key = sys.argv[1] if len(sys.argv) > 1 else "basic_65536"
    source = sys.argv[2] if len(sys.argv) > 2 else "scripts/pmc.sh + scripts/pmc_reduce.py"
    fetch_kib, nf = per_launch("FETCH_SIZE")
    write_kib, nw = per_launch("WRITE_SIZE")
    read_b = 2.0 * fetch_kib * 1024.0  # gfx950 FETCH_SIZE correction (x2)
    write_b = write_kib * 1024.0
    out_path = os.path.join(ROOT, "profiles", "pmc_summary.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"fetch_size_kib_per_launch_raw": fetch_kib, "write_size_kib_per_launch": write_kib,
              "read_bytes_per_launch": read_b, "write_bytes_per_launch": write_b,
              "hbm_bytes_per_launch": read_b + write_b, "launches": [nf, nw], "source": source,
              "source_hash": source_hash(), "library_hash": built_hash(),
              "note": "rocprofv3 --pmc FETCH_SIZE / --pmc WRITE_SIZE in separate passes (scripts/pmc.sh); "
                      "FETCH_SIZE x2 per MI355X_MICROARCH.md gfx950 correction"}
    json.dump(d, open(out_path, "w"), indent=1)
    print(json.dumps(d[key], indent=1))
