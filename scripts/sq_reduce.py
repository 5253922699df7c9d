"""Per-launch averages of the SQ counters collected by scripts/sq.sh for hk::step_kernel (single-step launches),
and profiles/sq_summary.json[<key>] for bench.py's VALU roofline.

Units (MI355X_MICROARCH.md, rocprofv3 PMC / cycle constants): SQ_WAVE_CYCLES, SQ_WAIT_*, SQ_ACTIVE_INST_* count
quad-cycles summed over waves.  One wave alone on its SIMD issues a VALU op in 4 cycles = one quad-cycle
(SQ_ACTIVE_INST_VALU ~= SQ_INSTS_VALU confirms it), so SQ_THREAD_CYCLES_VALU (active lanes x quad-cycles) is
the active-lane VALU operation count of the launch.

Usage: python scripts/sq_reduce.py [key] [source-label]"""
import collections
import csv
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "hockey-env_amd"))
from hockey_amd._native import built_hash, source_hash  # noqa: E402  (pure Python: no GPU, no library load)
acc = collections.defaultdict(list)
for fn in glob.glob(os.path.join(ROOT, "gpurun_out", "sq_*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(fn)):
        if "step_kernel<false>" in row["Kernel_Name"]:
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(avg):
    print(f"{k:28s} {avg[k]:16.1f}")
w = avg.get("SQ_WAVES", 1)
lane_util = issue_util = None
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_THREAD_CYCLES_VALU" in avg:
    lane_util = avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"])
    print("lane utilisation of VALU (thread cycles / (64 x active VALU cycles)):", lane_util)
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_WAVE_CYCLES" in avg:
    issue_util = avg["SQ_ACTIVE_INST_VALU"] / avg["SQ_WAVE_CYCLES"]
    print("VALU issue share of wave time (active VALU / wave cycles):", issue_util)
    for k in ("SQ_WAIT_ANY", "SQ_WAIT_INST_ANY", "SQ_ACTIVE_INST_ANY"):
        if k in avg:
            print(f"{k} share of wave time: {avg[k] / avg['SQ_WAVE_CYCLES']:.3f}")
    print(f"mean wave lifetime: {4 * avg['SQ_WAVE_CYCLES'] / w:.0f} cycles")
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
    if k in avg:
        print(f"{k} per wave: {avg[k] / w:.0f}")
if len(sys.argv) > 1 and "SQ_THREAD_CYCLES_VALU" in avg:
    key = sys.argv[1]
    out_path = os.path.join(ROOT, "profiles", "sq_summary.json")
    d = json.load(open(out_path)) if os.path.exists(out_path) else {}
    d[key] = {"valu_lane_ops_per_launch": avg["SQ_THREAD_CYCLES_VALU"], "valu_lane_util": lane_util,
              "valu_issue_util": issue_util, "valu_insts_per_wave": avg.get("SQ_INSTS_VALU", 0) / w,
              "waves": w, "counters": avg,
              "source": sys.argv[2] if len(sys.argv) > 2 else "scripts/sq.sh + scripts/sq_reduce.py",
              "source_hash": source_hash(), "library_hash": built_hash()}
    json.dump(d, open(out_path, "w"), indent=1)
