"""Per-launch averages of the SQ counters collected by scripts/sq.sh for hk::step_kernel."""
import collections
import csv
import glob
import os

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
acc = collections.defaultdict(list)
for fn in glob.glob(os.path.join(ROOT, "gpurun_out", "sq_*", "**", "*counter_collection.csv"), recursive=True):
    for row in csv.DictReader(open(fn)):
        if "step_kernel<false>" in row["Kernel_Name"]:
            acc[row["Counter_Name"]].append(float(row["Counter_Value"]))
avg = {k: sum(v) / len(v) for k, v in acc.items()}
for k in sorted(avg):
    print(f"{k:28s} {avg[k]:16.1f}")
w = avg.get("SQ_WAVES", 1)
if "SQ_ACTIVE_INST_VALU" in avg and "SQ_THREAD_CYCLES_VALU" in avg:
    print("lane utilisation of VALU (thread cycles / (64 x active VALU cycles)):",
          avg["SQ_THREAD_CYCLES_VALU"] / (64 * avg["SQ_ACTIVE_INST_VALU"]))
for k in ("SQ_INSTS_VALU", "SQ_INSTS_SALU", "SQ_INSTS_VMEM", "SQ_INSTS_LDS", "SQ_INSTS_SMEM", "SQ_INSTS_BRANCH"):
    if k in avg:
        print(f"{k} per wave: {avg[k] / w:.0f}")
