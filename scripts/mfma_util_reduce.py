"""Per-kernel MFMA utilisation of the fused learner from scripts/gpu_r04af.sh's PMC pass: SQ_VALU_MFMA_BUSY_CYCLES
(cycles summed over the chip's SIMDs; 32 per v_mfma_f32_16x16x4_f32, which the FLOP count checks) over the kernel's
SIMD-cycles, GRBM_GUI_ACTIVE / 8 x 256 CUs x 4 SIMDs (GRBM_GUI_ACTIVE is summed over the 8 XCDs: it reads 8 x
~2.44 GHz x the dispatch duration), per dispatch, averaged per kernel after the first fifth of the dispatches.
Usage: python scripts/mfma_util_reduce.py DIR [OUT.json]"""
import csv
import glob
import json
import os
import sys
from collections import defaultdict

SIMDS = 256 * 4
XCDS = 8


def main():
    d = sys.argv[1]
    per = defaultdict(lambda: defaultdict(dict))
    for fn in glob.glob(os.path.join(d, "**", "*counter_collection.csv"), recursive=True):
        with open(fn) as f:
            for row in csv.DictReader(f):
                name = row["Kernel_Name"].split("(")[0]
                if not name.startswith("hkl::"):
                    continue
                per[name][row["Dispatch_Id"]][row["Counter_Name"]] = float(row["Counter_Value"])
    out = {}
    for name, disp in sorted(per.items()):
        ids = sorted(disp, key=int)
        ids = ids[len(ids) // 5:]
        u = [disp[i]["SQ_VALU_MFMA_BUSY_CYCLES"] / (disp[i]["GRBM_GUI_ACTIVE"] / XCDS * SIMDS) for i in ids
             if disp[i].get("GRBM_GUI_ACTIVE")]
        if u:
            out[name] = {"mfma_busy_frac": sum(u) / len(u), "dispatches": len(u)}
            print(f"{name:32s} MFMA busy {100 * out[name]['mfma_busy_frac']:5.1f} %  ({len(u)} dispatches)")
    if len(sys.argv) > 2:
        with open(sys.argv[2], "w") as f:
            json.dump({"what": __doc__.split(".")[0], "kernels": out}, f, indent=1)


if __name__ == "__main__":
    main()
