#!/bin/bash
# r04d: rocprofv3 kernel stats of the fused learner (batch 16 384).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04d
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/learner_profile.py 16384 100 fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
grep "^{" $O/prof.log | tail -1
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp "$f" $O/learner_kernel_stats.csv
python3 - "$O/learner_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r["TotalDurationNs"]))[:20]:
    print(f'{r["Name"][:70]:70s} {r["Calls"]:>7s} {float(r["AverageNs"])/1e3:9.1f} us {float(r["Percentage"]):6.2f} %')
PY
