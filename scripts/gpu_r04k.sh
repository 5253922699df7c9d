#!/bin/bash
# r04k: rocprofv3 kernel stats of the bench command at this head (step kernel duration without HIP-event markers).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04k
mkdir -p $O
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --streams 0 --rollout 0 --facade-steps 0 --c5-steps 0 --c4-steps 0 > $O/prof_bench.log 2>&1 || { tail $O/prof_bench.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); cp $f $O/kernel_stats.csv; head -3 $O/kernel_stats.csv
grep "^{" $O/prof_bench.log | cut -c1-200
