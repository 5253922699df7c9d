#!/bin/bash
# r03ah: the bench with no arguments (every default: 500 timed steps after 300 warmup and the 1000-step preroll,
# every side leg, the CPU baseline), as a driver may run it; wall time of the whole command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ah
mkdir -p $O
t0=$(date +%s)
timeout -k 10 600 python3 bench.py > $O/bench_default.log 2>&1 || { tail -5 $O/bench_default.log; exit 1; }
echo "wall_s $(( $(date +%s) - t0 ))"
grep -o '"value": [0-9.e+]*\|"counters_stale": [a-z]*\|"ms_per_step": [0-9.]*' $O/bench_default.log | head -8
