#!/bin/bash
# r04aa: bench.py with no flags (its defaults: N=1, 500 timed steps after 300, every auxiliary line), timed.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04aa
mkdir -p $O
t0=$(date +%s)
timeout -k 10 900 python3 bench.py > $O/bench_default.log 2>&1 || { tail -20 $O/bench_default.log; exit 1; }
echo "bench.py default: $(( $(date +%s) - t0 )) s wall"
tail -1 $O/bench_default.log | cut -c1-300
