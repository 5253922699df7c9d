#!/bin/bash
# r03m: multi-stream shard sweep (scripts/stream_sweep.py) under 4 / 8 / 16 hardware queues per process.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03m
mkdir -p $O
for Q in 4 8 16; do
  GPU_MAX_HW_QUEUES=$Q timeout -k 10 240 python3 scripts/stream_sweep.py 1 2 3 4 8 16 > $O/sweep_q$Q.log 2>&1 || { tail -5 $O/sweep_q$Q.log; exit 1; }
  grep hw_queues $O/sweep_q$Q.log
done
