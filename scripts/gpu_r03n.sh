#!/bin/bash
# r03n: multi-stream shard sweep, one process per (hardware queues, streams) configuration.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03n
mkdir -p $O
for Q in 4 8 16; do
  for S in 2 3 4 6 8; do
    GPU_MAX_HW_QUEUES=$Q timeout -k 10 120 python3 scripts/stream_sweep.py $S >> $O/sweep.log 2>&1 || { tail -5 $O/sweep.log; exit 1; }
  done
done
grep hw_queues $O/sweep.log
