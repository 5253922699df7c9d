#!/bin/bash
# Instruction-mix / stall / cache counters of the step kernel (rocprofv3 --pmc, counters only, one pass per
# group; at most 8 SQ-block counters per pass).  Override the passes with P1..P4; reduce with sq_reduce.py.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---no-cpu-baseline --rollout 0 --streams 0 --facade-steps 0 --c5-steps 0 --c4-steps 0 --steps 40 --warmup 20}
P1=${P1-"SQ_WAVES SQ_INSTS_VALU SQ_INSTS_SALU SQ_INSTS_SMEM SQ_INSTS_VMEM SQ_INSTS_LDS SQ_INSTS_BRANCH SQ_BUSY_CYCLES"}
P2=${P2-"SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_THREAD_CYCLES_VALU SQ_ACTIVE_INST_LDS SQ_ACTIVE_INST_SCA SQ_WAVE_CYCLES"}
P3=${P3-}
P4=${P4-}
i=0
for P in "$P1" "$P2" "$P3" "$P4"; do
  i=$((i+1))
  [ -n "$P" ] || continue
  rm -rf gpurun_out/sq_$i
  timeout -s KILL 120 rocprofv3 --pmc $P -d gpurun_out/sq_$i -o run --output-format csv -- python3 bench.py $ARGS > gpurun_out/sq_$i.log 2>&1
  echo "pass $i ok"
done
