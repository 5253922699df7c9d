#!/bin/bash
# HBM traffic of the step kernel from rocprofv3 PMC counters: FETCH_SIZE and WRITE_SIZE in separate passes
# (they do not fit one pass on gfx950), counters only (no trace domains), same bench command as bench.py.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
ARGS=${BENCH_ARGS:---no-cpu-baseline --rollout 0 --streams 0 --facade-steps 0 --c5-steps 0 --c4-steps 0 --steps 40 --warmup 20}
for C in FETCH_SIZE WRITE_SIZE; do
  rm -rf gpurun_out/pmc_$C
  timeout -k 10 600 rocprofv3 --pmc $C -d gpurun_out/pmc_$C -o run --output-format csv -- \
    python3 bench.py $ARGS > gpurun_out/pmc_$C.log 2>&1
  echo "$C pass rc=$?"
done
