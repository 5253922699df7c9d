#!/bin/bash
# Quick GPU iteration: parity tests then the bench line (no CPU baseline).  Stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*' gpurun_out/bench.log
