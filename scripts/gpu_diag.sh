#!/bin/bash
# GPU diagnostics round-trip: parity tests, bench (no CPU baseline), per-phase cycles and tail statistics
# (diagnostics library libhockey_hip_timers.so).  Stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > gpurun_out/pytest_gpu.log 2>&1 || { tail -30 gpurun_out/pytest_gpu.log; exit 1; }
tail -1 gpurun_out/pytest_gpu.log
timeout -k 10 300 python bench.py --no-cpu-baseline ${BENCH_ARGS:-} > gpurun_out/bench.log 2>&1
grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*' gpurun_out/bench.log
timeout -k 10 300 python scripts/phase_timers.py 65536 strong > gpurun_out/phase.log 2>&1
grep -v amdgpu.ids gpurun_out/phase.log
timeout -k 10 300 python scripts/tail_stats.py 65536 30 > gpurun_out/tail.log 2>&1
grep -v amdgpu.ids gpurun_out/tail.log | head -8
