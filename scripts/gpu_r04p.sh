#!/bin/bash
# r04p: lone-lane drains (single-arena contexts walk their own queues) -- GPU suite, facade latency split.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04p
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/facade_profile.py 5000 > $O/facade_profile.log 2>&1 || { tail -20 $O/facade_profile.log; exit 1; }
tail -1 $O/facade_profile.log
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline --rollout 0 --streams 0 > $O/bench_long.log 2>&1 || { tail -20 $O/bench_long.log; exit 1; }
grep "^{" $O/bench_long.log | cut -c1-200
