#!/bin/bash
# One GPU round-trip: parity tests, smoke, a short bench, and a rocprofv3 kernel-trace summary.
# Every GPU step has its own time limit; a crash/timeout (exit >= 124 or signal) stops the script.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
OUT=gpurun_out
mkdir -p $OUT
ok() { local rc=$1; [ "$rc" -eq 0 ] || [ "$rc" -eq 1 ]; }   # 1 = test failures (not a crash)
timeout -k 10 ${T_TEST:-900} python -m pytest tests -m gpu -x -q ${PYTEST_ARGS:-} > $OUT/pytest_gpu.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 $OUT/pytest_gpu.log
ok $rc || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $OUT/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -3 $OUT/smoke.log
[ $rc -eq 0 ] || exit $rc
timeout -k 10 ${T_BENCH:-600} python bench.py ${BENCH_ARGS:-} > $OUT/bench.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -3 $OUT/bench.log
[ $rc -eq 0 ] || exit $rc
if [ "${PROFILE:-1}" = "1" ]; then
  timeout -k 10 600 rocprofv3 --kernel-trace --stats -d $OUT/prof -o run --output-format csv -- \
    python3 bench.py --no-cpu-baseline ${BENCH_ARGS:-} > $OUT/prof.log 2>&1
  rc=$?; echo "rocprof rc=$rc"; tail -3 $OUT/prof.log
  find $OUT/prof -name "*stats*" | head
fi
