#!/bin/bash
# r03i: full GPU suite on the final-candidate kernel (cooperative collide, no rot_set2), then where the facade's
# time goes (bare hk_step_host mapped vs staged, empty round trip, facade) with the N=1 kernel trace.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03i
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python3 scripts/facade_profile.py 3000 > $O/facade_profile.log 2>&1 || exit 1
tail -1 $O/facade_profile.log
rm -rf gpurun_out/prof_facade
timeout -k 10 180 rocprofv3 --kernel-trace --memory-copy-trace --stats -d gpurun_out/prof_facade -o run --output-format csv -- \
  python3 scripts/facade_profile.py 2000 > $O/facade_prof_run.log 2>&1 || exit 1
find gpurun_out/prof_facade -name "*kernel_stats.csv" -exec cp {} $O/facade_kernel_stats.csv \;
find gpurun_out/prof_facade -name "*memory_copy_stats.csv" -exec cp {} $O/facade_copy_stats.csv \;
head -5 $O/facade_kernel_stats.csv | cut -c1-200
