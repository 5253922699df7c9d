#!/bin/bash
# r04g: facade after the Python trims -- its GPU tests, the latency split (scripts/facade_profile.py) and the N=1
# step kernel's duration under rocprofv3 --kernel-trace --stats.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -2 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -60; exit $rc; }
timeout -k 10 300 python -u scripts/facade_profile.py 5000 > $O/facade_profile.log 2>&1 || { tail -20 $O/facade_profile.log; exit 1; }
tail -1 $O/facade_profile.log
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/facade_profile.py 3000 > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
f=$(find $O/prof -name "*kernel_stats.csv" | head -1); head -5 "$f"
