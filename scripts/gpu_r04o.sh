#!/bin/bash
# r04o: the whole GPU suite at this head.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04o
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
