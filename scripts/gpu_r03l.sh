#!/bin/bash
# r03l: full GPU suite at the current head, then the round evidence (scripts/profile_round.sh: PMC traffic, SQ
# counters, the driver's bench command, rocprofv3 kernel stats, tail statistics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03l
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
TAG=r03l ./scripts/profile_round.sh
