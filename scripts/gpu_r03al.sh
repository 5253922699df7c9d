#!/bin/bash
# r03al: validation and round evidence after the iterative-ilp machine scheduler: the full GPU suite,
# __graft_entry__.smoke(), the driver's bench command, then scripts/profile_round.sh.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03al
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke(); print('smoke ok')" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -5 $O/driver_cmd.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"counters_stale": [a-z]*\|"streams": {[^}]*}' $O/driver_cmd.log | head -6
# round evidence at this head (counters stamped with the library hash)
TAG=r03al ./scripts/profile_round.sh
