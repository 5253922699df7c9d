#!/bin/bash
# r03v: the driver's bench command after bench.py raises GPU_MAX_HW_QUEUES to 8 over the box's exported 4 (r03t's
# line had the 4-shard streams leg at 115 M: two shard streams shared a queue), and the facade GPU tests after the
# facade's action / increment staging change.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03v
mkdir -p $O
echo "box GPU_MAX_HW_QUEUES=${GPU_MAX_HW_QUEUES:-unset}"
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -v --timeout 120 --timeout-method thread > $O/pytest_facade.log 2>&1
rc=$?; tail -2 $O/pytest_facade.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -5 $O/driver_cmd.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"streams": {[^}]*}\|"facade_single_env": {"value": [0-9.e+]*' $O/driver_cmd.log | head -5
