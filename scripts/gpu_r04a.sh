#!/bin/bash
# r04a: the GPU suite (new: every shipped checkpoint vs its recorded win rates, hk_step_host on fresh contexts),
# then the driver's bench command.  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04a
mkdir -p $O
export HK_PIN_OUT=$O/checkpoint_pins.json
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -5 $O/driver_cmd.log; exit 1; }
grep -o '"value": [0-9.e+]*\|"streams": {[^}]*}' $O/driver_cmd.log | head -6
