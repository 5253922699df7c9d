#!/bin/bash
# r03g: facade (hk_step_host) tests + timing, then the stage-1 learning pin (episode_end=done).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03g
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread > $O/pytest_facade.log 2>&1
rc=$?; tail -2 $O/pytest_facade.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 120 python -c "import json, bench; print(json.dumps(bench.time_facade(3000, 'cuda:0')))" > $O/facade.log 2>&1 || exit 1
tail -1 $O/facade.log
timeout -k 10 700 python -u scripts/td3_stage1_pin.py --out $O/stage1_pin.json --checkpoint $O/td3_stage1_last.pt > $O/pin.log 2>&1
tail -2 $O/pin.log
