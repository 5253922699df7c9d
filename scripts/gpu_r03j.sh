#!/bin/bash
# r03j: single-arena latency split (launch+sync / back-to-back / rollout), then the round's counter and profile
# refresh (scripts/profile_round.sh: PMC, SQ, driver command, long bench, rocprof kernel stats, tail stats).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03j
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread > $O/pytest_facade.log 2>&1 || exit 1
tail -1 $O/pytest_facade.log
timeout -k 10 120 python3 scripts/facade_profile.py 3000 > $O/facade_profile.log 2>&1 || exit 1
tail -1 $O/facade_profile.log
timeout -k 10 120 python3 scripts/single_env_latency.py > $O/single_env_latency.log 2>&1 || exit 1
tail -2 $O/single_env_latency.log
TAG=r03 ./scripts/profile_round.sh
