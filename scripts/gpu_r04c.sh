#!/bin/bash
# r04c: the fused MFMA learner -- its GPU tests (G9 eager on the GPU, G9b fused, fused vs eager, graph replay), then
# the learner profile (ms per update, torch vs fused).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04c
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_learner.py -x -v --timeout 200 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; tail -15 $O/pytest_learner.log; [ $rc -eq 0 ] || { grep -B2 -A30 "Error\|assert" $O/pytest_learner.log | head -80; exit $rc; }
timeout -k 10 300 python -u scripts/learner_profile.py 16384 100 > $O/learner_profile.log 2>&1 || { tail -20 $O/learner_profile.log; exit 1; }
tail -1 $O/learner_profile.log
timeout -k 10 300 python -u scripts/learner_profile.py 256 400 > $O/learner_profile_b256.log 2>&1 || { tail -20 $O/learner_profile_b256.log; exit 1; }
tail -1 $O/learner_profile_b256.log
bash scripts/gpu_r04d.sh
