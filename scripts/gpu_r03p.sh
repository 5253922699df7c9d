#!/bin/bash
# r03p: learner update cost at the C5 batch (eager vs graph, and the rocprofv3 kernel split), then the stage-1
# learning pin on 4 arenas (episodes end at done), 10 000 episodes.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03p
mkdir -p $O
timeout -k 10 120 python3 scripts/learner_profile.py 16384 200 > $O/learner.log 2>&1 || { tail -5 $O/learner.log; exit 1; }
tail -1 $O/learner.log
rm -rf gpurun_out/prof_learner
timeout -k 10 180 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner -o run --output-format csv -- python3 scripts/learner_profile.py 16384 100 > $O/learner_prof.log 2>&1 || exit 1
find gpurun_out/prof_learner -name "*kernel_stats.csv" -exec cp {} $O/learner_kernel_stats.csv \;
head -12 $O/learner_kernel_stats.csv | cut -c1-160
timeout -k 10 1000 python -u scripts/td3_stage1_pin.py --arenas 4 --episodes 10000 --out $O/stage1_pin_n4.json > $O/pin_n4.log 2>&1
tail -2 $O/pin_n4.log | cut -c1-300
