#!/bin/bash
# r03ac: where a C5 learner update's time goes (scripts/learner_profile.py at the C5 batch of 16 384 and at the
# reference's 256; eager vs graph-replayed), with the rocprofv3 kernel split of the graph-replayed 16 384 case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ac
mkdir -p $O
timeout -k 10 150 python3 scripts/learner_profile.py 16384 200 > $O/learner_16384.log 2>&1 || { tail -5 $O/learner_16384.log; exit 1; }
tail -1 $O/learner_16384.log
timeout -k 10 150 python3 scripts/learner_profile.py 256 2000 > $O/learner_256.log 2>&1 || { tail -5 $O/learner_256.log; exit 1; }
tail -1 $O/learner_256.log
rm -rf gpurun_out/prof_learner
timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner -o run --output-format csv -- python3 scripts/learner_profile.py 16384 100 > $O/learner_prof.log 2>&1 || exit 1
find gpurun_out/prof_learner -name "*kernel_stats.csv" -exec cp {} $O/learner_kernel_stats.csv \;
head -25 $O/learner_kernel_stats.csv | cut -d, -f1-5 | cut -c1-200
