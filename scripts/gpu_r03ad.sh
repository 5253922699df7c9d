#!/bin/bash
# r03ad: learner update cost with torch's two BLAS back ends on ROCm (hipBLASLt, the default, and rocBLAS), at the
# C5 batch and the reference's 256; rocprofv3 kernel split of the rocBLAS case.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ad
mkdir -p $O
for b in cublaslt cublas; do
  for B in 16384 256; do
    HK_BLAS=$b timeout -k 10 150 python3 scripts/learner_profile.py $B 300 > $O/learner_${b}_$B.log 2>&1 || { tail -5 $O/learner_${b}_$B.log; exit 1; }
    tail -1 $O/learner_${b}_$B.log
  done
done
rm -rf gpurun_out/prof_learner2
HK_BLAS=cublas timeout -k 10 200 rocprofv3 --kernel-trace --stats -d gpurun_out/prof_learner2 -o run --output-format csv -- python3 scripts/learner_profile.py 16384 100 > $O/learner_prof.log 2>&1 || exit 1
find gpurun_out/prof_learner2 -name "*kernel_stats.csv" -exec cp {} $O/learner_kernel_stats_rocblas.csv \;
head -8 $O/learner_kernel_stats_rocblas.csv | cut -d, -f1-4 | cut -c1-160
