#!/bin/bash
# r04af: MFMA busy cycles of the fused learner's kernels (rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE,
# counters only, one pass) over scripts/learner_profile.py at batch 16 384; reduce with scripts/mfma_util_reduce.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04af
mkdir -p $O
timeout -s KILL 300 rocprofv3 --pmc SQ_VALU_MFMA_BUSY_CYCLES GRBM_GUI_ACTIVE -d $O/pmc -o run --output-format csv -- \
  python3 scripts/learner_profile.py 16384 50 fused > $O/pmc.log 2>&1
rc=$?; echo "pmc pass rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/pmc.log; exit $rc; }
