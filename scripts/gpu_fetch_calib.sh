#!/bin/bash
# FETCH_SIZE / WRITE_SIZE calibration of the step kernel's access widths (scripts/micro/fetch_calib.hip), one
# counter per rocprofv3 pass, then scripts/fetch_calib_reduce.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/fetch_calib
mkdir -p $O
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -o /tmp/fetch_calib scripts/micro/fetch_calib.hip 2> $O/build.log || { tail $O/build.log; exit 1; }
timeout -k 10 60 /tmp/fetch_calib > $O/known.txt || exit 1
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 60 rocprofv3 --pmc $C -d $O/pmc_$C -o run --output-format csv -- /tmp/fetch_calib > $O/pmc_$C.log 2>&1 || { tail $O/pmc_$C.log; exit 1; }
done
python3 scripts/fetch_calib_reduce.py $O
