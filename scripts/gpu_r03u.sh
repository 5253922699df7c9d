#!/bin/bash
# r03u: single-env facade latency, the committed kernel (libhockey_hip_base.so: hk_step_host synchronises the
# stream) against the completion-word wait (the kernel stores the launch's sequence number into the mapped
# buffer after its last output; the host polls it), twice each, then the facade and parity GPU tests.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03u
mkdir -p $O
L=hockey-env_amd/hockey_amd/_lib
for lib in libhockey_hip_base.so libhockey_hip.so libhockey_hip_base.so libhockey_hip.so; do
  HK_LIB=$L/$lib timeout -k 10 120 python scripts/facade_profile.py 3000 > $O/facade_$lib.log 2>&1 || { tail -5 $O/facade_$lib.log; exit 1; }
  echo "$lib $(grep -v amdgpu.ids $O/facade_$lib.log | tail -1)"
done
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
