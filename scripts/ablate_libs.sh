#!/bin/bash
# Timing ablations: the bench (no CPU baseline, no rollout) with each diagnostic library in $LIBS.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS}; do
  HK_LIB=hockey-env_amd/hockey_amd/_lib/$L timeout -k 10 120 python bench.py --no-cpu-baseline --rollout ${ROLL:-0} --steps 300 --warmup 200 > gpurun_out/abl_$L.log 2>&1
  echo "$L $(grep -o '"kernel_avg_ms": [0-9.e+]*' gpurun_out/abl_$L.log) $(grep -o '"rollout": {[^}]*}' gpurun_out/abl_$L.log | grep -o '"ms_per_step": [0-9.]*')"
done
