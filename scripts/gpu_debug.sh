#!/bin/bash
# GPU-vs-host lockstep divergence report for a list of library builds.  Each GPU step has its own time
# limit; any failure (crash, timeout) ends the script (set -e).
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
mkdir -p gpurun_out
for L in ${LIBS:-libhockey_hip.so}; do
  echo "== $L"
  HK_LIB=hockey-env_amd/hockey_amd/_lib/$L timeout -k 10 200 python scripts/debug_lockstep.py 1 3 128 260 > gpurun_out/dbg_a.log 2>&1
  grep -E "^step|counters" gpurun_out/dbg_a.log || true
  HK_LIB=hockey-env_amd/hockey_amd/_lib/$L timeout -k 10 200 python scripts/debug_lockstep.py 0 1 1024 400 strong > gpurun_out/dbg_b.log 2>&1
  grep -E "^step|counters" gpurun_out/dbg_b.log || true
done
