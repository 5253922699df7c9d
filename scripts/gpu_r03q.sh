#!/bin/bash
# r03q: step-start latency.  A/B of the committed kernel (libhockey_hip_base.so) against the prefetching one
# (first step's HBM words issued before the scene copy, 16-B scene copy), tail statistics with phase 0 split
# into scene copy / arena load / policy (slots 8 / 9 / 10) for both, then the full GPU suite on the new build.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03q
mkdir -p $O
L=hockey-env_amd/hockey_amd/_lib
for lib in libhockey_hip_base.so libhockey_hip.so libhockey_hip_base.so libhockey_hip.so; do
  HK_LIB=$L/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --rollout 50 --streams 0 --facade-steps 2000 \
    --c5-steps 0 --c4-steps 0 --steps 300 --warmup 200 > $O/ab_$lib.log 2>&1 || { tail -5 $O/ab_$lib.log; exit 1; }
  echo "$lib $(grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*\|"facade_single_env": {[^}]*}' $O/ab_$lib.log | tr '\n' ' ')"
  grep -o '"rollout": {[^}]*}' $O/ab_$lib.log | cut -c1-200
done
for t in tsplit_old tsplit; do
  HK_LIB=$L/libhockey_hip_$t.so timeout -k 10 240 python scripts/tail_stats.py 65536 20 > $O/tail_$t.log 2>&1 || { tail -5 $O/tail_$t.log; exit 1; }
  HK_LIB=$L/libhockey_hip_$t.so timeout -k 10 120 python scripts/tail_stats.py 64 200 > $O/tail64_$t.log 2>&1 || { tail -5 $O/tail64_$t.log; exit 1; }
  echo "== $t"; sed -n 6,20p $O/tail_$t.log; sed -n 6,20p $O/tail64_$t.log
done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; exit $rc
