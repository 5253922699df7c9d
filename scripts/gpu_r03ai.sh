#!/bin/bash
# r03ai: A/B of the general velocity family with per-slot wave-uniform point-count rows (one iteration per trip,
# the snapshot every 4th) against the committed head, three alternations; tail statistics of both diagnostics
# builds; the full GPU suite.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ai
mkdir -p $O
L=hockey-env_amd/hockey_amd/_lib
for i in 1 2 3; do
  for lib in libhockey_hip_base.so libhockey_hip.so; do
    HK_LIB=$L/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --rollout 50 --streams 0 --facade-steps 0 \
      --c5-steps 0 --c4-steps 0 --steps 300 --warmup 200 > $O/ab_${lib}_$i.log 2>&1 || { tail -5 $O/ab_${lib}_$i.log; exit 1; }
    echo "$i $lib $(grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*' $O/ab_${lib}_$i.log | tr '\n' ' ')"
  done
done
for t in timers_base timers; do HK_LIB=$L/libhockey_hip_$t.so timeout -k 10 240 python scripts/tail_stats.py 65536 20 > $O/tail_$t.log 2>&1 || { tail -5 $O/tail_$t.log; exit 1; }; echo "== $t"; sed -n 2,2p $O/tail_$t.log; sed -n 6,20p $O/tail_$t.log; done
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1; rc=$?; tail -2 $O/pytest_gpu.log; exit $rc
