#!/bin/bash
# r03e: coop-TOI parity + A/B bench vs the round-start library, then TD3 learning diagnostics (eager vs graph).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03e
mkdir -p $O
timeout -k 10 300 python -u -m pytest tests/test_gpu_parity.py -x -q --timeout 200 --timeout-method thread -k "lockstep or rollout or large_island or c4" > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="--steps 300 --warmup 50 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline --streams 0"
for k in 1 2; do
  timeout -k 10 120 python3 bench.py $B > $O/bench_new_$k.log 2>&1 || exit 1
  HK_LIB=hockey-env_amd/hockey_amd/_lib/libhockey_hip_prev.so timeout -k 10 120 python3 bench.py $B > $O/bench_prev_$k.log 2>&1 || exit 1
  python3 -c "
import json
for t in ('new','prev'):
    d=json.loads(open('$O/bench_'+t+'_$k.log').read().strip().splitlines()[-1]); print(t, round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_avg_ms'],4), 'ms', 'rollout', round(d['rollout']['value']/1e6,1))"
done
timeout -k 10 300 python -u scripts/td3_diag.py 3600 20 0 30 > $O/td3_eager.log 2>&1; tail -3 $O/td3_eager.log
timeout -k 10 300 python -u scripts/td3_diag.py 3600 20 1 30 > $O/td3_graph.log 2>&1; tail -3 $O/td3_graph.log
