#!/bin/bash
# r03k: wave regrouping -- GPU parity (full suite, including regrouped == fixed lanes), A/B bench (regrouped vs
# HK_DIAG_FIXED_LANES, interleaved), tail statistics of the regrouped kernel.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03k
mkdir -p $O
timeout -k 10 700 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -3 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="--steps 300 --warmup 50 --facade-steps 0 --c5-steps 0 --no-cpu-baseline --streams 0"
for k in 1 2; do
  timeout -k 10 150 python3 bench.py $B > $O/bench_regroup_$k.log 2>&1 || exit 1
  timeout -k 10 150 python3 bench.py $B --fixed-lanes > $O/bench_fixed_$k.log 2>&1 || exit 1
  python3 -c "
import json
for t in ('regroup','fixed'):
    d=json.loads(open('$O/bench_'+t+'_$k.log').read().strip().splitlines()[-1]); print(t, round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_avg_ms'],4), 'ms', 'rollout', round(d['rollout']['value']/1e6,1), 'c4', round(d['c4_shard']['value']/1e6,1))"
done
timeout -k 10 300 python scripts/tail_stats.py 65536 30 > $O/tail_stats.txt 2>&1 || exit 1
head -20 $O/tail_stats.txt
