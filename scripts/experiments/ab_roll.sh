#!/bin/bash
# One-off A/B (r05): the step kernel with its velocity-family iteration loops rolled
# (`#pragma unroll 1` on the 4-iteration trips of vone / vtwo / vgen: lib exp/libhockey_hip_roll_r3.so; vtwo and
# vgen only: roll_r2) against the product library, alternated on one box: bench (500 steps, 50-step rollouts) and
# one FETCH_SIZE / WRITE_SIZE pass each.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ab_roll
mkdir -p $O
declare -A LIB=([base]=hockey-env_amd/hockey_amd/_lib/libhockey_hip.so [r3]=hockey-env_amd/hockey_amd/_lib/exp/libhockey_hip_roll_r3.so [r2]=hockey-env_amd/hockey_amd/_lib/exp/libhockey_hip_roll_r2.so)
B="--no-cpu-baseline --streams 0 --facade-steps 0 --c5-steps 0 --c4-steps 0"
for rep in 1 2; do
  for v in base r3 r2; do
    HK_LIB=${LIB[$v]} timeout -k 10 200 python3 bench.py $B --steps 500 --warmup 50 > $O/bench_${v}_$rep.log 2>&1
    echo "$v $rep $(grep -o '"value": [0-9.e+]*' $O/bench_${v}_$rep.log | head -2 | tr '\n' ' ')$(grep -o '"kernel_avg_ms": [0-9.e+]*' $O/bench_${v}_$rep.log)"
  done
done
for v in base r3 r2; do
  for C in FETCH_SIZE WRITE_SIZE; do
    rm -rf $O/pmc_${v}_$C
    HK_LIB=${LIB[$v]} timeout -k 10 300 rocprofv3 --pmc $C -d $O/pmc_${v}_$C -o run --output-format csv -- \
      python3 bench.py $B --rollout 0 --steps 40 --warmup 20 > $O/pmc_${v}_$C.log 2>&1
    echo "$v $C rc=$?"
  done
done
