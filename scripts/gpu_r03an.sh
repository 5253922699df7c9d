#!/bin/bash
# r03an: further build variants against the product build (iterative-ilp): w1 -fno-unroll-loops, w2 kernel-argument
# preloading (16 SGPRs), w3 the AMDGPU register-pressure trackers in scheduling, w4 no post-RA scheduling; two alternations.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03an
mkdir -p $O
L=hockey-env_amd/hockey_amd/_lib
for i in 1 2; do
  for lib in libhockey_hip.so libhockey_hip_w1.so libhockey_hip_w2.so libhockey_hip_w3.so libhockey_hip_w4.so; do
    HK_LIB=$L/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --rollout 50 --streams 0 --facade-steps 0 \
      --c5-steps 0 --c4-steps 0 --steps 300 --warmup 200 > $O/ab_${lib}_$i.log 2>&1 || { tail -5 $O/ab_${lib}_$i.log; exit 1; }
    echo "$i $lib $(grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*' $O/ab_${lib}_$i.log | tr '\n' ' ')"
  done
done
