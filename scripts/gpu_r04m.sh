#!/bin/bash
# r04m: the stage-1 learning pin on 20 arenas with the fused MFMA learner (now train()'s default on the GPU), seeds
# 420-423 side by side -- the r03 eager-learner study (scripts/gpu_r03ae.sh) repeated on the new update path.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04m
mkdir -p $O
pids=""
for seed in 420 421 422 423; do
  OMP_NUM_THREADS=4 timeout -k 10 1050 python -u scripts/td3_stage1_pin.py --arenas 20 --episodes 10000 --seed $seed \
    --learner fused --out $O/stage1_pin_n20_fused_s$seed.json > $O/pin_n20_fused_s$seed.log 2>&1 &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
for seed in 420 421 422 423; do echo "seed $seed: $(tail -1 $O/pin_n20_fused_s$seed.log | cut -c1-300)"; done
exit 0
