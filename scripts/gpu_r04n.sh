#!/bin/bash
# r04n: more seeds of the 20-arena stage-1 pin with the fused learner (424-435, twelve side by side), for the seed
# distribution next to r03's eager-learner study.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04n
mkdir -p $O
pids=""
for seed in 424 425 426 427 428 429 430 431 432 433 434 435; do
  OMP_NUM_THREADS=2 timeout -k 10 1050 python -u scripts/td3_stage1_pin.py --arenas 20 --episodes 10000 --seed $seed \
    --learner fused --out $O/stage1_pin_n20_fused_s$seed.json > $O/pin_n20_fused_s$seed.log 2>&1 &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
for seed in 424 425 426 427 428 429 430 431 432 433 434 435; do echo "seed $seed: $(tail -1 $O/pin_n20_fused_s$seed.log | cut -c1-300)"; done
exit 0
