#!/bin/bash
# r04ab: the stage-1 learning pin on 20 arenas with the round's final fused learner (soft_update folded into Adam,
# the actor's dW2 in 256-sample chunks): eight new seeds 436-443 side by side, as a check that learning still works.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04ab
mkdir -p $O
pids=""
for seed in 436 437 438 439 440 441 442 443; do
  OMP_NUM_THREADS=2 timeout -k 10 1050 python -u scripts/td3_stage1_pin.py --arenas 20 --episodes 10000 --seed $seed \
    --learner fused --out $O/stage1_pin_n20_fused_s$seed.json > $O/pin_n20_fused_s$seed.log 2>&1 &
  pids="$pids $!"
done
for p in $pids; do wait $p; done
for seed in 420 421 422 423; do echo "seed $seed: $(tail -1 $O/pin_n20_fused_s$seed.log | cut -c1-300)"; done
exit 0
