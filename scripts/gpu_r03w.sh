#!/bin/bash
# r03w: the stage-1 learning pin on 4 arenas (episodes end at done), 10 000 episodes, four seeds run side by side
# (seeds 424-427: four more for the seed-to-seed spread next to r03r's 420-423).  Each run writes its curve after every
# evaluation, so a run stopped by its time limit still leaves the episodes it finished.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03w
mkdir -p $O
pids=""
for seed in 424 425 426 427; do
  timeout -k 10 1050 python -u scripts/td3_stage1_pin.py --arenas 4 --episodes 10000 --seed $seed \
    --out $O/stage1_pin_n4_s$seed.json > $O/pin_n4_s$seed.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for seed in 424 425 426 427; do echo "seed $seed: $(tail -1 $O/pin_n4_s$seed.log | cut -c1-300)"; done
exit $rc
