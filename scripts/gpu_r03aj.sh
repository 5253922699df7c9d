#!/bin/bash
# r03aj: the stage-1 learning pin on 20 arenas (episodes end at done), 10 000 episodes, seeds 424-427 side by side
# (four more seeds next to r03ae's 420-423).  Each run writes its curve after every
# evaluation, so a run stopped by its time limit still leaves the episodes it finished.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03aj
mkdir -p $O
pids=""
for seed in 424 425 426 427; do
  timeout -k 10 1050 python -u scripts/td3_stage1_pin.py --arenas 20 --episodes 10000 --seed $seed \
    --out $O/stage1_pin_n20_s$seed.json > $O/pin_n20_s$seed.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for seed in 424 425 426 427; do echo "seed $seed: $(tail -1 $O/pin_n20_s$seed.log | cut -c1-300)"; done
exit $rc
