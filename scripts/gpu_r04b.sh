#!/bin/bash
# r04b: the stage-1 learning pin with ONE arena per run -- the reference's own round structure (one episode, then
# 32 updates) -- for the eight seeds of the r03 20-arena study, side by side (does the batched
# round structure explain the plateaued seeds?).  Curves are written after every evaluation.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04b
mkdir -p $O
pids=""
for seed in 420 421 422 423 424 425 426 427; do
  OMP_NUM_THREADS=2 timeout -k 10 1080 python -u scripts/td3_stage1_pin.py --arenas 1 --episodes 10000 --seed $seed \
    --out $O/stage1_pin_n1_s$seed.json > $O/pin_n1_s$seed.log 2>&1 &
  pids="$pids $!"
done
rc=0
for p in $pids; do wait $p || rc=$?; done
for seed in 420 421 422 423 424 425 426 427; do echo "seed $seed: $(tail -1 $O/pin_n1_s$seed.log | cut -c1-300)"; done
exit 0
