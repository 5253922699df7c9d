#!/bin/bash
# One-off A/B (r05): hkl_adam variants (the 16-lanes-per-element reduction of the small many-chunk
# segments; then 32 slab loads in flight per thread) in the product libhockey_learner.so against the previous library (exp/libhockey_learner_base.so): parameters
# after 12 fused updates (bitwise, uniform and prioritized ring), learner_profile.py alternated, rocprofv3 stats.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/../..}"
export TMPDIR=/tmp
O=gpurun_out/ab_adam
mkdir -p $O
declare -A LIB=([base]=hockey-env_amd/hockey_amd/_lib/exp/libhockey_learner_base.so [new]=hockey-env_amd/hockey_amd/_lib/libhockey_learner.so)
for v in base new; do
  HK_LEARNER_LIB=${LIB[$v]} timeout -k 10 200 python3 scripts/experiments/learner_params_dump.py $O/params_$v.pt 16384 12
  HK_LEARNER_LIB=${LIB[$v]} timeout -k 10 200 python3 scripts/experiments/learner_params_dump.py $O/params_per_$v.pt 16384 12 per
done
python3 - <<'PY'
import torch
for tag in ("", "per_"):
    a, b = (torch.load(f"gpurun_out/ab_adam/params_{tag}{v}.pt", weights_only=True) for v in ("base", "new"))
    print(tag or "uniform", {k: bool(torch.equal(a[k], b[k])) for k in a})
PY
for rep in 1 2; do
  for v in base new; do
    HK_LEARNER_LIB=${LIB[$v]} timeout -k 10 300 python3 scripts/learner_profile.py 16384 300 fused > $O/profile_${v}_$rep.log 2>&1
    echo "$v $rep $(grep -o '"fused_ms_per_update_[a-z]*": [0-9.]*' $O/profile_${v}_$rep.log | tr '\n' ' ')"
  done
done
for v in base new; do
  rm -rf $O/prof_$v
  HK_LEARNER_LIB=${LIB[$v]} timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof_$v -o run --output-format csv -- \
    python3 scripts/learner_profile.py 16384 200 fused > $O/prof_$v.log 2>&1
  find $O/prof_$v -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats_$v.csv \;
  grep -i "adam\|critic_step" $O/kernel_stats_$v.csv | cut -d, -f1-4
done
