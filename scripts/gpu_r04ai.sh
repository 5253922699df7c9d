#!/bin/bash
# r04ai: actor_step's Q1 head back on the MFMA tile (critic_step keeps the VALU heads):
# the learner GPU tests, the update cost (scripts/learner_profile.py), its rocprofv3 kernel stats, and the
# driver's bench command (c5_round).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04ai
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests/test_gpu_learner.py tests/test_td3.py -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_learner.log 2>&1
rc=$?; tail -2 $O/pytest_learner.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_learner.log | head -80; exit $rc; }
# A/B on this box: ab_prev/ holds the previous learner (host module + library, commit 35c963d), alternated twice
for r in 1 2; do
  HK_PKG_DIR=$PWD/ab_prev timeout -k 10 300 python -u scripts/learner_profile.py 16384 300 fused > $O/ab_prev_$r.log 2>&1 || { tail -20 $O/ab_prev_$r.log; exit 1; }
  echo "prev $r $(tail -1 $O/ab_prev_$r.log | cut -c1-400)"
  timeout -k 10 300 python -u scripts/learner_profile.py 16384 300 fused > $O/ab_new_$r.log 2>&1 || { tail -20 $O/ab_new_$r.log; exit 1; }
  echo "new $r $(tail -1 $O/ab_new_$r.log | cut -c1-400)"
done
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d $O/prof -o run --output-format csv -- python3 scripts/learner_profile.py 16384 100 fused > $O/prof.log 2>&1 || { tail -20 $O/prof.log; exit 1; }
find $O/prof -name "*kernel_stats.csv" -exec cp {} $O/learner_kernel_stats.csv \;
head -9 $O/learner_kernel_stats.csv | cut -d, -f1-4
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
python3 - $O <<'PY'
import json, sys
d = [json.loads(l) for l in open(f"{sys.argv[1]}/driver_cmd.log") if l.startswith("{")][-1]
print(round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), d["roofline"]["counters_stale"],
      {k: round(d[k]["value"] / 1e6, 4) for k in ("rollout", "streams", "facade_single_env", "c5_round", "c4_shard", "cpu_baseline") if k in d and "value" in d[k]},
      d["c5_round"].get("update_s"))
PY
