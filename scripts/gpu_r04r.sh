#!/bin/bash
# r04r: the driver's bench command at this head (c5_round with the current learner).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04r
mkdir -p $O
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
python3 - $O <<'PY'
import json, sys
d = [json.loads(l) for l in open(f"{sys.argv[1]}/driver_cmd.log") if l.startswith("{")][-1]
print(round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), d["roofline"]["counters_stale"],
      {k: round(d[k]["value"] / 1e6, 4) for k in ("rollout", "streams", "facade_single_env", "c5_round", "c4_shard", "cpu_baseline") if k in d and "value" in d[k]},
      d["c5_round"].get("update_s"))
PY
