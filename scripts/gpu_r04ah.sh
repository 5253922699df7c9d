#!/bin/bash
# r04ah: the round's final head -- the whole GPU suite, __graft_entry__.smoke() and the driver's bench command
# (the step library is r04u's; the learner changed since).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04ah
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
python3 - $O <<'PY'
import json, sys
d = [json.loads(l) for l in open(f"{sys.argv[1]}/driver_cmd.log") if l.startswith("{")][-1]
print(round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), d["roofline"]["counters_stale"],
      {k: round(d[k]["value"] / 1e6, 4) for k in ("rollout", "streams", "facade_single_env", "c5_round", "c4_shard", "cpu_baseline") if k in d and "value" in d[k]},
      d["c5_round"].get("update_s"))
PY
