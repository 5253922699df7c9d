#!/bin/bash
# r04f: the facade and TD3 GPU tests after the facade trims and the fused learner at batch 256, the per-step kernel
# time over a long run of the bench workload (scripts/step_profile.py), then the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04f
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_facade.py tests/test_td3.py -m gpu -x -v --timeout 200 --timeout-method thread > $O/pytest.log 2>&1
rc=$?; tail -3 $O/pytest.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest.log | head -80; exit $rc; }
timeout -k 10 120 python -u scripts/step_profile.py 3000 > $O/step_profile.log 2>&1 || { tail -20 $O/step_profile.log; exit 1; }
cp gpurun_out/step_profile.json $O/
timeout -k 10 600 python -u bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
python - $O/driver_cmd.log <<'PY'
import json, sys
d = [json.loads(l) for l in open(sys.argv[1]) if l.startswith("{")][-1]
print({k: d[k] for k in ("value", "ms_per_step")}, d["roofline"]["kernel_avg_ms"])
for k in ("rollout", "streams", "facade_single_env", "c5_round", "c4_shard", "cpu_baseline"):
    v = d.get(k) or {}
    print(k, {x: v.get(x) for x in ("value", "collect_value", "update_s", "ms_per_step", "error")})
PY
bash scripts/gpu_fetch_calib.sh
