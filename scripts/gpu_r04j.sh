#!/bin/bash
# r04j: output rows staged through LDS (16-B stores of whole segments) -- FETCH/WRITE calibration of the
# output patterns, the GPU suite, the step kernel's PMC traffic and the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04j
mkdir -p $O
bash scripts/gpu_fetch_calib.sh > $O/fetch_calib.log 2>&1 || { tail $O/fetch_calib.log; exit 1; }
grep -E "obs_|info_|soa_dword " $O/fetch_calib.log
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
./scripts/pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python scripts/pmc_reduce.py basic_65536 "profiles/r04j: scripts/pmc.sh" > $O/pmc_reduce.log && cp profiles/pmc_summary.json $O/ && grep -E "bytes_per_launch" $O/pmc_reduce.log
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --c5-steps 0 --c4-steps 0 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline > $O/bench_long.log 2>&1 || { tail -20 $O/bench_long.log; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("driver_cmd.log", "bench_long.log"):
    d = [json.loads(l) for l in open(f"{sys.argv[1]}/{f}") if l.startswith("{")][-1]
    print(f, round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_avg_ms"], 4),
          {k: round(d[k]["value"] / 1e6, 3) for k in ("rollout", "streams", "facade_single_env") if k in d and "value" in d[k]})
PY
