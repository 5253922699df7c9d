#!/bin/bash
# One A/B measurement of the current step library (r06): the GPU suite (optional), the driver's bench command,
# a 500-step bench, and per-wave tail statistics from the diagnostics build.  Outputs in gpurun_out/<tag>.
#   scripts/gpu_ab.sh <tag> [tests]
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { echo "FAILED: $1 (rc $2)"; exit "$2"; }
if [ "${2:-}" = "tests" ]; then
  timeout -k 10 900 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > "$O/pytest_gpu.log" 2>&1 \
    || { grep -B5 -A30 "FAILED\|Error" "$O/pytest_gpu.log" | head -60; fail pytest $?; }
  tail -1 "$O/pytest_gpu.log"
fi
timeout -k 10 300 python3 bench.py --gpus 1 --steps 20 --warmup 5 --facade-steps 0 --c5-steps 0 --c4-steps 0 \
  --no-cpu-baseline --streams 0 --rollout 0 > "$O/driver_cmd.log" 2>&1 || fail driver $?
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 \
  --no-cpu-baseline --streams 0 > "$O/bench_long.log" 2>&1 || fail bench_long $?
python3 - "$O" <<'PY'
import json, sys
for f in ("driver_cmd.log", "bench_long.log"):
    d = json.loads([l for l in open(f"{sys.argv[1]}/{f}") if l.startswith("{")][-1])
    print(f, round(d["value"] / 1e6, 2), "M  kernel", round(d["roofline"]["kernel_avg_ms"], 4), "ms",
          "rollout", round(d.get("rollout", {}).get("value", 0) / 1e6, 1))
PY
if [ -f hockey-env_amd/hockey_amd/_lib/libhockey_hip_timers.so ]; then
  timeout -k 10 300 python scripts/tail_stats.py 65536 30 > "$O/tail_stats.txt" 2>&1 || fail tail_stats $?
  grep "max-per-step\|per iteration\|launch bound" "$O/tail_stats.txt"
fi
