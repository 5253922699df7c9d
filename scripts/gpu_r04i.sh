#!/bin/bash
# r04i: the one-contact position family -- GPU suite (bit-exact parity), the driver's bench command, a 500-step
# bench and per-wave tail statistics (diagnostics build).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/${TAG:-r04i}
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 --c5-steps 0 --c4-steps 0 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline > $O/bench_long.log 2>&1 || { tail -20 $O/bench_long.log; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("driver_cmd.log", "bench_long.log"):
    d = [json.loads(l) for l in open(f"{sys.argv[1]}/{f}") if l.startswith("{")][-1]
    print(f, round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_avg_ms"], 4),
          {k: round(d[k]["value"] / 1e6, 3) for k in ("rollout", "streams", "facade_single_env") if k in d and "value" in d[k]})
PY
timeout -k 10 300 python scripts/tail_stats.py 65536 30 > $O/tail_stats.txt 2>&1 || { tail $O/tail_stats.txt; exit 1; }
sed -n 2,2p $O/tail_stats.txt; sed -n 7,20p $O/tail_stats.txt
