#!/bin/bash
# r04h: changed-only state stores -- the GPU suite (bit-exact parity), HBM traffic of the single-step kernel
# (scripts/pmc.sh), the same counters for 50-step rollout launches (per step: does a launch re-fetch its code?),
# then the driver's bench command.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04h
mkdir -p $O
timeout -k 10 800 python -u -m pytest tests -m gpu -x -q --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
./scripts/pmc.sh > $O/pmc.log 2>&1 || { tail $O/pmc.log; exit 1; }
python scripts/pmc_reduce.py basic_65536 "profiles/r04h: scripts/pmc.sh" > $O/pmc_reduce.log && cp profiles/pmc_summary.json $O/ && grep -E "bytes_per_launch" $O/pmc_reduce.log
for C in FETCH_SIZE WRITE_SIZE; do
  timeout -s KILL 300 rocprofv3 --pmc $C -d $O/roll_$C -o run --output-format csv -- python3 bench.py --no-cpu-baseline --streams 0 --rollout 50 --steps 100 --warmup 5 --facade-steps 0 --c5-steps 0 --c4-steps 0 > $O/roll_$C.log 2>&1 || { tail $O/roll_$C.log; exit 1; }
done
python3 - $O <<'PY'
import csv, glob, sys
for c in ("FETCH_SIZE", "WRITE_SIZE"):
    for kern in ("step_kernel<false>", "step_kernel<true>"):
        v = [float(r["Counter_Value"]) for f in glob.glob(f"{sys.argv[1]}/roll_{c}/**/*counter_collection.csv", recursive=True)
             for r in csv.DictReader(open(f)) if kern in r["Kernel_Name"] and r["Counter_Name"] == c]
        if v:
            per = sum(v) / len(v) * 1024 / (50 if "true" in kern else 1)
            print(f"{c} {kern}: {len(v)} launches, {per / 65536:.1f} B per env-step (x2 for FETCH)")
PY
timeout -k 10 600 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1 || { tail -20 $O/driver_cmd.log; exit 1; }
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline > $O/bench_long.log 2>&1 || { tail -20 $O/bench_long.log; exit 1; }
python3 - $O <<'PY'
import json, sys
for f in ("driver_cmd.log", "bench_long.log"):
    d = [json.loads(l) for l in open(f"{sys.argv[1]}/{f}") if l.startswith("{")][-1]
    print(f, round(d["value"] / 1e6, 1), round(d["ms_per_step"], 4), round(d["roofline"]["kernel_avg_ms"], 4),
          {k: round(d[k]["value"] / 1e6, 3) for k in ("rollout", "streams", "facade_single_env", "c5_round", "c4_shard") if k in d and "value" in d[k]})
PY
