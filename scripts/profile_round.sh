#!/bin/bash
# Round evidence for the current kernel ($TAG, e.g. r03): PMC HBM traffic (FETCH_SIZE / WRITE_SIZE passes ->
# profiles/pmc_summary.json), SQ instruction / stall counters (-> profiles/sq_summary.json), both stamped with
# the library's source hash; the driver's bench command; a rocprofv3 --kernel-trace --stats summary of the
# bench command; per-wave tail statistics from the diagnostics build.  Outputs in gpurun_out/$TAG; copy into
# profiles/<round>/.  Every GPU step has its own time limit and the script stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r03}
O=gpurun_out/$TAG
mkdir -p $O
./scripts/pmc.sh
python scripts/pmc_reduce.py basic_65536 "profiles/$TAG: scripts/pmc.sh (rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE)" > $O/pmc_reduce.log
./scripts/sq.sh
python scripts/sq_reduce.py basic_65536 "profiles/$TAG: scripts/sq.sh (rocprofv3 --pmc, 2 SQ passes)" > $O/sq_counters.txt
cp profiles/pmc_summary.json profiles/sq_summary.json $O/
timeout -k 10 400 python3 bench.py --gpus 1 --steps 20 --warmup 5 > $O/driver_cmd.log 2>&1
tail -c 300 $O/driver_cmd.log
timeout -k 10 300 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline > $O/bench_long.log 2>&1
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --streams 0 --rollout 0 --facade-steps 0 --c5-steps 0 --c4-steps 0 > $O/prof_bench.log 2>&1
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
tail -1 $O/prof_bench.log | cut -c1-200
head -4 $O/kernel_stats.csv
if [ -f hockey-env_amd/hockey_amd/_lib/libhockey_hip_timers.so ]; then
  timeout -k 10 300 python scripts/tail_stats.py 65536 30 > $O/tail_stats.txt 2>&1
  head -3 $O/tail_stats.txt
fi
