#!/bin/bash
# Round evidence for the current kernel ($TAG, e.g. r02_v12): PMC HBM traffic (FETCH_SIZE / WRITE_SIZE
# passes -> profiles/pmc_summary.json), SQ instruction / stall counters (-> profiles/sq_summary.json), the
# bench line, and a rocprofv3 --kernel-trace --stats summary of the bench command.  All bench runs use the
# same steady-state workload (preroll 1000).  Outputs in gpurun_out/$TAG; copy into profiles/<round>/.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${TAG:-r02}
O=gpurun_out/$TAG
mkdir -p $O
./scripts/pmc.sh
python scripts/pmc_reduce.py basic_65536 "profiles/$TAG: scripts/pmc.sh (rocprofv3 --pmc FETCH_SIZE, --pmc WRITE_SIZE)" > $O/pmc_reduce.log
./scripts/sq.sh
python scripts/sq_reduce.py basic_65536 "profiles/$TAG: scripts/sq.sh (rocprofv3 --pmc, 2 SQ passes)" > $O/sq_counters.txt
cp profiles/pmc_summary.json profiles/sq_summary.json $O/
timeout -k 10 300 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log
rm -rf gpurun_out/prof
timeout -k 10 300 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --streams 0 --rollout 0 --facade-steps 0 --c5-steps 0 --c4-steps 0 > $O/prof_bench.log 2>&1
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find gpurun_out/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
tail -1 $O/prof_bench.log
head -4 $O/kernel_stats.csv
