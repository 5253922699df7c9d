#!/bin/bash
# Round-end evidence for one kernel version ($V): GPU parity tests, smoke, PMC HBM traffic (FETCH_SIZE /
# WRITE_SIZE passes -> profiles/pmc_summary.json, read by bench.py), SQ instruction/stall counters, the
# full bench line (with the CPU baseline) and a rocprofv3 --kernel-trace --stats summary of the bench.
# Outputs land in gpurun_out/; copy the ones to keep into profiles/r01/.  Stops at the first failure.
set -euo pipefail
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
V=${V:-v}
O=gpurun_out/$V
mkdir -p $O
timeout -k 10 600 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1 || { tail -30 $O/pytest_gpu.log; exit 1; }
tail -1 $O/pytest_gpu.log
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1
tail -1 $O/smoke.log
./scripts/pmc.sh
python scripts/pmc_reduce.py basic_65536 > $O/pmc_reduce.log
cp profiles/pmc_summary.json $O/
./scripts/sq.sh
python scripts/sq_reduce.py > $O/sq_counters.txt
timeout -k 10 600 python bench.py > $O/bench.log 2>&1
tail -1 $O/bench.log
rm -rf gpurun_out/prof
timeout -k 10 600 rocprofv3 --kernel-trace --stats -d gpurun_out/prof -o run --output-format csv -- \
  python3 bench.py --no-cpu-baseline --streams 0 > $O/prof_bench.log 2>&1
find gpurun_out/prof -name "*kernel_stats.csv" -exec cp {} $O/kernel_stats.csv \;
find gpurun_out/prof -name "*kernel_trace.csv" -exec cp {} $O/kernel_trace.csv \;
head -3 $O/kernel_stats.csv
