#!/bin/bash
# r04t: FETCH_SIZE / WRITE_SIZE of hk::step_kernel at three arena counts (same bench workload), so that the
# per-launch traffic splits into a part that scales with the arenas and a fixed part per launch (instruction and
# scene fetches into each XCD's L2).  Counters only, one counter per pass.  Reduce with scripts/pmc_fixed_cost.py.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04t
mkdir -p $O
for N in 4096 16384 65536; do
  for C in FETCH_SIZE WRITE_SIZE; do
    timeout -s KILL 300 rocprofv3 --pmc $C -d $O/n${N}_$C -o run --output-format csv -- \
      python3 bench.py --arenas $N --no-cpu-baseline --rollout 0 --streams 0 --facade-steps 0 --c5-steps 0 \
      --c4-steps 0 --steps 40 --warmup 20 > $O/n${N}_$C.log 2>&1
    rc=$?; echo "N=$N $C rc=$rc"; [ $rc -eq 0 ] || { tail -20 $O/n${N}_$C.log; exit $rc; }
  done
done
