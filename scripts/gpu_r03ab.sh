#!/bin/bash
# r03ab: A/B of the TOI event changes (island build's far tests as a uniform loop over the pair table, the event
# pair's update without the broad-phase shortcut) against the committed head, three alternations; tail statistics
# with the event lanes; then the round's final validation and evidence (scripts/gpu_r03x.sh: full GPU suite,
# smoke, the driver's bench command, scripts/profile_round.sh).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03ab
mkdir -p $O
L=hockey-env_amd/hockey_amd/_lib
for i in 1 2 3; do
  for lib in libhockey_hip_base.so libhockey_hip.so; do
    HK_LIB=$L/$lib timeout -k 10 180 python bench.py --no-cpu-baseline --rollout 50 --streams 0 --facade-steps 0 \
      --c5-steps 0 --c4-steps 0 --steps 300 --warmup 200 > $O/ab_${lib}_$i.log 2>&1 || { tail -5 $O/ab_${lib}_$i.log; exit 1; }
    echo "$i $lib $(grep -o '"value": [0-9.e+]*\|"kernel_avg_ms": [0-9.e+]*' $O/ab_${lib}_$i.log | tr '\n' ' ')"
  done
done
HK_LIB=$L/libhockey_hip_timers.so timeout -k 10 240 python scripts/tail_stats.py 65536 30 > $O/tail_timers.log 2>&1 || { tail -5 $O/tail_timers.log; exit 1; }
sed -n 2,2p $O/tail_timers.log; sed -n 6,20p $O/tail_timers.log; tail -8 $O/tail_timers.log
bash scripts/gpu_r03x.sh
