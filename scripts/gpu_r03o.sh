#!/bin/bash
# r03o: puck-rotation shortcut in the position solver -- GPU parity (lockstep / rollout / facade subset) and an
# interleaved A/B against the previous library (libhockey_hip_prev.so, built from the commit before).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r03o
mkdir -p $O
timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_facade.py -x -q --timeout 200 --timeout-method thread -k "lockstep or rollout or large_island or facade or g1 or g2 or begin_contact or c1 or hockey_one or set_state or mode_switch or partial" > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || exit $rc
B="--steps 300 --warmup 50 --facade-steps 0 --c5-steps 0 --c4-steps 0 --no-cpu-baseline --streams 0"
L=hockey-env_amd/hockey_amd/_lib
for k in 1 2; do
  timeout -k 10 120 python3 bench.py $B > $O/bench_new_$k.log 2>&1 || exit 1
  HK_LIB=$L/libhockey_hip_prev.so timeout -k 10 120 python3 bench.py $B > $O/bench_prev_$k.log 2>&1 || exit 1
  python3 -c "
import json
for t in ('new','prev'):
    d=json.loads(open('$O/bench_'+t+'_$k.log').read().strip().splitlines()[-1]); print(t, round(d['value']/1e6,1), 'M', round(d['roofline']['kernel_avg_ms'],4), 'ms', 'rollout', round(d['rollout']['value']/1e6,1))"
done
# timing probe of the one-arena stage-1 run (the reference's sequential loop shape): 400 episodes, 2 evaluations
timeout -k 10 300 python -u scripts/td3_stage1_pin.py --arenas 1 --episodes 400 --out $O/stage1_n1_probe.json > $O/stage1_n1_probe.log 2>&1 || exit 1
tail -3 $O/stage1_n1_probe.log | cut -c1-300
