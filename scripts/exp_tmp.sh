set -euo pipefail
export HK_TRACE=1 HKH_LIB=hockey-env_amd/hockey_amd/_lib/libhockey_hostcheck_trace.so
for v in A B; do
  HK_LIB=hockey-env_amd/hockey_amd/_lib/libhockey_hip_trace_$v.so timeout -k 10 200 python scripts/debug_lockstep.py 0 1 1024 300 strong > gpurun_out/dbg_$v.log 2>&1
  echo "$v: $(grep -E '^step|no div' gpurun_out/dbg_$v.log | head -2 | tr '\n' ' ')"
done
