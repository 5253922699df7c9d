#!/bin/bash
# Same-box A/B of step libraries (r06): the 500-step bench (no side legs) for each library given, alternated
# REPS times, so box-to-box spread does not enter the comparison.  Outputs in gpurun_out/<tag>/libab.txt.
#   scripts/gpu_libab.sh <tag> <reps> <lib.so>...
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
TAG=${1:?tag}; REPS=${2:?reps}; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
for r in $(seq 1 "$REPS"); do
  for lib in "$@"; do
    HK_LIB=$lib timeout -k 10 200 python3 bench.py --steps 500 --warmup 100 --facade-steps 0 --c5-steps 0 --c4-steps 0 \
      --no-cpu-baseline --streams 0 --rollout 0 > "$O/ab.log" 2>&1 || { tail -5 "$O/ab.log"; echo "FAILED $lib"; exit 1; }
    python3 - "$O/ab.log" "$lib" "$r" <<'PY' | tee -a "$O/libab.txt"
import json, sys
d = json.loads([l for l in open(sys.argv[1]) if l.startswith("{")][-1])
print(f"rep {sys.argv[3]} {sys.argv[2].split('/')[-1]:28s} {d['value'] / 1e6:7.2f} M  kernel {d['roofline']['kernel_avg_ms']:.4f} ms")
PY
  done
done
