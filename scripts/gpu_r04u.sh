#!/bin/bash
# r04u: round evidence at the final head -- the GPU suite, __graft_entry__.smoke(), then scripts/profile_round.sh (PMC
# and SQ counter passes stamped with the library hash, the driver's bench command, a 500-step bench, rocprofv3
# kernel stats of the bench command, per-wave tail statistics).  Stops at the first failure.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04u
mkdir -p $O
export HK_PIN_OUT=$O/checkpoint_pins.json
timeout -k 10 800 python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread > $O/pytest_gpu.log 2>&1
rc=$?; tail -2 $O/pytest_gpu.log; [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" $O/pytest_gpu.log | head -80; exit $rc; }
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > $O/smoke.log 2>&1 || { tail -5 $O/smoke.log; exit 1; }
tail -1 $O/smoke.log
TAG=r04u ./scripts/profile_round.sh
