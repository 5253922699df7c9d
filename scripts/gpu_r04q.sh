#!/bin/bash
# r04q: A/B of the lone-lane drains on the facade (same box): HK_LIB = the previous head's library vs this one,
# alternated twice.
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
O=gpurun_out/r04q
mkdir -p $O
for r in 1 2; do
  HK_LIB=$PWD/hockey-env_amd/hockey_amd/_lib/libhockey_hip_base.so timeout -k 10 300 python -u scripts/facade_profile.py 5000 > $O/base_$r.log 2>&1 || { tail $O/base_$r.log; exit 1; }
  echo "base $r $(tail -1 $O/base_$r.log)"
  timeout -k 10 300 python -u scripts/facade_profile.py 5000 > $O/lone_$r.log 2>&1 || { tail $O/lone_$r.log; exit 1; }
  echo "lone $r $(tail -1 $O/lone_$r.log)"
done
