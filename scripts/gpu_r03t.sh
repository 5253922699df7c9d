#!/bin/bash
# r03t: round evidence at the step-start-prefetch kernel (scripts/profile_round.sh: PMC traffic, SQ counters at
# the library hash, the driver's bench command, a 500-step line, rocprofv3 kernel stats, tail statistics).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
TAG=r03t ./scripts/profile_round.sh
