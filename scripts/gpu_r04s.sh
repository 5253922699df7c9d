#!/bin/bash
# r04s: the learner's gemm256 alone at critic_step's grid (scripts/micro/learner_gemm_bench.hip).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
/opt/rocm/bin/hipcc --offload-arch=gfx950 -O3 -std=c++17 -o /tmp/lgb scripts/micro/learner_gemm_bench.hip || exit 1
timeout -k 10 120 /tmp/lgb
