#!/bin/bash
# The one GPU launcher (replaces the per-call scripts/gpu_r0*.sh of rounds 1-4; they are in git history).
#   scripts/gpu_job.sh <job> <tag> [args...]      outputs under gpurun_out/<tag>
# Jobs:
#   round    the GPU suite, __graft_entry__.smoke(), then scripts/profile_round.sh (PMC / SQ counter passes, the
#            driver's bench command, a 500-step bench, rocprofv3 kernel stats, per-wave tail statistics)
#   tests    the GPU suite only ([pytest -k expression])
#   bench    bench.py with the given arguments, then rocprofv3 --kernel-trace --stats of the same command
#   noise    scripts/noise_study.py: <protocol> <seed | noise:seed>... -> every noise x seed (or the named pairs)
#            side by side, one process each; protocol sp_per takes p<0|1>s<0|1>:seed (PER, self-play switches)
#   learner  scripts/learner_profile.py + rocprofv3 kernel stats of it
# Every GPU step runs under its own time limit; the script stops at the first failure (no retries).
set -u
cd "${GRAFT_REPO_ROOT:-$(dirname "$0")/..}"
export TMPDIR=/tmp
JOB=${1:?job}; TAG=${2:?tag}; shift 2
O=gpurun_out/$TAG
mkdir -p "$O"
fail() { echo "FAILED: $1 (rc $2)"; exit "$2"; }

gpu_tests() {
  local k=()
  [ $# -gt 0 ] && k=(-k "$1")
  timeout -k 10 ${T_TEST:-900} python -u -m pytest tests -m gpu -x -v --timeout 300 --timeout-method thread "${k[@]}" \
    > "$O/pytest_gpu.log" 2>&1
  local rc=$?
  tail -2 "$O/pytest_gpu.log"
  [ $rc -eq 0 ] || { grep -B5 -A40 "FAILED\|Error" "$O/pytest_gpu.log" | head -80; fail pytest $rc; }
}

case "$JOB" in
  round)
    export HK_PIN_OUT=$O/checkpoint_pins.json
    gpu_tests
    timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > "$O/smoke.log" 2>&1 || fail smoke $?
    tail -1 "$O/smoke.log"
    TAG=$TAG ./scripts/profile_round.sh || fail profile_round $?
    ;;
  tests)
    gpu_tests "$@"
    ;;
  bench)
    timeout -k 10 ${T_BENCH:-400} python3 bench.py "$@" > "$O/bench.log" 2>&1 || { tail -20 "$O/bench.log"; fail bench $?; }
    tail -c 400 "$O/bench.log"
    if [ "${PROFILE:-1}" = "1" ]; then
      rm -rf "$O/prof"
      timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/prof" -o run --output-format csv -- \
        python3 bench.py --no-cpu-baseline "$@" > "$O/prof_bench.log" 2>&1 || fail rocprof $?
      find "$O/prof" -name "*kernel_stats.csv" -exec cp {} "$O/kernel_stats.csv" \;
      head -6 "$O/kernel_stats.csv"
    fi
    ;;
  noise)
    PROTO=${1:?protocol}; shift
    pids=""
    runs=""
    for tok in "$@"; do
      case "$tok" in
        *:*) runs="$runs $tok" ;;
        *) for noise in gaussian ou pink uniform; do runs="$runs $noise:$tok"; done ;;
      esac
    done
    for r in $runs; do
      noise=${r%%:*}; seed=${r##*:}
      extra=""
      case "$noise" in  # sp_per: the token names the switches, p<0|1>s<0|1> (prioritized replay, self-play)
        p?s?) extra="--per ${noise:1:1} --sp ${noise:3:1}"; noise=ou ;;
      esac
      OMP_NUM_THREADS=1 timeout -k 10 ${T_RUN:-1080} python -u scripts/noise_study.py --protocol "$PROTO" \
        --noise $noise --seed $seed $extra --out "$O" > "$O/${PROTO}_${r/:/_s}.log" 2>&1 &
      pids="$pids $!"
    done
    rc=0
    for p in $pids; do wait $p || rc=$?; done
    for f in "$O"/${PROTO}_*.log; do echo "$(basename $f): $(tail -1 $f | cut -c1-240)"; done
    exit $rc
    ;;
  learner)
    timeout -k 10 400 python -u scripts/learner_profile.py "$@" > "$O/learner_profile.log" 2>&1 || fail learner $?
    tail -5 "$O/learner_profile.log"
    rm -rf "$O/lprof"
    timeout -k 10 400 rocprofv3 --kernel-trace --stats -d "$O/lprof" -o run --output-format csv -- \
      python3 scripts/learner_profile.py "$@" > "$O/learner_prof.log" 2>&1 || fail rocprof $?
    find "$O/lprof" -name "*kernel_stats.csv" -exec cp {} "$O/learner_kernel_stats.csv" \;
    head -12 "$O/learner_kernel_stats.csv"
    ;;
  *)
    fail "unknown job $JOB" 2
    ;;
esac
