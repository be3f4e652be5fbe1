#!/bin/bash
# One parametrised GPU session (replaces round 3's one-off tools/gpu_r03_g*.sh scripts, which are in git history).
# Usage (on the GPU box, e.g. gpurun -- bash tools/gpu_steps.sh STEP...), each STEP one quoted word list (split like a
# shell command line, so an argument with spaces is quoted inside it):
#   "tests [pytest args]"       GPU tests (default: every -m gpu test), log gpurun_out/<tag>_tests.log
#   "bench TAG [bench args]"    bench.py -> gpurun_out/TAG.json (+ .err)
#   "profile NAME"              tools/gpu_profile.sh NAME (env FIF, VIEW, PASSES as that script reads them)
#   "ab UNIFORM V0 V1 [...]"    tools/uniform_ab_views.sh (same-box A/B of a path-tracer uniform, both views)
#   "py [K=V ...] SCRIPT [args]" any python tool under tools/ (e.g. frame_shard_sim.py); leading K=V words are exported
#                               for that step only
# Every step runs under its own time limit (STEP_TIMEOUT, default 900 s) and the session stops at the first failure
# (no GPU step after a fault, abort, time limit or hang: the script exits with that step's status).
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-s$(date +%H%M%S)}
T=${STEP_TIMEOUT:-900}
n=0
for step in "$@"; do
  n=$((n + 1))
  eval "a=($step)"  # shell word splitting: quote an argument that holds spaces ("tests -k 'a or b'")
  kind=${a[0]}
  args=("${a[@]:1}")
  echo "[$(date +%H:%M:%S)] step $n: $step"
  case "$kind" in
    tests)
      [ ${#args[@]} -eq 0 ] && args=(tests -m gpu)
      timeout -k 10 "$T" python -u -m pytest "${args[@]}" -x -q --timeout 300 --timeout-method thread \
        > "gpurun_out/${TAG}_tests$n.log" 2>&1
      rc=$?; tail -3 "gpurun_out/${TAG}_tests$n.log" ;;
    bench)
      out=${args[0]}; rest=("${args[@]:1}")
      timeout -k 10 "$T" python bench.py "${rest[@]}" > "gpurun_out/$out.json" 2> "gpurun_out/$out.err"
      rc=$?; tail -c 400 "gpurun_out/$out.json" ;;
    profile)
      timeout -k 10 "$T" bash tools/gpu_profile.sh "${args[@]}"; rc=$? ;;
    ab)
      timeout -k 10 "$T" bash tools/uniform_ab_views.sh "${args[@]}"; rc=$? ;;
    py)
      envs=()
      while [[ ${#args[@]} -gt 0 && "${args[0]}" == *=* ]]; do envs+=("${args[0]}"); args=("${args[@]:1}"); done
      timeout -k 10 "$T" env "${envs[@]}" python -u "tools/${args[0]}" "${args[@]:1}" > "gpurun_out/${TAG}_py$n.log" 2>&1
      rc=$?; tail -20 "gpurun_out/${TAG}_py$n.log" ;;
    *) echo "unknown step kind '$kind'"; exit 2 ;;
  esac
  echo "[$(date +%H:%M:%S)] step $n rc=$rc"
  [ $rc -eq 0 ] || exit $rc
done
