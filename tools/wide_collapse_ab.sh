#!/bin/bash
# Tree-build A/B (VAR = PTSVGF_WIDE_COLLAPSE by default, capi.hip pack_wide; or PTSVGF_TREELET, treelet_optimize):
# visits and bits per value (tools/wide_collapse_ab.py), the wide-tree parity tests under MODES' last value, then the
# bench alternating the values on both views, REPS times. Logs: gpurun_out/${TAG:-wide_ab}/.
# usage: MODES="0 2 1" REPS=2 bash tools/wide_collapse_ab.sh; VAR=PTSVGF_TREELET MODES="0 1" TAG=treelet_ab bash ...
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-wide_ab}
VAR=${VAR:-PTSVGF_WIDE_COLLAPSE}
mkdir -p $O
MODES=${MODES:-0 2 1}
for c in $MODES; do
  for v in default surface; do
    PTSVGF_WIDE_STATS=1 env $VAR=$c timeout -k 10 180 python -u tools/wide_collapse_ab.py 3840 2160 $v \
      >> $O/visits.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/visits.log
last=${MODES##* }
env $VAR=$last timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  -k "wide_tree or far_eye or closest_tree or refill or bench_configuration" -x -q --timeout 300 --timeout-method thread \
  > $O/tests_mode$last.log 2>&1 || { tail -20 $O/tests_mode$last.log; exit 1; }
tail -2 $O/tests_mode$last.log
for rep in $(seq 1 ${REPS:-2}); do
  for c in $MODES; do
    for v in default surface; do
      env $VAR=$c timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-1080p \
        --no-extras --view $v > $O/bench_${v}_m${c}_r$rep.json 2> $O/bench_${v}_m${c}_r$rep.err || exit 1
      echo "rep $rep mode $c $v: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'])" $O/bench_${v}_m${c}_r$rep.json)"
    done
  done
done
echo wide-ab-done
