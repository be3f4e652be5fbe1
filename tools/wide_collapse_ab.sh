#!/bin/bash
# 4-wide collapse A/B (PTSVGF_WIDE_COLLAPSE, capi.hip pack_wide): visits and bits per mode (tools/wide_collapse_ab.py),
# the wide-tree parity tests under MODES' last mode, then the bench alternating the modes on both views, REPS times.
# Logs: gpurun_out/wide_ab/. usage: MODES="0 2 1" REPS=2 bash tools/wide_collapse_ab.sh
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/wide_ab
mkdir -p $O
MODES=${MODES:-0 2 1}
for c in $MODES; do
  for v in default surface; do
    PTSVGF_WIDE_STATS=1 PTSVGF_WIDE_COLLAPSE=$c timeout -k 10 180 python -u tools/wide_collapse_ab.py 3840 2160 $v \
      >> $O/visits.log 2>&1 || exit 1
  done
done
grep -v amdgpu.ids $O/visits.log
last=${MODES##* }
PTSVGF_WIDE_COLLAPSE=$last timeout -k 10 400 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py \
  -k "wide_tree or far_eye or closest_tree or refill or bench_configuration" -x -q --timeout 300 --timeout-method thread \
  > $O/tests_mode$last.log 2>&1 || { tail -20 $O/tests_mode$last.log; exit 1; }
tail -2 $O/tests_mode$last.log
for rep in $(seq 1 ${REPS:-2}); do
  for c in $MODES; do
    for v in default surface; do
      PTSVGF_WIDE_COLLAPSE=$c timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-1080p \
        --no-extras --view $v > $O/bench_${v}_m${c}_r$rep.json 2> $O/bench_${v}_m${c}_r$rep.err || exit 1
      echo "rep $rep mode $c $v: $(python -c "import json,sys; d=json.load(open(sys.argv[1])); print(d['value'])" $O/bench_${v}_m${c}_r$rep.json)"
    done
  done
done
echo wide-ab-done
