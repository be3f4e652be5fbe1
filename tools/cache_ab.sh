#!/bin/bash
# Shadow occluder cache A/B (uniform shadow_cache: 0 off, 1 bounce 0, 3 bounces 0 and 1) on one library, alternating,
# 4K K = 4 default and surface views, then one frame at a time. usage: REPS=2 bash tools/cache_ab.sh "0 1 3"
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/cache_ab"
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-2}"); do
  for c in $1; do
    for V in default surface serial; do
      A="--view $V"
      [ "$V" = serial ] && A="--frames-in-flight 1"
      N=c${c}_${V}_$rep
      timeout -k 10 300 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras $A --pt-uniform shadow_cache=$c \
        > "$OUT/$N.json" 2> "$OUT/$N.err" || { echo "$N failed"; exit 1; }
      python3 -c "
import json; d = json.loads(open('$OUT/$N.json').read()); pt = d['path_tracer']
print('$N', d['value'], 'shadow visits', pt['visits_per_frame']['shadow_visits'], pt['shadow_split'], 'pt_ms', d['passes_ms']['pathtrace'])"
    done
  done
done
