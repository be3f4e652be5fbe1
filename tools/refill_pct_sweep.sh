#!/bin/bash
# 4K (K = 4) and surface-view frame rates for several lane-refill shares (trace_refill, percent of each list)
R="$GRAFT_REPO_ROOT"
for pct in ${PCTS:-65 75 85 95 75}; do
  timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --pt-uniform trace_refill=$pct > "$R/gpurun_out/rp.json" 2>/dev/null || exit $?
  timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --view surface --pt-uniform trace_refill=$pct > "$R/gpurun_out/rps.json" 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/rp.json').read()); s=json.loads(open('$R/gpurun_out/rps.json').read())
print('refill $pct %:', d['value'], 'surface', s['value'])"
done
