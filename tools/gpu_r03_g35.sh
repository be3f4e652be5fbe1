#!/bin/bash
# A/B: wf_shade compiled for 6 / 8 waves per SIMD (93 VGPRs = 5 by default), default and surface views.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT"
for L in lib lib_exp/shade6 lib_exp/shade8 lib lib_exp/shade6 lib_exp/shade8; do
  PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras > "$R/gpurun_out/ab_d.json" 2>/dev/null || exit $?
  PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --view surface > "$R/gpurun_out/ab_s.json" 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('$R/gpurun_out/ab_d.json').read()); s=json.loads(open('$R/gpurun_out/ab_s.json').read())
print('$L default', d['value'], 'surface', s['value'], 'shade ms', d['passes_ms'].get('pathtrace'))"
done
