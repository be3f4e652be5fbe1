#!/bin/bash
# Same-box A/B of in-tree library builds on the headline configuration (4K, K = 4) and the surface view, alternating
# the libraries REPS times so drift hits every variant alike. Libraries are dirs under path-tracing-svgf_amd/ (lib,
# lib_exp/<name> from tools/exp_build.sh). Extra bench args via BENCH_ARGS. Prints one line per run.
# usage: REPS=2 bash tools/ab_libs.sh lib lib_exp/a lib_exp/b
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/ab_libs"
mkdir -p "$OUT"
for rep in $(seq 1 "${REPS:-2}"); do
  for L in "$@"; do
    for V in ${VIEWS:-default surface}; do
      N=$(echo "$L" | tr '/' '_')_${V}_$rep
      PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 300 python3 "$R/bench.py" --no-cpu-baseline --no-1080p \
        --no-extras --view "$V" $BENCH_ARGS > "$OUT/$N.json" 2> "$OUT/$N.err" || { echo "$N failed"; exit 1; }
      python3 -c "
import json; d = json.loads(open('$OUT/$N.json').read()); pt = d['path_tracer']; pm = d['passes_ms']
print('$L', '$V', 'rep $rep', d['value'], 'fps', 'lanes', pt['lane_efficiency'], 'pt_ms', pm.get('pathtrace'),
      'atrous', d['roofline']['avg_launch_ms'])"
    done
  done
done
