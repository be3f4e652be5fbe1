#!/bin/bash
# 4K bench (pipelined K=4 and serial K=1) for in-tree library builds: bash tools/lib_ab.sh "<uniforms>" lib_dir ...
# (lib_dir relative to path-tracing-svgf_amd/, e.g. lib or lib_exp/x; uniforms like "trace_refill=1")
set -o pipefail
U=$1
shift
R="$GRAFT_REPO_ROOT"
mkdir -p "$R/gpurun_out/lib_ab"
ARGS=""
for kv in $(echo "$U" | tr ',' ' '); do ARGS="$ARGS --pt-uniform $kv"; done
for L in "$@"; do
  for K in ${KLIST:-4 1}; do
    N=$(echo "$L" | tr '/' '_')_k$K
    PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/$L" timeout -k 10 200 python3 "$R/bench.py" --no-cpu-baseline --no-1080p \
      --no-extras --frames-in-flight $K $ARGS > "$R/gpurun_out/lib_ab/$N.json" 2> "$R/gpurun_out/lib_ab/$N.err" || exit $?
    python3 -c "
import json; d = json.loads(open('$R/gpurun_out/lib_ab/$N.json').read())
print('$L', 'K=$K', d['value'], d['path_tracer']['lane_efficiency'])"
  done
done
