#!/bin/bash
# Full-frame 4K bench + the 72-row band probe (tools/band_scale.py) for the default build and lib_exp variants.
# usage: bash tools/gpu_lib_ab.sh name1 name2 ...
cd "$GRAFT_REPO_ROOT"
for v in default "$@"; do
  d="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib"; [ "$v" != default ] && d="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib_exp/$v"
  PTSVGF_LIB_DIR="$d" timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-1080p > gpurun_out/ab_$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json, sys
line = [l for l in open(f"gpurun_out/ab_{sys.argv[1]}.log") if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1], "frame", d["ms_per_step"], {k: v for k, v in d["passes_ms"].items() if k in ("gbuffer", "pathtrace")})
PY
  PTSVGF_LIB_DIR="$d" BAND_H="${BAND_H:-72 576}" timeout -k 10 300 python tools/band_scale.py 2>&1 | grep "^h=" || exit $?
done
