#!/bin/bash
# 4K + 1080p bench of the default build and lib_exp variants, same box.  usage: bash tools/exp_lib_1080.sh v1 v2 ...
cd "$GRAFT_REPO_ROOT"
for v in default "$@"; do
  d="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib"; [ "$v" != default ] && d="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib_exp/$v"
  PTSVGF_LIB_DIR="$d" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline > gpurun_out/l1080_$v.log 2>&1 || exit $?
  python - "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/l1080_{sys.argv[1]}.log") if l.startswith("{")][-1])
print(sys.argv[1], "4K", d["ms_per_step"], "1080p", d.get("ms_per_step_1080p"))
PY
done
