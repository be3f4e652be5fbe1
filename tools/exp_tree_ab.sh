#!/bin/bash
# A/B of the SAH trees: G-buffer leaf size (PTSVGF_RASTER_LEAF, an experiment build knob since removed: leaf 8 kept) and the any-hit tree (shadow_tree uniform),
# full 4K frame + the 72/576-row band probe.
cd "$GRAFT_REPO_ROOT"
for cfg in "8 1" "8 0"; do
  set -- $cfg
  PTSVGF_RASTER_LEAF=$1 timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --pt-uniform shadow_tree=$2 > gpurun_out/tree_$1_$2.log 2>&1 || exit $?
  python - "$1" "$2" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/tree_{sys.argv[1]}_{sys.argv[2]}.log") if l.startswith("{")][-1])
print("leaf", sys.argv[1], "shadow_tree", sys.argv[2], "4K", d["ms_per_step"], "1080p", d.get("ms_per_step_1080p"), {k: v for k, v in d["passes_ms"].items() if k in ("gbuffer", "pathtrace")})
PY
done
