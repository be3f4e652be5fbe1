#!/bin/bash
# closest_budget A/B with the serial and surface-view extras: alternating repetitions on one box.
# usage: bash tools/budget_ab2.sh "256 512 1024" [reps]
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/bud2
for rep in $(seq 1 ${2:-2}); do
  for c in $1; do
    timeout -k 10 300 python bench.py --no-1080p --no-cpu-baseline --steps 40 --pt-uniform closest_budget=$c \
      > gpurun_out/bud2/c${c}_$rep.json 2> gpurun_out/bud2/c${c}_$rep.err || exit 1
    python3 - gpurun_out/bud2/c${c}_$rep.json c$c rep$rep <<'PY'
import json, sys
d = json.loads(open(sys.argv[1]).read())
print(sys.argv[2], sys.argv[3], "4K", d["value"], "serial", d.get("fps_serial"), "surface", (d.get("surface_view") or {}).get("fps"))
PY
  done
done
