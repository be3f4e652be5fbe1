#!/bin/bash
# Same-box A/B of one path-tracing-pass int uniform over several values (bench.py --pt-uniform), 4K default and
# surface views (K = 4), alternating values within each repetition.
# usage: REPS=2 bash tools/uniform_ab_views.sh NAME V1 V2 ... [-- extra bench args]
cd "$GRAFT_REPO_ROOT"
N=$1; shift
VALS=()
while [ $# -gt 0 ] && [ "$1" != "--" ]; do VALS+=("$1"); shift; done
[ "$1" == "--" ] && shift
for rep in $(seq 1 ${REPS:-2}); do
  for v in "${VALS[@]}"; do
    for view in ${VIEWS_AB:-default surface}; do
      f=gpurun_out/uab_${N}_${v}_$view.log
      timeout -k 10 300 python bench.py --steps 40 --warmup 5 --no-cpu-baseline --no-1080p --no-extras \
        --view $view --pt-uniform "$N=$v" "$@" > $f 2>&1 || exit $?
      python - "$N" "$v" "$view" "$f" <<'PY'
import json, sys
d = json.loads([l for l in open(sys.argv[4]) if l.startswith("{")][-1])
pt = d["path_tracer"]
print(f"{sys.argv[1]}={sys.argv[2]} {sys.argv[3]:8s} fps {d['value']:8.2f}  pt_ms {d['passes_ms'].get('pathtrace', 0):6.3f}"
      f"  visits/ray {pt['visits_per_ray']}  lanes {pt['lane_efficiency']}  rewalks {pt['tie_rewalks']}", flush=True)
PY
    done
  done
done
