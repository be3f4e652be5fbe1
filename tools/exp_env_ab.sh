#!/bin/bash
# Same-box A/B of one environment switch: 4K + 1080p bench with NAME=A and NAME=B, twice, alternating.
# usage: bash tools/exp_env_ab.sh NAME A B [bench args...]
cd "$GRAFT_REPO_ROOT"
N=$1; A=$2; B=$3; shift 3
for rep in 1 2; do
  for v in "$A" "$B"; do
    env "$N=$v" timeout -k 10 300 python bench.py --steps 30 --warmup 5 --no-cpu-baseline "$@" > gpurun_out/eab_$v.log 2>&1 || exit $?
    python - "$N" "$v" <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/eab_{sys.argv[2]}.log") if l.startswith("{")][-1])
print(f"{sys.argv[1]}={sys.argv[2]}", "4K", d["ms_per_step"], "1080p", d.get("ms_per_step_1080p"),
      {k: v for k, v in d["passes_ms"].items() if k in ("gbuffer", "pathtrace")})
PY
  done
done
