#!/bin/bash
# Bench A/B over environment configurations, alternating, REPS times, both 4K views (bench.py --steps 20 --warmup 5,
# no CPU baseline / 1080p / extras). Each argument: NAME=ENV1=V1+ENV2=V2 (NAME=- for the defaults).
# Logs: gpurun_out/<TAG>/bench_<view>_<name>_r<rep>.json; prints one line per run and the per-configuration means.
# usage: TAG=fine_ab REPS=2 bash tools/env_bench_ab.sh base=- f2=PTSVGF_FINE_LEAVES=2
cd "$GRAFT_REPO_ROOT" || exit 1
O=gpurun_out/${TAG:-env_ab}
mkdir -p $O
for rep in $(seq 1 ${REPS:-2}); do
  for spec in "$@"; do
    name=${spec%%=*}
    envs=${spec#*=}
    for v in ${VIEWS:-default surface}; do
      ( [ "$envs" != "-" ] && for kv in ${envs//+/ }; do export "$kv"; done
        timeout -k 10 240 python -u bench.py --steps 20 --warmup 5 --no-cpu-baseline --no-1080p --no-extras --view $v \
          > $O/bench_${v}_${name}_r$rep.json 2> $O/bench_${v}_${name}_r$rep.err ) || exit 1
      echo "rep $rep $name $v: $(python -c "import json,sys; print(json.load(open(sys.argv[1]))['value'])" $O/bench_${v}_${name}_r$rep.json)"
    done
  done
done
python - $O <<'PY'
import glob, json, os, sys
from collections import defaultdict
m = defaultdict(list)
for f in sorted(glob.glob(os.path.join(sys.argv[1], "bench_*.json"))):
    _, view, *name, rep = os.path.basename(f)[:-5].split("_")
    m[("_".join(name), view)].append(json.load(open(f))["value"])
for (n, v), xs in sorted(m.items()):
    print(f"{n:10s} {v:8s} mean {sum(xs) / len(xs):8.2f}  runs {xs}")
PY
echo env-ab-done
