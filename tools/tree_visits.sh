#!/bin/bash
# Traversal visits of the bench scene at 4K, both views, per tree-build configuration (tools/wide_collapse_ab.py: node
# + triangle visits per kind and the planes' digest). Each argument: NAME=ENV1=V1+ENV2=V2 (NAME=- for the defaults).
# Log: gpurun_out/tree_visits_<TAG>.log. usage: TAG=a bash tools/tree_visits.sh base=- c1=PTSVGF_WIDE_COLLAPSE=1
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
L=gpurun_out/tree_visits_${TAG:-a}.log
for spec in "$@"; do
  name=${spec%%=*}
  envs=${spec#*=}
  for v in default surface; do
    ( [ "$envs" != "-" ] && for kv in ${envs//+/ }; do export "$kv"; done
      echo -n "$name $v: " >> $L
      PTSVGF_WIDE_STATS=1 timeout -k 10 180 python -u tools/wide_collapse_ab.py 3840 2160 $v 2>>$L.err | tail -1 >> $L ) || exit 1
  done
done
python - "$L" <<'PY'
import json, sys
rows = {}
for line in open(sys.argv[1]):
    name, rest = line.split(": ", 1)
    d = json.loads(rest)
    rows.setdefault(name.split()[0], {})[d["view"]] = d
base = next(iter(rows.values()))
for n, r in rows.items():
    out = []
    for v in ("default", "surface"):
        d, b = r[v], base[v]
        out.append(f"{v}: bounce {d['bounce_visits'] / b['bounce_visits'] - 1:+.2%} shadow {d['shadow_visits'] / b['shadow_visits'] - 1:+.2%} "
                   f"total {(d['bounce_visits'] + d['shadow_visits']) / (b['bounce_visits'] + b['shadow_visits']) - 1:+.2%} {d['planes_sha256']}")
    print(f"{n:12s} " + " | ".join(out))
PY
