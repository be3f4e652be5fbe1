#!/bin/bash
# frames in flight at 4K re-checked at the round's last commit (default view), twice each
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for K in 3 4 5 6 4 5 3 6; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $K > gpurun_out/k.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/k.json').read()); print('K=$K', d['value'])"
done
