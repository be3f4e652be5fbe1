#!/bin/bash
# hardware queues per process (PTSVGF_HW_QUEUES -> GPU_MAX_HW_QUEUES, at most 32 on this pool) at 4K K = 4, default view
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for q in 8 16 24 32 16 24 32 8; do
  PTSVGF_HW_QUEUES=$q timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras > gpurun_out/q.json 2>/dev/null || exit $?
  python3 -c "import json; d=json.loads(open('gpurun_out/q.json').read()); print('queues=$q', d['value'])"
done
