#!/bin/bash
# 4K frames/s for several frames-in-flight counts (headline config, no extras)
cd "$GRAFT_REPO_ROOT"
for K in ${KS:-3 4 5 6}; do
  timeout -k 10 200 python bench.py --no-extras --no-cpu-baseline --no-1080p --steps 200 --warmup 20 --frames-in-flight $K ${BENCH_ARGS} > gpurun_out/k4_$K.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/k4_$K.log').read().strip().splitlines()[-1]); print('K=$K', d['value'])"
done
