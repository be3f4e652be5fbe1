#!/bin/bash
# 1-GPU bench for fork / frames-in-flight combinations (A/B), then the 8-band simulation for two of them
cd "$GRAFT_REPO_ROOT"
for cfg in "4 0 0" "4 0 1" "4 1 1" "2 1 1" "3 0 0"; do set -- $cfg
  PTSVGF_GBUFFER_FORK=$2 timeout -k 10 300 python bench.py --no-cpu-baseline --frames-in-flight $1 --pt-uniform trace_fork=$3 2>&1 | grep "^{" | python -c "import json,sys; d=json.loads(sys.stdin.read()); print('K=$1 gfork=$2 tfork=$3', d['value'], d['fps_1080p'])" || exit $?
done
for cfg in "3 0 0" "2 1 1"; do set -- $cfg
  GPU_MAX_HW_QUEUES=16 FIF=$1 BALANCE=0 PTSVGF_GBUFFER_FORK=$2 PTSVGF_TRACE_FORK=$3 timeout -k 10 300 python tools/band_sim.py 8 2>&1 | grep predicted | sed "s/^/K=$1 gfork=$2 tfork=$3: /" || exit $?
done
