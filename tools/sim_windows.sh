#!/bin/bash
# Frame-shard exchange window x band slots at 8 ranks, 4K, equal bands (tools/frame_shard_sim.py): throughput and
# camera-to-modulate latency. Each config is one simulator run under its own time limit; the first failure stops.
R=$GRAFT_REPO_ROOT
for cfg in ${CFGS:-"8 34" "8 16" "1 12" "1 16"}; do
  set -- $cfg
  echo "window $1 K $2: $(date +%T)"
  WINDOW=$1 K=$2 BALANCE=0 timeout -k 10 600 python -u "$R/tools/frame_shard_sim.py" 8 > "$R/gpurun_out/sim_w$1_k$2.log" 2>&1 \
    || { echo "window $1 K $2 failed"; tail -5 "$R/gpurun_out/sim_w$1_k$2.log"; exit 1; }
  grep predicted "$R/gpurun_out/sim_w$1_k$2.log"
done
