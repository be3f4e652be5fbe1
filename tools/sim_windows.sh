#!/bin/bash
# Frame-shard exchange window x band slots x burst at 8 ranks, 4K, equal bands (tools/frame_shard_sim.py): throughput
# and camera-to-modulate latency. CFGS: space-separated window:K[:burst] tokens. Each config is one simulator run under
# its own time limit; the first failure stops.
R=$GRAFT_REPO_ROOT
for cfg in ${CFGS:-8:34 8:16 1:12 1:16}; do
  IFS=: read -r w k b <<< "$cfg"
  b=${b:-1}
  echo "window $w K $k burst $b: $(date +%T)"
  WINDOW=$w K=$k BURST=$b BALANCE=0 timeout -k 10 600 python -u "$R/tools/frame_shard_sim.py" 8 \
    > "$R/gpurun_out/sim_w${w}_k${k}_b${b}.log" 2>&1 \
    || { echo "window $w K $k burst $b failed"; tail -5 "$R/gpurun_out/sim_w${w}_k${k}_b${b}.log"; exit 1; }
  grep predicted "$R/gpurun_out/sim_w${w}_k${k}_b${b}.log"
done
