#!/bin/bash
# Tile shard at 8 ranks, 4K, equal bands (tools/frame_shard_sim.py SHARD=tiles): batch x band slots x own slots.
# CFGS: space-separated batch:K:own tokens.
R=$GRAFT_REPO_ROOT
for cfg in ${CFGS:-1:8:4 2:8:4 4:12:8}; do
  IFS=: read -r b k o <<< "$cfg"
  echo "tile batch $b K $k own $o: $(date +%T)"
  SHARD=tiles TBATCH=$b K=$k OWN=$o BALANCE=0 timeout -k 10 600 python -u "$R/tools/frame_shard_sim.py" 8 \
    > "$R/gpurun_out/sim_tiles_b${b}_k${k}_o${o}.log" 2>&1 \
    || { echo "batch $b K $k failed"; tail -5 "$R/gpurun_out/sim_tiles_b${b}_k${k}_o${o}.log"; exit 1; }
  grep predicted "$R/gpurun_out/sim_tiles_b${b}_k${k}_o${o}.log"
done
