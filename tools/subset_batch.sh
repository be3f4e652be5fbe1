#!/bin/bash
# Tile-subset path tracer at 4K: whole frame, one stride-8 subset, and stride-8 subsets of B frames batched
# (tools/pt_subset_prof.py), each under its own time limit.
R=$GRAFT_REPO_ROOT
for cfg in "1 1" "8 1" "8 4" "8 8" "1 2"; do
  set -- $cfg
  STRIDE=$1 BATCH=$2 FRAMES=32 timeout -k 10 300 python3 "$R/tools/pt_subset_prof.py" 2>&1 | grep "per draw" || exit 1
done
