#!/bin/bash
# End-of-round check: the driver's round-end sequence (tools/gpu_roundend.sh), then the 8-rank frame-shard simulation
# of the default mode (window 4, K 16; equal then balanced bands) for the multi-GPU numbers in README / DESIGN.
R=$GRAFT_REPO_ROOT
cd "$R" || exit 1
bash tools/gpu_roundend.sh || exit $?
WINDOW=4 K=16 timeout -k 10 900 python -u tools/frame_shard_sim.py 8 > gpurun_out/sim_final.log 2>&1 || exit 1
grep -E "predicted|balanced bounds" gpurun_out/sim_final.log
