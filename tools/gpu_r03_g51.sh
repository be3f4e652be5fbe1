#!/bin/bash
# 8-rank frame-shard simulation at the round's last commit (fused modulate), bench defaults (balanced bands)
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_final_n8.log 2>&1
rc=$?; echo "sim8 rc=$rc"; grep -E '^pred' gpurun_out/fs_final_n8.log; exit $rc
