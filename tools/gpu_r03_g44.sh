#!/bin/bash
# Frame-shard simulations at HEAD with the bench's defaults (bands balanced by measured band work), 2 / 4 / 8 ranks.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
for n in 2 4 8; do
  timeout -k 10 400 python -u tools/frame_shard_sim.py $n > gpurun_out/fs_head_n$n.log 2>&1
  rc=$?; echo "sim$n rc=$rc"; grep -E '^rank|^pred' gpurun_out/fs_head_n$n.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
done
