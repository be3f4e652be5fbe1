#!/bin/bash
# Frame shard, 8 simulated ranks: the calibrated bounds alone (first in the process), then equal bands again.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
BOUNDS=0,306,568,832,1006,1208,1444,1744,2160 timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8_b1.log 2>&1
rc=$?; echo "b1 rc=$rc"; grep -E '^rank|^pred' gpurun_out/fs_sim8_b1.log; [ $rc -eq 0 ] || exit $rc
BALANCE=0 timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8_e1.log 2>&1
rc=$?; echo "e1 rc=$rc"; grep -E '^rank|^pred' gpurun_out/fs_sim8_e1.log; exit $rc
