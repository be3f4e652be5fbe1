#!/bin/bash
# Ghost-zone frame shard with the early history exchange: 8/4/2-rank simulations.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8.log 2>&1
rc=$?; echo "sim8 rc=$rc"; grep -E '^rank|^pred|passes alone' gpurun_out/fs_sim8.log; [ $rc -eq 0 ] || exit $rc
RANKS=0,1 timeout -k 10 200 python -u tools/frame_shard_sim.py 2 > gpurun_out/fs_sim2.log 2>&1
rc=$?; echo "sim2 rc=$rc"; grep -E '^rank|^pred|passes alone' gpurun_out/fs_sim2.log; [ $rc -eq 0 ] || exit $rc
RANKS=0,2 timeout -k 10 200 python -u tools/frame_shard_sim.py 4 > gpurun_out/fs_sim4.log 2>&1
rc=$?; echo "sim4 rc=$rc"; grep -E '^rank|^pred|passes alone' gpurun_out/fs_sim4.log; exit $rc
