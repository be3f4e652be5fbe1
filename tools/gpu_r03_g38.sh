#!/bin/bash
# Why is simulated rank 3 slower? Ranks 2, 3, 4 with the frame counter as is, then offset by 1 (rank r then traces
# the frames rank r + 1 traced).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
RANKS=2,3,4 BALANCE=0 timeout -k 10 300 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_fc0.log 2>&1
rc=$?; echo "fc0 rc=$rc"; grep -E '^rank' gpurun_out/fs_fc0.log | cut -c1-120; [ $rc -eq 0 ] || exit $rc
FC_OFFSET=1 RANKS=2,3,4 BALANCE=0 timeout -k 10 300 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_fc1.log 2>&1
rc=$?; echo "fc1 rc=$rc"; grep -E '^rank' gpurun_out/fs_fc1.log | cut -c1-120; exit $rc
