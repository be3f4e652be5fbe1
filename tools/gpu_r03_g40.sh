#!/bin/bash
# Host issue cost of a frame-shard rank (8 ranks simulated, rank 3): cProfile.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 300 python -u tools/host_profile_frames.py 3 8 > gpurun_out/host_frames.log 2>&1; rc=$?
echo "rc=$rc"; grep -E "^rank|ncalls|tottime" -A32 gpurun_out/host_frames.log | head -45; exit $rc
