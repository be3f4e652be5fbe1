#!/bin/bash
# HEAD check: every GPU test (gloo frame-shard rehearsals included), then the 8-rank frame-shard simulation.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t41.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t41.log; [ $rc -eq 0 ] || exit $rc
BALANCE=0 timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8_head.log 2>&1
rc=$?; echo "sim8 rc=$rc"; grep -E '^rank|^pred' gpurun_out/fs_sim8_head.log | cut -c1-150; exit $rc
