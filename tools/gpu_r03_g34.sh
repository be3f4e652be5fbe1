#!/bin/bash
# Ghost zone with the G-buffer on the reprojection's rows only: gloo bench rehearsals, then simulations.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_bands.py -x -v --timeout 300 --timeout-method thread > gpurun_out/fs_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -7 gpurun_out/fs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 400 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8.log 2>&1
rc=$?; echo "sim8 rc=$rc"; grep -E '^rank|^pred|passes alone' gpurun_out/fs_sim8.log; [ $rc -eq 0 ] || exit $rc
RANKS=0 timeout -k 10 200 python -u tools/frame_shard_sim.py 2 > gpurun_out/fs_sim2.log 2>&1
rc=$?; echo "sim2 rc=$rc"; grep -E '^rank|^pred|passes alone' gpurun_out/fs_sim2.log; exit $rc
