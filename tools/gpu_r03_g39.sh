#!/bin/bash
# Shipped G-buffer (pt_raster_pass_adopt): GPU tests of the raster/parity files + gloo bench rehearsals, then
# 8-rank simulations with and without it (ranks 1, 3, 5).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_bench_bands.py tests/test_gpu_raster.py tests/test_gpu_atrous.py -x -v --timeout 300 --timeout-method thread > gpurun_out/ship_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "PASS|FAIL|passed|failed" gpurun_out/ship_tests.log | tail -12; [ $rc -eq 0 ] || exit $rc
SHIP=1 RANKS=1,3,5 BALANCE=0 timeout -k 10 300 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_ship1.log 2>&1
rc=$?; echo "ship1 rc=$rc"; grep -E '^rank|passes alone' gpurun_out/fs_ship1.log | cut -c1-240; [ $rc -eq 0 ] || exit $rc
SHIP=0 RANKS=1,3,5 BALANCE=0 timeout -k 10 300 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_ship0.log 2>&1
rc=$?; echo "ship0 rc=$rc"; grep -E '^rank|passes alone' gpurun_out/fs_ship0.log | cut -c1-240; exit $rc
