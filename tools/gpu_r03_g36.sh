#!/bin/bash
# Frame shard with bands balanced by measured band work: gloo bench rehearsals, then the 8-rank simulation
# (equal bands, then the calibrated bounds).
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_bands.py -x -v --timeout 300 --timeout-method thread -k frames > gpurun_out/fs_tests.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -5 gpurun_out/fs_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs_sim8_bal.log 2>&1
rc=$?; echo "sim8 rc=$rc"; grep -E '^rank|^pred|^balanced|^---' gpurun_out/fs_sim8_bal.log; exit $rc
