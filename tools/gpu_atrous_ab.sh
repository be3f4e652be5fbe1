#!/bin/bash
# a-trous: GPU tests, then A/B timing of variant specs (tools/bench_atrous.py) on the 4K default and surface views.
# usage: bash tools/gpu_atrous_ab.sh <variant spec> ...
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ta.log 2>&1
rc=$?; tail -3 gpurun_out/ta.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=${ROUNDS:-5} timeout -k 10 500 python -u tools/bench_atrous.py "$@" > gpurun_out/ba.log 2>&1
rc=$?; grep -E "mean_us|identical" gpurun_out/ba.log; exit $rc
