#!/bin/bash
# What the driver runs at round end: every GPU test, smoke(), then the default bench (one JSON line).
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 300 python -c "import __graft_entry__ as g; g.smoke()" > gpurun_out/smoke.log 2>&1
rc=$?; echo "smoke rc=$rc"; tail -1 gpurun_out/smoke.log; [ $rc -eq 0 ] || exit $rc
start=$(date +%s)
timeout -k 10 900 python bench.py > gpurun_out/bench.json 2> gpurun_out/bench.err
rc=$?; echo "bench rc=$rc wall=$(( $(date +%s) - start ))s"; tail -c 300 gpurun_out/bench.json; exit $rc
