#!/bin/bash
# GPU session: all GPU tests, then the 4K bench.
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -m pytest tests -x -q -m gpu -s > gpurun_out/t.log 2>&1
rc=$?
echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/t.log | tail -5
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 10 --warmup 3 --no-cpu-baseline ${BENCH_ARGS} > gpurun_out/b.log 2>&1
rc=$?; echo "bench rc=$rc"; tail -c 1200 gpurun_out/b.log
