#!/bin/bash
cd "$GRAFT_REPO_ROOT"
echo "host: $(hostname) nproc=$(nproc)"; rocm-smi --showproductname 2>/dev/null | grep -i -E "card|series" | head -3
timeout -k 10 900 python -m pytest tests/test_gpu_parity.py -x -q -m gpu -s > gpurun_out/t1.log 2>&1
rc=$?
echo "pytest rc=$rc"
if [ $rc -ne 0 ] && [ $rc -ne 1 ]; then echo "stopping (rc=$rc)"; exit $rc; fi
timeout -k 10 600 python bench.py --steps 5 --warmup 2 --no-cpu-baseline > gpurun_out/b1.log 2>&1
echo "bench rc=$?"
