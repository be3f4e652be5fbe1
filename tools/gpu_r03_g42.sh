#!/bin/bash
# Reprojection block fetch: parity tests, then same-box timing of the reprojection (per-pass HIP events) both ways.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t42.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t42.log; [ $rc -eq 0 ] || exit $rc
for v in default surface; do for b in 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --view $v --svgf-uniform reproj_block=$b > gpurun_out/rb.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/rb.json').read()); print('$v block=$b', d['value'], 'reproject ms', d['passes_ms']['reproject'])"
done; done
