#!/bin/bash
# a-trous tile width A/B (nx8: 128-column tiles for S = 8; nx16a: 64-column tiles for S = 16) on both views: the a-trous
# HIP-event launch average and fps, same box; plus the a-trous bit-identity tests on each variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT/path-tracing-svgf_amd"
for L in lib_exp/nx8 lib_exp/nx16a; do
  PTSVGF_LIB_DIR=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t49.log 2>&1
  rc=$?; echo "$L pytest rc=$rc"; tail -1 gpurun_out/t49.log; [ $rc -eq 0 ] || exit $rc
done
for v in surface default; do for L in lib lib_exp/nx8 lib_exp/nx16a lib lib_exp/nx8 lib_exp/nx16a; do
  PTSVGF_LIB_DIR=$R/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --view $v > gpurun_out/ab49.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab49.json').read()); r=d['roofline']; print('$v $L', d['value'], 'atrous ms', r['avg_launch_ms'], 'frac', r['frac'])"
done; done
