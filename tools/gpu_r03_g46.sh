#!/bin/bash
# a-trous tile height A/B (PT_ATROUS_TJ: rows per tile for S <= 8; tj4 also S = 16) on both views: the a-trous
# HIP-event launch average and fps, same box; plus the a-trous bit-identity tests on each variant.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT/path-tracing-svgf_amd"
for L in lib_exp/tj16 lib_exp/tj4; do
  PTSVGF_LIB_DIR=$R/$L timeout -k 10 300 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 120 --timeout-method thread > gpurun_out/t46.log 2>&1
  rc=$?; echo "$L pytest rc=$rc"; tail -1 gpurun_out/t46.log; [ $rc -eq 0 ] || exit $rc
done
for v in surface default; do for L in lib lib_exp/tj16 lib_exp/tj4 lib lib_exp/tj16 lib_exp/tj4; do
  PTSVGF_LIB_DIR=$R/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --view $v > gpurun_out/ab46.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab46.json').read()); r=d['roofline']; print('$v $L', d['value'], 'atrous ms', r['avg_launch_ms'], 'frac', r['frac'])"
done; done
