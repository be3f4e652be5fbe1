#!/bin/bash
# Primary-raster tile cull: its parity tests, then a same-box A/B against the library built before it.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out"
cd "$R" || exit 1
timeout -k 10 600 python -u -m pytest -x -q --timeout 300 --timeout-method thread -m gpu tests/test_gpu_raster.py \
  tests/test_gpu_fullsize.py tests/test_tiles.py > gpurun_out/cull_tests.log 2>&1 || { tail -30 gpurun_out/cull_tests.log; exit 1; }
tail -2 gpurun_out/cull_tests.log
PTSVGF_LIB_DIR="$R/path-tracing-svgf_amd/lib_exp/sort" timeout -k 10 600 python -u -m pytest -x -q --timeout 300 \
  --timeout-method thread -m gpu tests/test_gpu_raster.py > gpurun_out/sort_tests.log 2>&1 || { tail -30 gpurun_out/sort_tests.log; exit 1; }
tail -2 gpurun_out/sort_tests.log
REPS=${REPS:-2} timeout -k 10 1500 bash tools/ab_libs.sh lib_exp/base lib lib_exp/sort
