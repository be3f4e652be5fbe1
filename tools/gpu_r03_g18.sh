# 8 waves/SIMD for the traversal kernels: a 20- or 16-entry LDS stack spilling to global memory, same box
cd "$GRAFT_REPO_ROOT"
L=$GRAFT_REPO_ROOT/path-tracing-svgf_amd
PTSVGF_LIB_DIR=$L/lib_exp/s20w8 timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py -x -q -k "frames_match or refill or wide or config0 or prune" --timeout 400 --timeout-method thread > gpurun_out/g18_tests.log 2>&1
rc=$?; tail -1 gpurun_out/g18_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/env_ab_views.sh PTSVGF_LIB_DIR $L/lib $L/lib_exp/s20w8 $L/lib_exp/s16w8 $L/lib_exp/s20w6
