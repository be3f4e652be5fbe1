# SLP vectorizer off for the library (fewer VGPRs: refill kernels 96 -> 64-66): parity tests, then A/B
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py -x -q --timeout 400 --timeout-method thread > gpurun_out/g17_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g17_tests.log; [ $rc -eq 0 ] || exit $rc
L=$GRAFT_REPO_ROOT/path-tracing-svgf_amd
REPS=2 bash tools/env_ab_views.sh PTSVGF_LIB_DIR $L/lib_exp/slp $L/lib $L/lib_exp/nslp6
