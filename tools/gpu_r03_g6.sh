cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py -k "wide or refill or config0" -x -q --timeout 300 --timeout-method thread > gpurun_out/g6_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g6_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/uniform_ab_views.sh wide_bvh 0 1 || exit $?
PTSVGF_LIB_DIR=$GRAFT_REPO_ROOT/path-tracing-svgf_amd/lib_exp/ssort REPS=1 bash tools/uniform_ab_views.sh wide_bvh 1
