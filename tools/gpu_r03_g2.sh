# fine leaves: parity tests, then A/B of the leaf size
cd "$GRAFT_REPO_ROOT"
timeout -k 10 600 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deep.py -x -q --timeout 300 --timeout-method thread > gpurun_out/g2_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g2_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=1 bash tools/env_ab_views.sh PTSVGF_FINE_LEAVES 0 1 2 4
