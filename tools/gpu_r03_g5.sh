# 4-wide any-hit tree: parity, then A/B
cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_parity.py tests/test_gpu_fullsize.py tests/test_gpu_deep.py tests/test_gpu_bands.py -x -q --timeout 400 --timeout-method thread > gpurun_out/g5_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g5_tests.log; [ $rc -eq 0 ] || exit $rc
REPS=2 bash tools/uniform_ab_views.sh wide_bvh 0 1
