cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 200 --timeout-method thread > gpurun_out/g21_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g21_tests.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=5 timeout -k 10 300 python -u tools/bench_atrous.py 0 3 > gpurun_out/g21_ba.log 2>&1
rc=$?; grep -E "mean_us|identical" gpurun_out/g21_ba.log; exit $rc
