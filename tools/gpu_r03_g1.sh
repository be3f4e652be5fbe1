cd "$GRAFT_REPO_ROOT"
timeout -k 10 400 python -u -m pytest tests/test_gpu_atrous.py tests/test_gpu_parity.py -k "atrous or config0" -x -q --timeout 200 --timeout-method thread > gpurun_out/g1_tests.log 2>&1
rc=$?; tail -3 gpurun_out/g1_tests.log; [ $rc -eq 0 ] || exit $rc
timeout -k 10 600 python -u -m pytest tests/test_gpu_bench_bands.py -x -q -s --timeout 500 --timeout-method thread > gpurun_out/g1_bands.log 2>&1
rc=$?; tail -3 gpurun_out/g1_bands.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=5 timeout -k 10 300 python -u tools/bench_atrous.py 0 2 > gpurun_out/g1_ba.log 2>&1
rc=$?; grep -E "mean_us|identical" gpurun_out/g1_ba.log; [ $rc -eq 0 ] || exit $rc
FIF=1 VIEW=surface PASSES=trace bash tools/gpu_profile.sh r03s1
