cd "$GRAFT_REPO_ROOT"
timeout -k 10 900 python -u -m pytest tests/test_gpu_bvh.py tests/test_gpu_raster.py tests/test_gpu_bands.py -x -q --timeout 400 --timeout-method thread > gpurun_out/g9_tests.log 2>&1
rc=$?; tail -2 gpurun_out/g9_tests.log; grep -E "point:|nan_object:" gpurun_out/g9_tests.log; exit $rc
