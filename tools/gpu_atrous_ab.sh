cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 120 --timeout-method thread > gpurun_out/ta.log 2>&1
rc=$?; tail -3 gpurun_out/ta.log; [ $rc -eq 0 ] || exit $rc
ROUNDS=5 timeout -k 10 400 python -u tools/bench_atrous.py 0 4 4:atrous_chunks=3 4:atrous_chunks=12 4:atrous_xcd=1 4:atrous_nx=2 4:atrous_nx=1 > gpurun_out/ba.log 2>&1
rc=$?; grep -E "mean_us|identical" gpurun_out/ba.log; exit $rc
