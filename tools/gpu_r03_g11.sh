cd "$GRAFT_REPO_ROOT"
XLAT_US=20 XGBS=50 FIF=8 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsw.log 2>&1 || exit $?
grep -E "^rank|predicted" gpurun_out/bsw.log
XLAT_US=0 XGBS=0 FIF=8 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsw0.log 2>&1 || exit $?
grep -E "^rank|predicted" gpurun_out/bsw0.log
