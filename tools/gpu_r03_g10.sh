# 8-band simulation with exchange stand-ins after removing the unused G-buffer fork streams
cd "$GRAFT_REPO_ROOT"
for x in "0 0" "20 50"; do
  set -- $x
  XLAT_US=$1 XGBS=$2 FIF=8 ROUNDS=1 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsz_$1.log 2>&1 || exit $?
  echo "N=8 K=8 lat=$1 bw=$2: $(grep best gpurun_out/bsz_$1.log)"
done
XLAT_US=20 XGBS=50 FIF=4 ROUNDS=1 timeout -k 10 400 python -u tools/band_sim.py 2 > gpurun_out/bsz_2.log 2>&1 || exit $?
echo "N=2 K=4 lat=20 bw=50: $(grep best gpurun_out/bsz_2.log)"
