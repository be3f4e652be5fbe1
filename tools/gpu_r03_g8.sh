# 8-band simulation with and without the exchange stand-ins, same box
cd "$GRAFT_REPO_ROOT"
for x in "0 0" "20 50" "0 0" "20 50"; do
  set -- $x
  XLAT_US=$1 XGBS=$2 FIF=8 ROUNDS=1 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsy_$1.log 2>&1 || exit $?
  echo "N=8 K=8 lat=$1 bw=$2: $(grep best gpurun_out/bsy_$1.log)"; grep -E "^rank" gpurun_out/bsy_$1.log | tail -8 | awk '{print $2, $5, $6, $9, $10, $11}' | tr '\n' ';'; echo
done
