# back lag / frames in flight sweep, 8 simulated equal bands with exchange stand-ins
cd "$GRAFT_REPO_ROOT"
for kl in "8 2" "8 4" "8 7" "12 4" "12 8" "16 8"; do
  set -- $kl
  PTSVGF_BAND_LAG=$2 XLAT_US=20 XGBS=50 FIF=$1 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsl_$1_$2.log 2>&1 || exit $?
  echo "K=$1 lag=$2: $(grep predicted gpurun_out/bsl_$1_$2.log | cut -c1-90) waits $(grep -E '^rank' gpurun_out/bsl_$1_$2.log | sed 's/.*motion wait \([0-9.]*\).*/\1/' | tr '\n' ' ')"
done
