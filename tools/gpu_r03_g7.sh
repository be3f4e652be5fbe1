# band simulations with the exchange stand-ins: 2 bands (K = 4) and 8 bands (K = 8), binary and 4-wide walks
cd "$GRAFT_REPO_ROOT"
for w in 0 1; do
  for nk in "2 4" "8 8"; do
    set -- $nk
    PT_UNIFORMS=wide_bvh=$w FIF=$2 ROUNDS=1 timeout -k 10 400 python -u tools/band_sim.py $1 > gpurun_out/bsx_$1_w$w.log 2>&1 || exit $?
    echo "N=$1 K=$2 wide=$w: $(grep -E 'spin calibration' gpurun_out/bsx_$1_w$w.log | head -1) $(grep best gpurun_out/bsx_$1_w$w.log)"
  done
done
