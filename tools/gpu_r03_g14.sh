# refill rounds on bands: resident-wave estimate per launch (refill_waves), 8 and 2 simulated equal bands
cd "$GRAFT_REPO_ROOT"
for w in 0 2560 1280 640 320; do
  PT_UNIFORMS=refill_waves=$w XLAT_US=20 XGBS=50 FIF=8 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsr_$w.log 2>&1 || exit $?
  echo "N=8 refill_waves=$w: $(grep predicted gpurun_out/bsr_$w.log | cut -c1-100)"
done
for w in 0 2560 1280; do
  PT_UNIFORMS=refill_waves=$w XLAT_US=20 XGBS=50 FIF=4 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 2 > gpurun_out/bsr2_$w.log 2>&1 || exit $?
  echo "N=2 refill_waves=$w: $(grep predicted gpurun_out/bsr2_$w.log | cut -c1-100)"
done
