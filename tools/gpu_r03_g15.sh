cd "$GRAFT_REPO_ROOT"
for rep in 1 2 3; do for w in 0 1280; do
  PT_UNIFORMS=refill_waves=$w XLAT_US=20 XGBS=50 FIF=8 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsr_$w.log 2>&1 || exit $?
  echo "N=8 refill_waves=$w: $(grep predicted gpurun_out/bsr_$w.log | sed 's/.*: \([0-9.]* ms = [0-9.]* fps\).*/\1/')  walls $(grep -E '^rank' gpurun_out/bsr_$w.log | sed 's/.*wall \([0-9.]*\) ms.*/\1/' | tr '\n' ' ')"
done; done
