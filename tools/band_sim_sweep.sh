cd "$GRAFT_REPO_ROOT"
for n in 2 4; do for f in 4 8; do
  FIF=$f ROUNDS=1 timeout -k 10 300 python -u tools/band_sim.py $n > gpurun_out/bs_${n}_${f}.log 2>&1 || exit $?
  echo "N=$n FIF=$f: $(grep best gpurun_out/bs_${n}_${f}.log)"
done; done
