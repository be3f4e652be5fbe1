# a-trous tile shapes: same box, both views, per-step us (tools/bench_atrous.py, variant 0 = tile kernel)
cd "$GRAFT_REPO_ROOT"
for L in lib lib_exp/t16 lib_exp/t16a lib_exp/t12 lib; do
  PTSVGF_LIB_DIR=$GRAFT_REPO_ROOT/path-tracing-svgf_amd/$L ROUNDS=5 timeout -k 10 300 python -u tools/bench_atrous.py 0 > gpurun_out/ta_$(echo $L | tr / _).log 2>&1 || exit $?
  echo "$L: $(grep -E 'mean_us' gpurun_out/ta_$(echo $L | tr / _).log | tr '\n' ' ')"
done
