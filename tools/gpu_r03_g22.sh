cd "$GRAFT_REPO_ROOT"
for L in lib lib_exp/oldat lib lib_exp/oldat; do
  PTSVGF_LIB_DIR=$GRAFT_REPO_ROOT/path-tracing-svgf_amd/$L ROUNDS=5 timeout -k 10 300 python -u tools/bench_atrous.py 0 > gpurun_out/ta22.log 2>&1 || exit $?
  echo "$L: $(grep -E 'mean_us' gpurun_out/ta22.log | tr '\n' ' ')"
done
