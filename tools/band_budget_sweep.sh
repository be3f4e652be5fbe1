cd "$GRAFT_REPO_ROOT"
run() { local name=$1; shift
  env "$@" ROUNDS=0 BOUNDS=${BOUNDS} timeout -k 10 300 python -u tools/band_sim.py ${N} > gpurun_out/bl_$name.log 2>&1 || exit $?
  echo "$name: $(grep predicted gpurun_out/bl_$name.log | tail -1)"; }
N=2 BOUNDS=0,864,2160
run n2_k4_budget FIF=4
run n2_k4_nobudget FIF=4 PT_UNIFORMS=shadow_budget=0,closest_budget=0
N=4 BOUNDS=0,420,884,1392,2160
run n4_k4_budget FIF=4
run n4_k4_nobudget FIF=4 PT_UNIFORMS=shadow_budget=0,closest_budget=0
