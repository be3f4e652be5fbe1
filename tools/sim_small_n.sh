R=$GRAFT_REPO_ROOT
for cfg in "4 4 12" "4 4 18" "2 2 12" "2 2 16"; do
  set -- $cfg
  WINDOW=$2 K=$3 BALANCE=0 timeout -k 10 600 python -u $R/tools/frame_shard_sim.py $1 > $R/gpurun_out/sim_n$1_w$2_k$3.log 2>&1 || exit 1
  echo "N $1 window $2 K $3: $(grep predicted $R/gpurun_out/sim_n$1_w$2_k$3.log)"
done
