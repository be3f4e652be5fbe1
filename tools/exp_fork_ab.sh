cd $GRAFT_REPO_ROOT
export GPU_MAX_HW_QUEUES=16 FIF=4 BALANCE=0
for cfg in "1 1" "0 1" "1 0" "0 0"; do set -- $cfg
  for rep in 1 2; do
  PTSVGF_GBUFFER_FORK=$1 PTSVGF_TRACE_FORK=$2 timeout -k 10 300 python tools/band_sim.py 8 2>&1 | grep predicted | sed "s/^/gfork=$1 tfork=$2: /" || exit $?
  done
done
