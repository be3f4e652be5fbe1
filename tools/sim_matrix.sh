#!/bin/bash
# Several tools/frame_shard_sim.py configurations in one GPU session, each under its own time limit, stopping at the
# first failure. Each argument: NAME=ENV1=V1+ENV2=V2+... (the environment of that simulation; BOUNDS, ROTATIONS, N
# etc. may be given in the session's environment for all). Logs: gpurun_out/<TAG>_<NAME>.log.
# usage: TAG=r06b bash tools/sim_matrix.sh base=OWN=2 r16=OWN=2+PTSVGF_OWN_CU_RESERVE=16 ...
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
TAG=${TAG:-sim}
for spec in "$@"; do
  name=${spec%%=*}
  envs=${spec#*=}
  echo "[$(date +%T)] $name: $envs"
  ( for kv in ${envs//+/ }; do export "$kv"; done
    timeout -k 10 ${SIM_TIMEOUT:-600} python -u tools/frame_shard_sim.py ${N:-8} > "gpurun_out/${TAG}_$name.log" 2>&1 ) || exit $?
  grep "predicted" "gpurun_out/${TAG}_$name.log"
done
