#!/bin/bash
# Band renderer: how much the host wait for the G-buffer motion bound costs (back_lag, NOSYNC = no wait, fixed reach)
cd "$GRAFT_REPO_ROOT"
run() { # name env...
  local name=$1; shift
  env "$@" ROUNDS=0 BOUNDS=${BOUNDS} timeout -k 10 300 python -u tools/band_sim.py ${N} > gpurun_out/bl_$name.log 2>&1 || exit $?
  echo "$name: $(grep predicted gpurun_out/bl_$name.log | tail -1)"
}
N=2 BOUNDS=0,864,2160
run n2_k4_lag2 FIF=4 PTSVGF_BAND_LAG=2
run n2_k4_lag3 FIF=4 PTSVGF_BAND_LAG=3
run n2_k4_nosync FIF=4 NOSYNC=1
run n2_k8_lag6 FIF=8 PTSVGF_BAND_LAG=6
N=8 BOUNDS=0,240,448,662,908,1188,1446,1762,2160
run n8_k8_lag2 FIF=8 PTSVGF_BAND_LAG=2
run n8_k8_lag5 FIF=8 PTSVGF_BAND_LAG=5
run n8_k8_nosync FIF=8 NOSYNC=1
