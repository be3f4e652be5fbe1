#!/bin/bash
# trace_fork session: its parity tests, the bench A/B (K = 4 and serial, both views), the 8-rank frame-shard simulation
# with and without it (window 4, K 12) and with the shipped G-buffer, then the primary-raster unroll builds.
set -o pipefail
R=$GRAFT_REPO_ROOT
mkdir -p "$R/gpurun_out"
cd "$R" || exit 1
timeout -k 10 300 python -u -m pytest -x -q --timeout 120 --timeout-method thread -m gpu tests/test_gpu_parity.py \
  -k "trace_fork or frames_in_flight" > gpurun_out/fork_tests.log 2>&1 || { tail -30 gpurun_out/fork_tests.log; exit 1; }
tail -2 gpurun_out/fork_tests.log
REPS=1 VARIANTS=';--pt-uniform trace_fork=1;--frames-in-flight 1;--frames-in-flight 1 --pt-uniform trace_fork=1' \
  timeout -k 10 900 bash tools/ab_args.sh || exit 1
for pu in "" "trace_fork=1"; do
  PT_UNIFORMS=$pu WINDOW=4 K=12 BALANCE=0 timeout -k 10 600 python -u tools/frame_shard_sim.py 8 \
    > "gpurun_out/sim_fork_${pu:-base}.log" 2>&1 || exit 1
  grep predicted "gpurun_out/sim_fork_${pu:-base}.log"
done
SHIP=1 WINDOW=4 K=12 BALANCE=0 timeout -k 10 600 python -u tools/frame_shard_sim.py 8 \
  > gpurun_out/sim_fork_ship.log 2>&1 || exit 1
grep predicted gpurun_out/sim_fork_ship.log
REPS=1 timeout -k 10 900 bash tools/ab_libs.sh lib lib_exp/pru4 lib_exp/pru2
