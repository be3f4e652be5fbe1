#!/bin/bash
# Kernel traces of the whole-frame path tracer (stride 1) and of one tile-shard subset (stride 8, the band traversal
# settings TileShardRenderer uses) at 4K: which launches a subset pays for at whole-frame size.
cd /tmp && export TMPDIR=/tmp
R=$GRAFT_REPO_ROOT
mkdir -p $R/gpurun_out/subset
for s in 1 8; do
  U="trace_refill=90"
  [ $s -gt 1 ] && U="trace_refill=90,shadow_budget=256,closest_budget=256,refill_waves=1280"
  STRIDE=$s PT_UNIFORMS=$U timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d $R/gpurun_out/subset/s$s \
    -o run -- python3 $R/tools/pt_subset_prof.py > $R/gpurun_out/subset/s$s.log 2>&1 || exit $?
  grep "per draw" $R/gpurun_out/subset/s$s.log
done
