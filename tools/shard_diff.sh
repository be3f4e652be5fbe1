#!/bin/bash
# Round 6: kernel traces of one simulated frame-shard rank (tools/frame_shard_sim.py, 8 ranks at
# 4K, one rank alone on the GPU) and of the one-GPU bench frame (K = 1 and K = 4), for a launch-by-launch diff
# (tools/launch_diff.py). SIMS: which simulated configurations (name=ENV,ENV...; default the bench's 8-rank default).
# usage: bash tools/shard_diff.sh <tag>
set -o pipefail
TAG=${1:-r06}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/shard_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
SIMS=${SIMS:-"default=OWN=2,K=16,WINDOW=4"}
for s in $SIMS; do
  name=${s%%=*}
  envs=${s#*=}
  echo "sim $name ($envs): $(date +%T)"
  ( export RANKS=${RANKS:-4} ROTATIONS=1 BALANCE=0 FRAMES=${FRAMES:-64}; for kv in ${envs//,/ }; do export "$kv"; done
    timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/sim_$name" -o run -- \
      python3 "$R/tools/frame_shard_sim.py" 8 > "$OUT/sim_$name.log" 2>&1 ) || exit $?
  grep "wall" "$OUT/sim_$name.log" | head -3
done
for k in 1 4; do
  echo "bench K=$k: $(date +%T)"
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/bench_k$k" -o run -- \
    python3 "$R/bench.py" --steps 16 --warmup 4 --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $k \
    > "$OUT/bench_k$k.json" 2> "$OUT/bench_k$k.err" || exit $?
  tail -c 200 "$OUT/bench_k$k.json"
done
echo shard-diff-done
