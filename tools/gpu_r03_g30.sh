#!/bin/bash
# Frame shard: frames in flight (band slots K) and own slots swept, N = 2 and 8.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { n=$1; tag=$2; shift 2; env "$@" timeout -k 10 200 python -u tools/frame_shard_sim.py $n > gpurun_out/fs_$tag.log 2>&1 || return $?; echo "== N=$n $*"; grep -E '^rank|^pred' gpurun_out/fs_$tag.log; }
run 2 n2a RANKS=0 K=10 OWN=3 && run 2 n2b RANKS=0 K=16 OWN=4 && run 2 n2c RANKS=0 K=24 OWN=6 && \
run 8 n8a RANKS=3,7 K=34 OWN=3 && run 8 n8b RANKS=3,7 K=50 OWN=4 && run 8 n8c RANKS=3,7 K=34 OWN=3 XLAT_US=0 XGBS=0
