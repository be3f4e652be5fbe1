#!/bin/bash
# Frame shard, 8 simulated ranks (0 and 4): what the SVGF stream's ~1 ms per frame is made of.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
run() { tag=$1; shift; env "$@" RANKS=0,4 timeout -k 10 200 python -u tools/frame_shard_sim.py 8 > gpurun_out/fs8_$tag.log 2>&1 || return $?; echo "== $tag $*"; grep -E '^rank|^pred' gpurun_out/fs8_$tag.log; }
run base && run noxchg XLAT_US=0 XGBS=0 && run rw3840 PT_UNIFORMS=refill_waves=3840 && run rw2560 PT_UNIFORMS=refill_waves=2560 && \
run norefill PT_UNIFORMS=trace_refill=0 && run lowprio PTSVGF_BACK_PRIORITY=0
