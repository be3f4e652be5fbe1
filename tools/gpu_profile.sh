#!/bin/bash
# rocprofv3 passes for the 4K frame: kernel trace + stats, then separate PMC passes (one counter group per run,
# within the per-block limits of MI355X_MICROARCH.md). One frame in flight, so every kernel runs alone and its
# durations compare with the bench's serialised per-pass HIP-event timing.
# usage: bash tools/gpu_profile.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r02}
shift
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-1080p --no-extras --frames-in-flight 1 $*"
timeout -s KILL 60 rocprofv3 --list-avail > "$OUT/list_avail.txt" 2>&1
timeout -k 10 600 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT/trace" -o run -- python3 $B > "$OUT/trace.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc FETCH_SIZE --output-format csv -d "$OUT/fetch" -o run -- python3 $B > "$OUT/fetch.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc WRITE_SIZE --output-format csv -d "$OUT/write" -o run -- python3 $B > "$OUT/write.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU --output-format csv -d "$OUT/sq" -o run -- python3 $B > "$OUT/sq.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE --output-format csv -d "$OUT/l2" -o run -- python3 $B > "$OUT/l2.log" 2>&1 || exit $?
timeout -k 10 600 rocprofv3 --pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE --output-format csv -d "$OUT/sq2" -o run -- python3 $B > "$OUT/sq2.log" 2>&1 || exit $?
echo profile-done
