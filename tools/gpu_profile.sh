#!/bin/bash
# rocprofv3 passes for the 4K frame: kernel trace + stats, then separate PMC passes (one counter group per run,
# within the per-block limits of MI355X_MICROARCH.md).
# FIF (default 1): frames in flight. 1 = every kernel runs alone, so its durations compare with the bench's
# serialised per-pass HIP-event timing; 4 = the headline configuration, whose traversal launches are the
# lane-refill kernels (wf_trace_closest_refill / wf_trace_shadow_refill, renderer.py trace_refill).
# VIEW (default "default"): bench.py --view. PASSES (default "trace fetch write sq l2 sq2"; also "ta": texture-address
# unit busy cycles, summed over the 256 TAs; "tcp": vector L1 tag accesses, its read requests to L2 and their summed
# latency): which runs.
# usage: FIF=4 VIEW=surface bash tools/gpu_profile.sh <tag> [extra bench args]
set -o pipefail
TAG=${1:-r03}
shift
FIF=${FIF:-1}
VIEW=${VIEW:-default}
PASSES=${PASSES:-trace fetch write sq l2 sq2}
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/prof_$TAG"
mkdir -p "$OUT"
cd /tmp && export TMPDIR=/tmp
B="$R/bench.py --steps 5 --warmup 2 --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $FIF --view $VIEW $*"
echo "$FIF $VIEW $B" > "$OUT/config.txt"
# the a-trous machine code this profile measures (bench.py compares it with the library it loads)
python3 "$R/tools/kernel_hash.py" "${PTSVGF_LIB_DIR:-$R/path-tracing-svgf_amd/lib}/libptsvgf.so" > "$OUT/atrous_code_sha256.txt"
for p in $PASSES; do
  case $p in
    trace) A="--kernel-trace --stats" ;;
    fetch) A="--pmc FETCH_SIZE" ;;
    write) A="--pmc WRITE_SIZE" ;;
    sq) A="--pmc SQ_WAVES SQ_WAVE_CYCLES SQ_BUSY_CYCLES SQ_WAIT_ANY SQ_WAIT_INST_ANY SQ_ACTIVE_INST_ANY SQ_ACTIVE_INST_VALU SQ_INSTS_VALU" ;;
    l2) A="--pmc TCC_HIT_sum TCC_MISS_sum GRBM_GUI_ACTIVE" ;;
    sq2) A="--pmc SQ_INSTS_VMEM_RD SQ_INSTS_LDS SQ_INSTS_SALU SQ_LDS_BANK_CONFLICT SQ_LDS_IDX_ACTIVE" ;;
    ta) A="--pmc TA_TA_BUSY_sum TA_BUSY_avr GRBM_GUI_ACTIVE SQ_INSTS_VMEM_RD SQ_WAVE_CYCLES SQ_BUSY_CYCLES" ;;
    tcp) A="--pmc TCP_TOTAL_CACHE_ACCESSES_sum TCP_TCC_READ_REQ_sum TCP_TCC_READ_REQ_LATENCY_sum GRBM_GUI_ACTIVE" ;;
    *) echo "unknown pass $p"; exit 2 ;;
  esac
  echo "pass $p: $(date +%T)"
  timeout -k 10 600 rocprofv3 $A --output-format csv -d "$OUT/$p" -o run -- python3 $B > "$OUT/$p.log" 2>&1 || exit $?
done
echo profile-done
