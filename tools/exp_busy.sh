#!/bin/bash
# Kernel-trace a bench run with frames in flight and report how much of the steady-state window has at least one
# kernel running (gaps = dependency / launch stalls) and the mean number of concurrent kernels.
# usage: bash tools/exp_busy.sh "<bench args>"
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --output-format csv -d "$R/gpurun_out/busy" -o run -- python3 "$R/bench.py" --no-cpu-baseline --no-1080p $1 > "$R/gpurun_out/busy.log" 2>&1 || exit $?
python3 "$R/tools/busy.py" "$R/gpurun_out/busy/run_kernel_trace.csv"
