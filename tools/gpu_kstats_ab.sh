#!/bin/bash
# per-kernel stats for two bench variants: bash tools/gpu_kstats_ab.sh "<args A>" "<args B>"
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
i=0
for args in "$@"; do
  i=$((i+1))
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ks$i" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-1080p $args > "$R/gpurun_out/ks$i.log" 2>&1 || exit $?
  echo "== variant $i: $args"
  cut -d, -f1-4 "$R/gpurun_out/ks$i/run_kernel_stats.csv" | head -12
done
