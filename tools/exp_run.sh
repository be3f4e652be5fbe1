#!/bin/bash
# On the GPU box: per-kernel time of each lib_exp variant (+ the default build) on the 4K bench frame.
# usage: bash tools/exp_run.sh name1 name2 ...
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for v in default "$@"; do
  d="$R/path-tracing-svgf_amd/lib"; [ "$v" != default ] && d="$R/path-tracing-svgf_amd/lib_exp/$v"
  PTSVGF_LIB_DIR="$d" timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/exp_$v" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-1080p > "$R/gpurun_out/exp_$v.log" 2>&1 || exit $?
  python3 - "$R/gpurun_out/exp_$v/run_kernel_stats.csv" "$v" <<'PY'
import csv, sys
import re
rows = {}
for r in csv.DictReader(open(sys.argv[1])):
    k = re.sub(r"<[^>]*>", "", r["Name"].replace("void ", "").split("(")[0])
    rows[k] = rows.get(k, 0.0) + float(r["TotalDurationNs"]) / 8e6
keys = ["ptk::wf_trace_shadow", "ptk::wf_trace_closest", "ptk::wf_primary", "ptk::gbuffer_kernel", "ptk::wf_shade"]
print(sys.argv[2], " ".join(f"{k.split('::')[1]}={rows.get(k, 0):.3f}" for k in keys), f"total={sum(rows.values()):.3f} ms/frame")
PY
done
