#!/bin/bash
# rocprofv3 kernel stats of a short 4K bench (per-kernel average ms per frame).
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$R/gpurun_out/ks" -o run -- python3 "$R/bench.py" --steps 5 --warmup 2 --no-cpu-baseline --no-1080p ${BENCH_ARGS} > "$R/gpurun_out/ks.log" 2>&1 || exit $?
python3 - "$R/gpurun_out/ks/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
frames = 8
for r in rows:
    print(f"{r['Name'][:70]:70s} calls {int(r['Calls']):4d} avg {float(r['AverageNs'])/1e3:8.1f} us  per-frame {float(r['TotalDurationNs'])/frames/1e6:.3f} ms")
PY
