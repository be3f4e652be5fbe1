#!/bin/bash
# Per-kernel durations (rocprofv3 --kernel-trace --stats) of the 4K bench frame with one frame in flight, for a list
# of path-tracer uniform settings: bash tools/kstats_ab.sh <tag> "trace_refill=0" "trace_refill=1" ...
set -o pipefail
TAG=$1
shift
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for U in "$@"; do
  N=$(echo "$U" | tr '=, ' '___')
  OUT="$R/gpurun_out/kstats_$TAG/$N"
  mkdir -p "$OUT"
  ARGS=""
  for kv in $(echo "$U" | tr ',' ' '); do ARGS="$ARGS --pt-uniform $kv"; done
  timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/bench.py" --steps 10 --warmup 3 --no-cpu-baseline --no-1080p --no-extras --frames-in-flight 1 $ARGS \
    > "$OUT/bench.json" 2> "$OUT/bench.err" || exit $?
  echo "== $U"
  python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:8]:
    print(f"  {r['Name'][:58]:58s} n={r['Calls']:>4} avg={float(r['AverageNs'])/1e3:8.1f} us")
PY
done
