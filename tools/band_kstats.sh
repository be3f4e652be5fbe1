#!/bin/bash
# Per-kernel time per frame (rocprofv3 --kernel-trace --stats) of single band_sim ranks:
# bash tools/band_kstats.sh <tag> <N> <bounds|-> <rank> [<rank> ...]   (FIF, PTSVGF_* env pass through)
set -o pipefail
TAG=$1; NR=$2; B=$3
shift 3
R="$GRAFT_REPO_ROOT"
cd /tmp && export TMPDIR=/tmp
for RK in "$@"; do
  OUT="$R/gpurun_out/bandk_$TAG/rank$RK"
  mkdir -p "$OUT"
  if [ "$B" != "-" ]; then export BOUNDS=$B; fi
  RANKS=$RK ROUNDS=0 timeout -k 10 300 rocprofv3 --kernel-trace --stats --output-format csv -d "$OUT" -o run -- \
    python3 "$R/tools/band_sim.py" "$NR" 3840 2160 > "$OUT/sim.log" 2>&1 || exit $?
  echo "== rank $RK of $NR: $(grep '^rank' "$OUT/sim.log")"
  python3 - "$OUT/run_kernel_stats.csv" <<'PY'
import csv, sys
rows = list(csv.DictReader(open(sys.argv[1])))
import os
K = int(os.environ.get("FIF", "1"))
frames = max(3, 2 * K) + 32  # band_sim: max(3, 2K) warm-up + 30 timed + 1 probe + 1 profiled frames
tot = sum(float(r['TotalDurationNs']) for r in rows)
print(f"  kernel time per frame {tot / frames / 1e3:8.1f} us")
for r in sorted(rows, key=lambda r: -float(r['TotalDurationNs']))[:12]:
    print(f"  {r['Name'][:60]:60s} n/frame={int(r['Calls']) / frames:5.2f} avg={float(r['AverageNs'])/1e3:8.1f} us "
          f"per frame {float(r['TotalDurationNs']) / frames / 1e3:8.1f} us")
PY
done
