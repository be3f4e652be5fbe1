#!/bin/bash
# Same-box A/B of bench.py argument sets on one library (4K, the headline view and the surface view), alternating the
# variants REPS times so drift hits every variant alike. Variants are ';'-separated argument lists in VARIANTS (an
# empty one is the default). Prints one line per run.
# usage: REPS=2 VARIANTS=';--pt-uniform trace_fork=1' bash tools/ab_args.sh
set -o pipefail
R="$GRAFT_REPO_ROOT"
OUT="$R/gpurun_out/ab_args"
mkdir -p "$OUT"
IFS=';' read -r -a VARS <<< "${VARIANTS:-}"
[ ${#VARS[@]} -eq 0 ] && VARS=("")
for rep in $(seq 1 "${REPS:-2}"); do
  for i in "${!VARS[@]}"; do
    A="${VARS[$i]}"
    for V in ${VIEWS:-default surface}; do
      N=v${i}_${V}_$rep
      # shellcheck disable=SC2086
      timeout -k 10 300 python3 "$R/bench.py" --no-cpu-baseline --no-1080p --no-extras --view "$V" $A \
        > "$OUT/$N.json" 2> "$OUT/$N.err" || { echo "$N failed"; exit 1; }
      python3 -c "
import json; d = json.loads(open('$OUT/$N.json').read()); pm = d['passes_ms']
print('[$A]', '$V', 'rep $rep', d['value'], 'fps', 'pt_ms', pm.get('pathtrace'), 'latency',
      d.get('latency', {}).get('camera_to_modulate_ms'))"
    done
  done
done
