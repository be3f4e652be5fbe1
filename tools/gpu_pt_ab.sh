#!/bin/bash
# path-tracer A/B (4K, no CPU baseline) + GPU parity tests
cd "$GRAFT_REPO_ROOT"
for args in "" "--pt-uniform shadow_bvh4=0"; do
  timeout -k 10 300 python bench.py --steps 10 --warmup 3 --no-cpu-baseline --no-1080p $args > gpurun_out/ab.log 2>&1 || exit $?
  python - "$args" <<'PY'
import json, sys
line = [l for l in open("gpurun_out/ab.log") if l.startswith("{")][-1]
d = json.loads(line)
print(sys.argv[1] or "default", d["ms_per_step"], {k: v for k, v in d["passes_ms"].items() if k in ("gbuffer", "pathtrace")})
PY
done
timeout -k 10 900 python -m pytest tests -x -q -m gpu > gpurun_out/t.log 2>&1
rc=$?; echo "pytest rc=$rc"; grep -E "passed|failed|Error" gpurun_out/t.log | tail -5
