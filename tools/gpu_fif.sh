#!/bin/bash
# frames-in-flight: GPU tests of the pipelined driver, then the 4K bench at K = 1, 2, 3
cd "$GRAFT_REPO_ROOT"
timeout -k 10 300 python -m pytest tests -x -q -m gpu -k "frames_in_flight or fast_driver" > gpurun_out/tf.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -3 gpurun_out/tf.log
[ $rc -eq 0 ] || exit $rc
for k in 1 2 3; do
  timeout -k 10 300 python bench.py --steps 20 --warmup 5 --no-cpu-baseline --frames-in-flight $k > gpurun_out/fif$k.log 2>&1 || exit $?
  python - $k <<'PY'
import json, sys
d = json.loads([l for l in open(f"gpurun_out/fif{sys.argv[1]}.log") if l.startswith("{")][-1])
print("K", sys.argv[1], "4K", d["value"], "fps", d["ms_per_step"], "ms; 1080p", d.get("fps_1080p"), "fps")
PY
done
