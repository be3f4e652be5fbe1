#!/bin/bash
# Fused modulate (last a-trous iteration's epilogue): every GPU test, then same-box fps and per-pass times both ways.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
timeout -k 10 900 python -u -m pytest tests -x -q -m gpu --timeout 300 --timeout-method thread > gpurun_out/t45.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t45.log; [ $rc -eq 0 ] || exit $rc
for v in default surface; do for fm in 0 1 0 1; do
  timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --view $v --fuse-modulate $fm > gpurun_out/fm.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/fm.json').read()); p=d['passes_ms']
print('$v fuse=$fm', d['value'], 'atrous', p.get('atrous'), 'atrous_modulate', p.get('atrous_modulate'), 'modulate', p.get('modulate'))"
done; done
