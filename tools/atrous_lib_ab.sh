#!/bin/bash
# a-trous library A/B: the a-trous GPU tests on lib, then tools/bench_atrous.py (tile kernel, 4K default and surface
# views) alternating between library builds. usage: REPS=2 bash tools/atrous_lib_ab.sh lib_exp/base lib
cd "$GRAFT_REPO_ROOT"
mkdir -p gpurun_out/aab
timeout -k 10 300 python -u -m pytest tests/test_gpu_atrous.py -x -q --timeout 120 --timeout-method thread > gpurun_out/aab/tests.log 2>&1
rc=$?; tail -3 gpurun_out/aab/tests.log; [ $rc -eq 0 ] || exit $rc
for rep in $(seq 1 ${REPS:-2}); do
  for L in "$@"; do
    N=$(echo "$L" | tr '/' '_')_$rep
    PTSVGF_LIB_DIR="$GRAFT_REPO_ROOT/path-tracing-svgf_amd/$L" ROUNDS=${ROUNDS:-5} timeout -k 10 300 \
      python -u tools/bench_atrous.py 0 > gpurun_out/aab/$N.log 2>&1 || exit $?
    echo "$N $(python3 -c "
import json
rows = [json.loads(l) for l in open('gpurun_out/aab/$N.log') if l.startswith('{')]
for v in ('default', 'surface'):
    r = [x for x in rows if x.get('view') == v and 'us' in x]
    print(v, [x['us'] for x in r], end='  ')
")"
  done
done
