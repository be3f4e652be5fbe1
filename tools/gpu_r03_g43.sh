#!/bin/bash
# A-trous SoA pair kernel (lib_exp/soa, -DPT_ATROUS_SOA=1): bit-identity tests against the step kernel and the
# oracle, then same-box a-trous launch time (bench's HIP-event average over 20 launches) and fps, both libraries.
cd "$GRAFT_REPO_ROOT"; mkdir -p gpurun_out
R="$GRAFT_REPO_ROOT/path-tracing-svgf_amd"
PTSVGF_LIB_DIR=$R/lib_exp/soa timeout -k 10 600 python -u -m pytest tests/test_gpu_atrous.py tests/test_gpu_parity.py -x -q --timeout 300 --timeout-method thread > gpurun_out/t43.log 2>&1
rc=$?; echo "pytest rc=$rc"; tail -2 gpurun_out/t43.log; [ $rc -eq 0 ] || exit $rc
for v in default surface; do for L in lib lib_exp/soa lib lib_exp/soa; do
  PTSVGF_LIB_DIR=$R/$L timeout -k 10 200 python3 bench.py --no-cpu-baseline --no-1080p --no-extras --view $v > gpurun_out/ab43.json 2>/dev/null || exit $?
  python3 -c "
import json; d=json.loads(open('gpurun_out/ab43.json').read()); r=d['roofline']; print('$v $L', d['value'], 'atrous ms', r['avg_launch_ms'], 'frac', r['frac'], 'passes atrous', d['passes_ms'].get('atrous'))"
done; done
