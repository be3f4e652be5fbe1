#!/bin/bash
# Round 6: the production GPU SVGF chain against the float64 restatement (4K), then the one-GPU frame rate at 1-4 frames
# in flight (K = 1 with and without the bounce-0 fork): how much a second and third frame in flight buy (the question a
# frame-shard rank poses, DESIGN.md "Round 6: what a rank's frame is made of").
cd "$GRAFT_REPO_ROOT" || exit 1
timeout -k 10 600 python -u -m pytest tests/test_gpu_independent.py -k svgf -x -v -s --timeout 580 --timeout-method thread > gpurun_out/r06_svgf_indep.log 2>&1; tail -4 gpurun_out/r06_svgf_indep.log
for v in "1 --pt-uniform trace_fork=0" "1" "2" "3" "4"; do
  set -- $v
  timeout -k 10 300 python bench.py --frames-in-flight $v --no-extras --no-1080p --no-cpu-baseline --steps 100 > gpurun_out/r06_k_$1_$#.json 2> gpurun_out/r06_k_$1_$#.err || exit $?
  python -c "import json,sys; l=json.loads(open('gpurun_out/r06_k_$1_$#.json').read().strip().splitlines()[-1]); print('$v', l['value'], l['passes_ms']['pathtrace'])"
done
