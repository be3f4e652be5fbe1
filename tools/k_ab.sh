cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/kab
for rep in 1 2; do for K in 3 4 5 6; do
  timeout -k 10 200 python bench.py --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $K > gpurun_out/kab/k${K}_$rep.json 2>/dev/null || exit 1
  python3 -c "import json; d=json.loads(open('gpurun_out/kab/k${K}_$rep.json').read()); print('K=$K rep$rep', d['value'], d['latency']['camera_to_modulate_ms'])"
done; done
