R=$GRAFT_REPO_ROOT
REPS=2 timeout -k 10 900 bash $R/tools/ab_libs.sh lib lib_exp/pref || exit 1
for K in 5 6; do
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $K > $R/gpurun_out/k$K.json 2>/dev/null || exit 1
  timeout -k 10 300 python3 $R/bench.py --no-cpu-baseline --no-1080p --no-extras --frames-in-flight $K --view surface > $R/gpurun_out/k${K}s.json 2>/dev/null || exit 1
  python3 -c "import json; a=json.load(open('$R/gpurun_out/k$K.json')); b=json.load(open('$R/gpurun_out/k${K}s.json')); print('K $K', a['value'], b['value'], a['latency'])"
done
