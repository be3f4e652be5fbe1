cd "$GRAFT_REPO_ROOT"
for kb in "6 1" "8 1" "12 1" "8 2" "12 3" "12 2"; do
  set -- $kb
  timeout -k 10 200 python bench.py --width 1920 --height 1080 --no-extras --no-cpu-baseline --steps 300 --warmup 20 --frames-in-flight $1 --trace-batch $2 > gpurun_out/s_$1_$2.log 2>&1 || exit $?
  python -c "import json; d=json.loads(open('gpurun_out/s_$1_$2.log').read().strip().splitlines()[-1]); print('K=$1 B=$2', d['value'])"
done
