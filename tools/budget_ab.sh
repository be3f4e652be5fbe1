cd $GRAFT_REPO_ROOT
mkdir -p gpurun_out/bud
for rep in 1 2; do
for cfg in "256 256" "256 512" "256 128" "512 256" "128 256"; do
  set -- $cfg
  for V in default surface; do
    timeout -k 10 200 python bench.py --no-1080p --no-extras --no-cpu-baseline --view $V --steps 40 --pt-uniform shadow_budget=$1 --pt-uniform closest_budget=$2 > gpurun_out/bud/s$1_c$2_${V}_$rep.json 2> gpurun_out/bud/s$1_c$2_${V}_$rep.err || exit 1
    python3 -c "import json; d=json.loads(open('gpurun_out/bud/s$1_c$2_${V}_$rep.json').read()); print('s$1 c$2 $V rep$rep', d['value'])"
  done
done
done
