# high-priority SVGF back-end stream: one GPU (4K, both views) and 8 simulated bands
cd "$GRAFT_REPO_ROOT"
python -c "import torch; print('priority range', torch.cuda.Stream.priority_range())"
REPS=2 bash tools/env_ab_views.sh PTSVGF_BACK_PRIORITY 0 1 || exit $?
for v in 0 1; do
  PTSVGF_BACK_PRIORITY=$v XLAT_US=20 XGBS=50 FIF=8 ROUNDS=0 timeout -k 10 400 python -u tools/band_sim.py 8 > gpurun_out/bsp_$v.log 2>&1 || exit $?
  echo "prio=$v: $(grep predicted gpurun_out/bsp_$v.log)"; grep -E "^rank" gpurun_out/bsp_$v.log | sed 's/gbuf.*//' 
done
