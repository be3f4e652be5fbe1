#!/bin/bash
# The default multi-GPU bench (--shard frames: window 4, 12 band slots) rehearsed with 8 gloo ranks on the one GPU at
# W x H (default 4K) with a moving camera: band_parity must be bit-exact (a one-GPU render of the same camera path).
R=$GRAFT_REPO_ROOT
W=${W:-3840}; H=${H:-2160}
P=$(python3 -c "import socket; s=socket.socket(); s.bind(('127.0.0.1',0)); print(s.getsockname()[1])")
timeout -k 10 ${T:-900} python3 -m torch.distributed.run --nnodes=1 --nproc-per-node=8 --master-addr 127.0.0.1 \
  --master-port=$P "$R/bench.py" --gpus 8 --backend gloo --width $W --height $H --steps 16 --warmup 2 --no-extras \
  --no-1080p --no-cpu-baseline --moving --equal-bands 1 > "$R/gpurun_out/rehearse8_${W}x${H}.json" \
  2> "$R/gpurun_out/rehearse8_${W}x${H}.err"
rc=$?
python3 -c "
import json,sys; d=json.loads(open('$R/gpurun_out/rehearse8_${W}x${H}.json').read().strip().splitlines()[-1])
bp=d['band_parity']; print('band_parity', bp['bit_exact'], bp['max_abs'], bp['frames'], 'bands', d['bands']['window'], d['bands']['frames_in_flight'], 'history rows', d.get('max_history_rows'), 'latency', d.get('latency'))
" || true
exit $rc
