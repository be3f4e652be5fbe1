#!/bin/bash
# Band-parity diagnostics of the every-pass row bands (--shard bands) on 2 gloo ranks, one GPU: which setting makes
# the gathered bands differ from the one-GPU render. Prints bounds and per-plane differing pixels per variant.
cd "$GRAFT_REPO_ROOT" || exit 1
mkdir -p gpurun_out
port=29611
while IFS= read -r extra; do
  port=$((port + 1))
  timeout -k 10 300 python -m torch.distributed.run --nnodes=1 --nproc-per-node=2 --master-addr 127.0.0.1 \
    --master-port=$port bench.py --gpus 2 --backend gloo --width 320 --height 256 --steps 4 --warmup 2 --no-extras \
    --no-1080p --no-cpu-baseline --shard bands --ship-gbuffer 0 $extra > gpurun_out/diag.json 2> gpurun_out/diag.err \
    || { echo "run failed: $extra"; tail -20 gpurun_out/diag.err; exit 1; }
  grep -h "ref2" gpurun_out/diag.err
  python3 -c "
import json; d=json.loads(open('gpurun_out/diag.json').read().strip().splitlines()[-1]); bp=d['band_parity']
print('[$extra]', d['bands'].get('bounds'), d['bands'].get('calibration'), bp['bit_exact'], bp['frames'], {k:(v['differing_px'], round(v['max_abs'], 3)) for k,v in bp['planes'].items() if not v['bit_exact']})"
done <<< "${VARIANTS:---moving}"
