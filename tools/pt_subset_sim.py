"""Per-rank path-tracing throughput of two multi-GPU work splits, simulated on one GPU (ranks one after another).

  band:        rank r traces the rows [b_r, b_r+1) of cost-balanced bounds (ptsvgf.dist today)
  interleaved: rank r traces the 16x16 tiles t = 8k + r of the whole frame (tile_stride / tile_offset uniforms)

Each rank's path-tracing pass alone is issued FRAMES times round-robin over K streams (frames in flight) and
timed wall-clock. usage: python tools/pt_subset_sim.py [N] [W] [H]   env: FIF (8), BOUNDS (comma list)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch

from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.renderer import Renderer, _set_stream
from ptsvgf.scene import build_scene

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
H = int(sys.argv[3]) if len(sys.argv) > 3 else 2160
K = int(os.environ.get("FIF", "8"))
FRAMES = 24
BOUNDS = tuple(int(v) for v in os.environ.get("BOUNDS", "0,148,292,460,668,936,1232,1560,2160").split(","))

torch.cuda.set_device(0)
gl.init(0)
scene = build_scene("table_clock_plant")
cfg = parameter_config()


def pt_wall(r, stride=1, offset=0):
    for p, _ in r.pt_slots:
        p.set_uniform_int("tile_stride", stride)
        p.set_uniform_int("tile_offset", offset)
    def run(n):
        for f in range(n):
            _set_stream(r._streams[f % K])
            r._use_slot(f % K)
            r._path_trace()
    run(K)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    run(FRAMES)
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) * 1e3 / FRAMES


full = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                frames_in_flight=K)
full.frame()
torch.cuda.synchronize()
print(f"full frame PT: {pt_wall(full):.3f} ms/frame (K={K})")
inter = [pt_wall(full, N, r) for r in range(N)]
print("interleaved:", " ".join(f"{v:.3f}" for v in inter), f"max {max(inter):.3f} ms")
full.close()
band = []
for r in range(N):
    y0, y1 = BOUNDS[r], BOUNDS[r + 1]
    b = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                 frames_in_flight=K, band=(y0, y1, y0, y1 - y0))
    b.frame()
    torch.cuda.synchronize()
    band.append(pt_wall(b))
    b.close()
print("band:       ", " ".join(f"{v:.3f}" for v in band), f"max {max(band):.3f} ms")
gl.shutdown()
