"""cProfile of one band renderer's frame loop on one GPU (host issue cost per frame, exchanges stubbed by
tools/band_sim.py's stand-ins). usage: python tools/host_profile_band.py [rank] [N]"""
import cProfile
import os
import pstats
import sys
import time

sys.argv = [sys.argv[0], sys.argv[2] if len(sys.argv) > 2 else "8"] + sys.argv[1:2]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
rank = int(sys.argv[2]) if len(sys.argv) > 2 else 3
sys.argv = sys.argv[:2]
import band_sim as B  # noqa: E402  (sets up the library, the scene and the exchange stand-ins)
import torch  # noqa: E402

r = B.D.BandRenderer(B.scene, B.W, B.H, B.cfg, rank, B.N, B.FakeDist(), frames_in_flight=8)
for _ in range(20):
    r.frame()
torch.cuda.synchronize()
pr = cProfile.Profile()
t0 = time.perf_counter()
pr.enable()
for _ in range(50):
    r.frame()
pr.disable()
torch.cuda.synchronize()
print(f"rank {rank}: {(time.perf_counter() - t0) / 50 * 1e3:.3f} ms per frame (wall, 50 frames)")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(25)
r.close()
