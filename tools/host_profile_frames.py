"""cProfile of one frame-shard rank's frame loop on one GPU (host issue cost per frame; communication stood in for by
tools/frame_shard_sim.py's spin kernels). usage: python tools/host_profile_frames.py [rank] [N]"""
import cProfile
import os
import pstats
import sys
import time

rank = int(sys.argv[1]) if len(sys.argv) > 1 else 3
n = sys.argv[2] if len(sys.argv) > 2 else "8"
sys.argv = [sys.argv[0], n]
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(REPO, "tools"))
import frame_shard_sim as F  # noqa: E402  (sets up the library, the scene and the stand-ins)
import torch  # noqa: E402

r = F.D.FrameShardRenderer(F.scene, F.W, F.H, F.cfg, rank, F.N, F.FakeDist(), own_slots=F.OWN, frames_in_flight=F.K)
for _ in range(2 * F.K + F.N):
    r.frame()
r.r.flush()
torch.cuda.synchronize()
waits = []
orig = torch.cuda.Event.synchronize


def timed_sync(ev):
    t = time.perf_counter()
    orig(ev)
    waits.append(time.perf_counter() - t)


torch.cuda.Event.synchronize = timed_sync
pr = cProfile.Profile()
frames = 96
t0 = time.perf_counter()
pr.enable()
for _ in range(frames):
    r.frame()
pr.disable()
issue = time.perf_counter() - t0
torch.cuda.synchronize()
torch.cuda.Event.synchronize = orig
print(f"rank {rank}: issue {issue / frames * 1e3:.3f} ms per frame, of which {sum(waits) / frames * 1e3:.3f} blocked on "
      f"events; host work {(issue - sum(waits)) / frames * 1e3:.3f} ms per frame (under cProfile)")
st = pstats.Stats(pr)
st.sort_stats("tottime").print_stats(30)
r.close()
