"""Single-GPU prediction of an N-GPU strong-scaling frame (ptsvgf.dist bands), ranks simulated one after another.

For every rank r of N: build the BandRenderer of r with the halo exchanges replaced by a recorder, time its frame
(GPU time of the band + host issue time) and probe its per-row BVH visit counts. Then fit the cost model of
make_band_renderer (T = a*visits + b*rows over the ranks), derive the balanced bounds and simulate again.
The predicted N-GPU frame time is the slowest rank, its halo exchanges stood in for by spin kernels of the modelled
RCCL time on the band's back-end stream (fake_exchange; XLAT_US=0 XGBS=0 turns them off).
usage: python tools/band_sim.py [N] [W] [H]"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PTSVGF_HW_QUEUES", "16")  # as bench.py
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import numpy as np
import torch

from ptsvgf import dist as D
from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.scene import build_scene

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
H = int(sys.argv[3]) if len(sys.argv) > 3 else 2160
LOG = []


class FakeDist:
    """Stands in for torch.distributed: this rank's own motion bound is the all-reduced one."""
    class ReduceOp:
        MAX = "max"

    def get_backend(self, group=None):
        return "gloo"

    def all_reduce(self, t, op=None, group=None):
        return None


# Exchange stand-in (XLAT_US / XGBS, default 20 us + 50 GB/s; XLAT_US=0 and XGBS=0: none, the round-2 simulation):
# each batch_isend_irecv the real halo_exchange would issue becomes a spin kernel on the stream the exchange runs on
# (the band's SVGF back-end stream), lasting latency + max(bytes sent, bytes received) / bandwidth — RCCL P2P over
# one xGMI link per neighbour, the sends and receives of a batch overlapping. The SVGF pass behind it waits for it
# exactly as it waits for the real exchange.
XLAT_US = float(os.environ.get("XLAT_US", "20"))
XGBS = float(os.environ.get("XGBS", "50"))
_CYC_PER_US = None


def _spin(us):
    """torch.cuda._sleep spins on the shader clock: calibrated once against HIP events."""
    global _CYC_PER_US
    if us <= 0:
        return
    if _CYC_PER_US is None:
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        torch.cuda._sleep(1000)
        e0.record()
        torch.cuda._sleep(2_000_000)
        e1.record()
        e1.synchronize()
        _CYC_PER_US = 2_000_000 / (e0.elapsed_time(e1) * 1e3)
        print(f"spin calibration: {_CYC_PER_US:.0f} cycles/us", flush=True)
    torch.cuda._sleep(int(us * _CYC_PER_US))


def fake_exchange(items, plan, dist, group=None, wait=True):
    """Record the bytes the real exchange would send and receive (ghost-bounded) and stand in for its time."""
    sent_b = recv_b = 0
    for t, n in items:
        if plan.world == 1 or n <= 0:
            continue
        row = t.shape[1] * t.shape[2] * 4
        for send, a, b, _ in plan.halo_parts(n):  # the transfers dist.halo_exchange would issue
            if send:
                sent_b += row * (b - a)
            else:
                recv_b += row * (b - a)
    if sent_b or recv_b:
        LOG.append(sent_b)
        _spin(XLAT_US + (max(sent_b, recv_b) / (XGBS * 1e3) if XGBS > 0 else 0.0))


D.halo_exchange = fake_exchange
if os.environ.get("NOSYNC") == "1":  # experiment: no host wait for the G-buffer's motion bound (fixed reach)
    def _motion_nosync(self):
        self.plan.motion = D.REPROJ_REACH + 8
    D.BandRenderer._motion = _motion_nosync
torch.cuda.set_device(0)
gl.init(0)
from ptsvgf._lib import check, pt
check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
scene = build_scene("table_clock_plant")
cfg = parameter_config()


def sim_rank(rk, bounds, probe=False, K=30):
    r = D.BandRenderer(scene, W, H, cfg, rk, N, FakeDist(), bounds=bounds,
                       frames_in_flight=int(os.environ.get("FIF", "1")), trace_batch=int(os.environ.get("BATCH", "1")))
    r.pass_path_tracing.set_uniform_int("pt_kernel", int(os.environ.get("PTK", "0")))
    if "SHADOW_BUDGET" in os.environ:
        r.pass_path_tracing.set_uniform_int("shadow_budget", int(os.environ["SHADOW_BUDGET"]))
    for kv in filter(None, os.environ.get("PT_UNIFORMS", "").split(",")):  # name=value,... on the path tracer
        name, val = kv.split("=")
        r.pass_path_tracing.set_uniform_int(name, int(val))
    for _ in range(max(3, 2 * r.r.K)):  # every frame slot used before timing (first use allocates)
        r.frame()
    torch.cuda.synchronize()
    LOG.clear()
    torch.cuda.synchronize()
    waits = []  # host time blocked on the G-buffer motion bound (BandRenderer._motion)
    orig_motion = D.BandRenderer._motion

    def timed_motion(self, *a):
        tw = time.perf_counter()
        n = orig_motion(self, *a)
        waits.append(time.perf_counter() - tw)
        return n
    D.BandRenderer._motion = timed_motion
    r.r.back_events = []
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(K):
        r.frame()
    issue = (time.perf_counter() - t0) / K
    cpu = (time.process_time() - c0) / K
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / K
    D.BandRenderer._motion = orig_motion
    wait = sum(waits) / K
    r.r.flush()
    torch.cuda.synchronize()
    ev = [(a, b) for a, b in r.r.back_events if b is not None]
    r.r.back_events = None
    # the SVGF stream: busy time per frame (start to end of each back end) and idle gaps between consecutive ones
    busy = [a.elapsed_time(b) for a, b in ev]
    gaps = [ev[i][1].elapsed_time(ev[i + 1][0]) for i in range(len(ev) - 1)]
    back_ms = sum(busy) / max(len(busy), 1)
    gap_ms = sum(max(0.0, g) for g in gaps) / max(len(gaps), 1)
    xbytes = sum(LOG) / K
    nex = len(LOG) / K
    counts = None
    if probe:
        c = torch.zeros(r.plan.y1 - r.plan.y0, dtype=torch.int32, device="cuda")
        r.pass_path_tracing.set_row_cost(c.data_ptr())
        r.frame()
        torch.cuda.synchronize()
        r.pass_path_tracing.set_row_cost(0)
        counts = c.cpu().numpy().astype(np.float64)
    if os.environ.get("STATS") == "1":  # traversal counters of this band (rays, node + triangle visits by kind)
        st = r.trace_stats()
        vis = st["primary_visits"] + st["bounce_visits"] + st["shadow_visits"]
        print(f"rank {rk} stats: visits {vis / 1e6:.1f} M ({vis / 1e9 / (wall):.1f} G visits/s at the band's wall) "
              f"{st}", flush=True)
    r.profile(True)
    r.frame()
    torch.cuda.synchronize()
    pp = r.pass_times()
    r.profile(False)
    y0, y1 = r.plan.y0, r.plan.y1
    r.close()
    return dict(y0=y0, y1=y1, wall=wall * 1e3, issue=issue * 1e3, gpu=pp["frame_sum_ms"], pp=pp, counts=counts,
                xbytes=xbytes, nex=nex, cpu=cpu * 1e3, wait=wait * 1e3, back=back_ms, gap=gap_ms)


def report(tag, res):
    print(f"--- {tag}: N={N} {W}x{H}")
    for rk, s in enumerate(res):
        print(f"rank {rk}: rows {s['y0']}..{s['y1']} ({s['y1'] - s['y0']}) wall {s['wall']:.3f} ms gpu {s['gpu']:.3f} "
              f"issue {s['issue']:.3f} (host cpu {s['cpu']:.3f}, motion wait {s['wait']:.3f})  SVGF stream busy "
              f"{s['back']:.3f} ms/frame, idle {s['gap']:.3f}  gbuf {s['pp'].get('gbuffer', 0):.3f} pt {s['pp'].get('pathtrace', 0):.3f} "
              f"svgf {s['gpu'] - s['pp'].get('gbuffer', 0) - s['pp'].get('pathtrace', 0):.3f}  halo {s['nex']:.0f}x "
              f"{s['xbytes'] / 1e6:.2f} MB")
    mx = max(s["wall"] for s in res)
    print(f"predicted frame (slowest rank, exchanges {XLAT_US:g} us + bytes / {XGBS:g} GB/s): {mx:.3f} ms = {1e3 / mx:.1f} fps; "
          f"sum of rank GPU times {sum(s['gpu'] for s in res):.3f} ms; sum of rank walls "
          f"{sum(s['wall'] for s in res):.3f} ms")
    return mx


if __name__ == "__main__":
    # calibration as in ptsvgf.dist.make_band_renderer: per-rank band time alone (frames in flight) + row visits,
    # band_row_cost per round, bounds from the mean of the rounds' estimates
    ranks = [int(v) for v in os.environ["RANKS"].split(",")] if "RANKS" in os.environ else range(N)
    bounds = tuple(int(v) for v in os.environ["BOUNDS"].split(",")) if "BOUNDS" in os.environ else None
    res = [sim_rank(rk, bounds, probe=True) for rk in ranks]
    plans = [(report("given bands" if bounds else "equal bands", res), "initial")]
    bounds = bounds or tuple(D.BandPlan(W, H, 0, N).bounds)
    est = []
    for rnd in range(int(os.environ.get("ROUNDS", "2")) if N > 1 and os.environ.get("BALANCE", "1") != "0" else 0):
        visits = np.concatenate([s["counts"] for s in res])
        est.append(D.band_row_cost(visits, bounds, [s["wall"] for s in res]))
        bounds = D.balanced_bounds(np.mean(est, axis=0), N)
        print("round %d bounds %s" % (rnd, bounds))
        res = [sim_rank(rk, bounds, probe=True) for rk in range(N)]
        plans.append((report(f"balanced bands (round {rnd})", res), bounds))
    # as make_band_renderer: the measured plan with the smallest slowest band wins
    best = min(plans, key=lambda x: x[0])
    print(f"best measured plan: {best[1]} slowest band {best[0]:.3f} ms = {1e3 / best[0]:.1f} fps")
    gl.shutdown()
