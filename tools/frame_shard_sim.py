"""Single-GPU prediction of an N-GPU frame-shard run (ptsvgf.dist.FrameShardRenderer), ranks simulated one by one.

Rank r of N traces every N-th frame whole (G-buffer + path tracer) and, every frame, draws its band's G-buffer and
SVGF chain. Here one rank's share runs alone on the GPU with the communication stood in for by spin kernels of the
modelled RCCL time (20 us + bytes / 50 GB/s by default, XLAT_US / XGBS to change):
  * the exchange of a window of N frames (exchange_window: this rank's traced frame to the N - 1 other bands, the
    other N - 1 frames' rows of this band from their ranks, all links at once): latency + the largest per-peer
    volume / bandwidth, on the receive stream (the window's SVGF chains wait for it);
  * the SVGF halo exchanges: as tools/band_sim.py.
The arrival of another rank's frame is not delayed by that rank's path tracer: the run measures a rank's throughput
(frames in flight cover the latency), not the latency itself. Prints each simulated rank's ms per frame; the
predicted N-GPU frame is the slowest rank.
SHARD=tiles simulates dist.TileShardRenderer instead: every rank traces the tiles k * N + rank of every frame, and one
all-to-all per frame (exchange_tiles: latency + the largest per-peer message / bandwidth, on the receive stream) carries
them to the band owners. Both modes report the camera-to-modulate latency (HIP events, Renderer.latency_ms) in ms and
in frames of the rank's rate.
Every rank is simulated ROTATIONS times (default 3) in rotated orders and reported by its median (round 6: a rank's
wall depends on its position in the one-process sequence by up to 30 %).
usage: python tools/frame_shard_sim.py [N] [W] [H]   (RANKS=0,3 to simulate a subset; FRAMES, OWN, K, SHARD, WINDOW, BURST,
TBATCH, ROTATIONS)"""
import os
import sys
import time

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PTSVGF_HW_QUEUES", "16")  # as bench.py
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
import torch

from ptsvgf import dist as D
from ptsvgf import gl
from ptsvgf.camera import parameter_config
from ptsvgf.scene import build_scene

N = int(sys.argv[1]) if len(sys.argv) > 1 else 8
W = int(sys.argv[2]) if len(sys.argv) > 2 else 3840
H = int(sys.argv[3]) if len(sys.argv) > 3 else 2160
XLAT_US = float(os.environ.get("XLAT_US", "20"))
XGBS = float(os.environ.get("XGBS", "50"))
_CYC_PER_US = None
LOG = {"halo": 0, "send": 0, "recv": 0}
SHARD = os.environ.get("SHARD", "frames")


class FakeDist:
    """Stands in for torch.distributed (the frame loop itself makes no host collective since round 5: the history rows
    come from the host's own bound, dist.MotionCheck; calibration all-reduces are no-ops here)."""
    class ReduceOp:
        MAX = "max"

    def get_backend(self, group=None):
        return "gloo"

    def all_reduce(self, t, op=None, group=None):
        return None


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
    torch.cuda._sleep(int(us * _CYC_PER_US))


def _xfer_us(nbytes):
    return XLAT_US + (nbytes / (XGBS * 1e3) if XGBS > 0 else 0.0)


class FakeWork:
    """A stood-in transfer running on the comm stream: wait() makes the current stream wait for it (as RCCL's)."""
    def __init__(self, ev):
        self.ev = ev

    def wait(self):
        torch.cuda.current_stream().wait_event(self.ev)


_COMM = None


def fake_exchange(items, plan, dist, group=None, wait=True):
    """halo_exchange stand-in: the transfers to / from each peer run over that peer's link at once, so a batch lasts
    latency + the largest per-peer volume / bandwidth. wait=True: on the current stream (it waits anyway);
    wait=False (the ghost zone's early history exchange): on a comm stream after the current stream's work, the
    caller's later wait() joins it, as RCCL's stream does."""
    global _COMM
    per_peer = {}
    for t, n in items:
        if plan.world == 1 or n <= 0:
            continue
        row = t.shape[1] * t.shape[2] * 4
        for send, a, b, k in plan.halo_parts(n):
            per_peer[(send, k)] = per_peer.get((send, k), 0) + row * (b - a)
    if not per_peer:
        return []
    LOG["halo"] += sum(v for (snd, _), v in per_peer.items() if snd)
    us = _xfer_us(max(per_peer.values()))
    if wait:
        _spin(us)
        return []
    if _COMM is None:
        _COMM = torch.cuda.Stream()
    start = torch.cuda.Event()
    start.record()
    _COMM.wait_event(start)
    with torch.cuda.stream(_COMM):
        _spin(us)
    done = torch.cuda.Event()
    done.record(_COMM)
    return [FakeWork(done)]


def fake_window(window, plan, dist, group=None, rows=None):
    """exchange_window stand-in: the window's sends and receives run over all links at once, so the batch lasts
    latency + the largest per-peer volume (sent to or received from one peer) / link bandwidth."""
    per_peer, sent = {}, 0
    for src, planes in window:
        if src == plan.rank:
            for k in range(plan.world):
                if k != plan.rank:
                    nb = sum(t[slice(*(rows[j] if rows else plan.zone)(k))].numel() * 4 for j, t in enumerate(planes))
                    per_peer[("s", k)] = per_peer.get(("s", k), 0) + nb
                    sent += nb
        else:
            nb = sum(t.numel() * 4 for t in planes)
            per_peer[("r", src)] = per_peer.get(("r", src), 0) + nb
            LOG["recv"] += nb
    LOG["send"] += sent
    if per_peer:
        _spin(_xfer_us(max(per_peer.values())))
    return sent


def fake_tiles(send, sends, recv, recvs, dist, group=None):
    """exchange_tiles stand-in: every peer's message over its own link at once: latency + the largest one."""
    per_peer = {}
    for k, a, b in sends:
        per_peer[("s", k)] = (b - a) * 4
    for k, a, b in recvs:
        per_peer[("r", k)] = (b - a) * 4
        LOG["recv"] += (b - a) * 4
    sent = sum(v for (d, _), v in per_peer.items() if d == "s")
    LOG["send"] += sent
    if per_peer:
        _spin(_xfer_us(max(per_peer.values())))
    return sent


D.halo_exchange = fake_exchange
D.exchange_window = fake_window
D.exchange_tiles = fake_tiles
D.scatter_group = lambda dist: None
torch.cuda.set_device(0)
gl.init(0)
from ptsvgf._lib import check, pt  # noqa: E402

check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
scene = build_scene("table_clock_plant")
cfg = parameter_config()
FRAMES = int(os.environ.get("FRAMES", str(max(96, 24 * N))))
OWN = int(os.environ.get("OWN", "4"))
K = int(os.environ.get("K", str(max(16, 4 * N + 2) if SHARD == "frames" else 8)))  # bench.py's defaults


def sim_rank(rk, bounds=None):
    if SHARD == "tiles":
        r = D.TileShardRenderer(scene, W, H, cfg, rk, N, FakeDist(), own_slots=OWN, frames_in_flight=K, bounds=bounds,
                                batch=int(os.environ.get("TBATCH", "1")))
    else:
        r = D.FrameShardRenderer(scene, W, H, cfg, rk, N, FakeDist(), own_slots=OWN, frames_in_flight=K,
                                 bounds=bounds, ship_gbuffer=os.environ.get("SHIP", "0") == "1",
                                 window=int(os.environ.get("WINDOW", "0")) or None,
                                 burst=int(os.environ.get("BURST", "1")))
    r.camera.frameCounter += int(os.environ.get("FC_OFFSET", "0"))  # experiment: which frames a rank traces
    for kv in filter(None, os.environ.get("PT_UNIFORMS", "").split(",")):  # name=value,... on the path tracer
        name, val = kv.split("=")
        r.pass_path_tracing.set_uniform_int(name, int(val))
    rr = r.r  # SVGF_UNIFORMS=name:value;...: on the band's SVGF draws (as bench.py --svgf-uniform)
    for kv in filter(None, os.environ.get("SVGF_UNIFORMS", "").split(";")):
        name, val = kv.split(":")
        for sp in [*rr.reproject, rr.variance_compute_pass, *rr.atrous_to.values(), *rr.atrous_mod_to.values(),
                   rr.svgf_modulate_pass]:
            sp.set_uniform_int(name, int(val))
    for _ in range(2 * K + N):  # every band slot and own slot used before timing (first use allocates)
        r.frame()
    r.r.flush()
    torch.cuda.synchronize()
    for k in LOG:
        LOG[k] = 0
    r.r.back_events = []
    r.r.latency_events = []
    if hasattr(r, "own_events"):
        r.own_events = []
    # host time in BandRenderer._motion (round 4: a wait for the G-buffer's bound + the per-frame all-reduce; round 5:
    # the host's own bound, MotionCheck) and in the host pacing (Renderer host_pace: frame f waits for SVGF(f - K))
    waits = []
    pace0 = r.r.pace_wait_s
    orig_motion = D.BandRenderer._motion

    def timed_motion(self, *a):
        tw = time.perf_counter()
        n = orig_motion(self, *a)
        waits.append(time.perf_counter() - tw)
        return n
    D.BandRenderer._motion = timed_motion
    torch.arange(3, device="cuda")  # kernel-trace marker: the timed frames start (tools/launch_diff.py)
    t0 = time.perf_counter()
    c0 = time.process_time()
    for _ in range(FRAMES):
        r.frame()
    issue = (time.perf_counter() - t0) / FRAMES
    cpu = (time.process_time() - c0) / FRAMES
    torch.cuda.synchronize()
    wall = (time.perf_counter() - t0) / FRAMES
    torch.arange(3, device="cuda")  # kernel-trace marker: the timed frames have ended
    pace = (r.r.pace_wait_s - pace0) / FRAMES
    D.BandRenderer._motion = orig_motion
    r.r.flush()
    torch.cuda.synchronize()
    own = {}
    if getattr(r, "own_events", None):
        # the rank's own front ends (G-buffer + path tracer of a whole frame): their span on the GPU and how much of the
        # time two or more of them ran at once
        ref = r.own_events[0][1]
        iv = [(ref.elapsed_time(a), ref.elapsed_time(b)) for _, a, b in r.own_events]
        spans = [b - a for a, b in iv]
        pts = sorted([(a, 1) for a, _ in iv] + [(b, -1) for _, b in iv])
        cur, last, t2, tany = 0, None, 0.0, 0.0
        for t, dlt in pts:
            if last is not None:
                tany += (t - last) if cur >= 1 else 0.0
                t2 += (t - last) if cur >= 2 else 0.0
            cur += dlt
            last = t
        own = dict(own_span=sum(spans) / len(spans), own_n=len(spans), own_busy_frac=tany / (pts[-1][0] - pts[0][0]),
                   own_overlap_frac=t2 / max(tany, 1e-9))
        r.own_events = None
    ev = [(a, b) for a, b in r.r.back_events if b is not None]
    r.r.back_events = None
    busy = sum(a.elapsed_time(b) for a, b in ev) / max(len(ev), 1)
    lat = r.r.latency_ms()
    r.r.latency_events = None
    r.profile(True)  # the band's passes alone (a draw at a time, synchronised): the floor of its SVGF stream
    for _ in range(N):
        r.frame()
    r.r.flush()
    torch.cuda.synchronize()
    pp = r.pass_times()
    r.profile(False)
    out = dict(rows=(r.plan.y0, r.plan.y1), wall=wall * 1e3, issue=issue * 1e3, cpu=cpu * 1e3, back=busy,
               wait=sum(waits) / FRAMES * 1e3, pace=pace * 1e3, pp={k: v / N for k, v in pp.items()}, latency=lat,
               halo_mb=LOG["halo"] / FRAMES / 1e6, send_mb=LOG["send"] / FRAMES / 1e6,
               recv_mb=LOG["recv"] / FRAMES / 1e6, **own)
    r.close()
    return out


def report(tag, ranks, bounds):
    """Simulate every rank of `ranks` ROTATIONS times (default 3), each pass in a rotated order, so each rank runs at
    several positions of the sequence (a rank's wall varies up to +-30 % with its position in it); per rank
    the median of its passes, the predicted frame = the slowest rank's median."""
    rot = max(1, int(os.environ.get("ROTATIONS", "3")))
    print(f"--- {SHARD} shard ({tag}): N={N} {W}x{H} K={K} own slots {OWN} window {os.environ.get('WINDOW') or N} "
          f"burst {os.environ.get('BURST', '1')} tile batch {os.environ.get('TBATCH', '1')}, "
          f"{FRAMES} frames per rank, {rot} rotation(s) of the rank order, "
          f"links {XLAT_US:g} us + bytes / {XGBS:g} GB/s", flush=True)
    step = max(1, len(ranks) // rot)
    runs = {rk: [] for rk in ranks}
    for j in range(rot):
        order = ranks[(j * step) % len(ranks):] + ranks[:(j * step) % len(ranks)]
        for pos, rk in enumerate(order):
            s = sim_rank(rk, bounds)
            s["pos"] = pos
            runs[rk].append(s)
            print(f"rotation {j} pos {pos} rank {rk}: rows {s['rows'][0]}..{s['rows'][1]} wall {s['wall']:.3f} ms/frame "
                  f"({1e3 / s['wall']:.1f} fps) issue {s['issue']:.3f} (host cpu {s['cpu']:.3f}, motion {s['wait']:.3f}, "
                  f"pace wait {s['pace']:.3f})  SVGF stream busy {s['back']:.3f} ms/frame  per frame: "
                  f"halo {s['halo_mb']:.2f} MB, sent {s['send_mb']:.1f} MB, received {s['recv_mb']:.1f} MB; "
                  f"camera-to-modulate {s['latency']:.2f} ms = {s['latency'] / s['wall']:.1f} frames", flush=True)
            print("   passes alone, ms per frame: " + " ".join(f"{k} {v:.3f}" for k, v in sorted(s["pp"].items())),
                  flush=True)
            if "own_span" in s:
                print(f"   own front ends: {s['own_n']}, span {s['own_span']:.3f} ms each, one or more running "
                      f"{s['own_busy_frac']:.0%} of the time, two or more {s['own_overlap_frac']:.0%} of that", flush=True)
    res = []
    for rk in ranks:
        walls = sorted(s["wall"] for s in runs[rk])
        med = walls[len(walls) // 2]
        s = dict(min(runs[rk], key=lambda x: abs(x["wall"] - med)))  # the median run's other figures
        s["wall"] = med
        s["walls"] = [round(x["wall"], 3) for x in runs[rk]]
        res.append(s)
        print(f"rank {rk}: median wall {med:.3f} ms/frame over positions "
              f"{[x['pos'] for x in runs[rk]]}: {s['walls']}", flush=True)
    mx = max(s["wall"] for s in res)
    lat = max(s["latency"] for s in res)
    print(f"predicted frame (slowest rank's median): {mx:.3f} ms = {1e3 / mx:.1f} fps; latency (largest) {lat:.2f} ms "
          f"= {lat / mx:.1f} frames", flush=True)
    return res


if __name__ == "__main__":
    import numpy as np

    ranks = [int(v) for v in os.environ["RANKS"].split(",")] if "RANKS" in os.environ else list(range(N))
    given = tuple(int(v) for v in os.environ["BOUNDS"].split(",")) if "BOUNDS" in os.environ else None
    res = report("given bands" if given else "equal bands", ranks, given)
    if os.environ.get("BALANCE", "1") != "0" and len(ranks) == N and N > 1 and given is None:
        # make_frame_shard_renderer's calibration, one round: each band's work (its own passes, timed alone) spread
        # evenly over its rows, new bounds at equal quantiles
        b = D.BandPlan(W, H, 0, N).bounds
        cost = np.empty(H)
        for k, s in enumerate(res):
            work = s["pp"].get("frame_sum_ms", 0.0)  # the band renderer's own draws (full_* are the whole frame's)
            cost[b[k]:b[k + 1]] = work / (b[k + 1] - b[k])
        bounds = D.balanced_bounds(cost, N)
        print(f"balanced bounds {bounds}", flush=True)
        report("balanced bands", ranks, bounds)
    gl.shutdown()
