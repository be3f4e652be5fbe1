"""GPU band rendering: several ranks on the one visible GPU (gloo with host
staging — RCCL needs one device per rank, which the driver's 8-GPU scaling run
provides) render frames as bands with ptsvgf.dist.BandRenderer; the owned rows
must equal the single-GPU full-frame render bit for bit.

The 8-rank case is BASELINE configs[3]/[4] on one GPU: the bench scene at 4K,
equal 270-row bands, 8 frames in flight, TAA on, and a camera that moves up to
~35 rows per frame near the frame edges (where the band boundaries at rows 270
and 1890 sit), so the history exchanges are sized by the per-frame motion bound
(ptsvgf.dist.MotionCheck: the host's bound, verified against the device's) far beyond round 1's fixed 8 rows."""
import os
import socket
import tempfile

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

W, H, FRAMES = 64, 96, 3
KEYS = ("color", "albedo", "reproj_illum", "variance", "atrous", "modulate", "final")


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, outdir, moving, balance, fif=1, size=(W, H), bench_scene=False, moves=None, batch=1):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ptsvgf import gl
    from ptsvgf._lib import check, pt
    from ptsvgf.camera import parameter_config
    from ptsvgf.dist import make_band_renderer
    from ptsvgf.scene import build_scene
    torch.cuda.set_device(0)
    gl.init(0)
    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    scene = _scene(bench_scene)
    Wf, Hf = size
    r = make_band_renderer(scene, Wf, Hf, parameter_config(), rank, world, dist, balance=balance, run_taa=True,
                           frames_in_flight=fif, trace_batch=batch)
    for f in range(len(moves) if moves else FRAMES):
        mv = moves[f] if moves else ((1.5, 0.5) if moving and f else None)
        if mv:
            r.camera.orbit(*mv)
        r.frame()
    torch.cuda.synchronize()
    p = r.plan
    out = {k: gl.readback(r.planes()[k])[p.y0 - p.row0:p.y1 - p.row0] for k in KEYS}
    np.savez(os.path.join(outdir, f"rank{rank}.npz"), y0=p.y0, y1=p.y1, motion=np.array(r.motion_log), **out)
    gl.shutdown()
    dist.destroy_process_group()


def _scene(bench):
    from ptsvgf.scene import build_scene
    if bench:
        return build_scene("table_clock_plant")  # the bench scene, full size
    return build_scene("table_clock_plant", hdr_size=(256, 128), plant_leaves=40)


def _compare(bands, want):
    for b in bands:
        y0, y1 = int(b["y0"]), int(b["y1"])
        for k in KEYS:
            bad = np.argwhere(np.any(b[k].view(np.uint32) != want[k][y0:y1].view(np.uint32), axis=-1))
            if len(bad):
                rows = sorted(set(int(r) + y0 for r in bad[:, 0]))
                print(k, "band", (y0, y1), "differing rows", rows[:20], "count", len(bad),
                      "sample", b[k][tuple(bad[0])], want[k][y0:y1][tuple(bad[0])])
            assert len(bad) == 0, (k, y0, y1)


@pytest.mark.parametrize("moving,balance,fif,batch", [(False, False, 1, 1), (True, False, 1, 1), (True, True, 1, 1),
                                                      (True, True, 3, 1), (True, True, 4, 4)])
def test_two_bands_equal_full_frame(gpu, moving, balance, fif, batch):
    import torch.multiprocessing as mp

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer
    from ptsvgf.scene import build_scene

    gl = gpu
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(2, _port(), d, moving, balance, fif, (W, H), False, None, batch), nprocs=2, join=True)
        bands = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(2)]
    scene = build_scene("table_clock_plant", hdr_size=(256, 128), plant_leaves=40)
    full = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=True,
                    run_output=False)
    for f in range(FRAMES):
        if moving and f:
            full.camera.orbit(1.5, 0.5)
        full.frame()
    want = {k: gl.readback(full.planes()[k]) for k in KEYS}
    full.close()
    _compare(bands, want)


MOVES_4K = [None, (1.0, 0.75), (-1.5, -1.0), (0.5, 1.5)]


def test_eight_bands_4k_moving_equal_full_frame(gpu):
    """8 ranks x 270 rows of the 4K bench frame, frames in flight, TAA, moving camera: bit-equal to one GPU."""
    import torch.multiprocessing as mp

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer

    gl = gpu
    Wf, Hf, world = 3840, 2160, 8
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_worker, args=(world, _port(), d, True, False, 8, (Wf, Hf), True, MOVES_4K), nprocs=world,
                 join=True)
        bands = [dict(np.load(os.path.join(d, f"rank{r}.npz"))) for r in range(world)]
    motion = bands[0]["motion"]
    print("history rows each frame's measured motion needs, rows exchanged (host bound):", motion.tolist())
    assert motion[:, 0].max() > 30  # the camera really moved past round 1's 8 rows of history
    assert np.all(motion[:, 0] <= motion[:, 1])  # MotionCheck verified every frame's device bound
    full = Renderer(_scene(True), Wf, Hf, parameter_config(), mode="fast", aspect_corrected=True, run_taa=True,
                    run_output=False)
    for mv in MOVES_4K:
        if mv:
            full.camera.orbit(*mv)
        full.frame()
    want = {k: gl.readback(full.planes()[k]) for k in KEYS}
    full.close()
    _compare(bands, want)


def _p2p_worker(rank, world, port, outdir, window, burst, K, frames):
    import json
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    import torch
    import torch.distributed as dist
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    from ptsvgf import gl
    from ptsvgf._lib import check, pt
    from ptsvgf.camera import parameter_config
    from ptsvgf.dist import FrameShardRenderer, P2PRecorder
    torch.cuda.set_device(0)
    gl.init(0)
    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    D = P2PRecorder(dist)
    r = FrameShardRenderer(_scene(False), 320, 256, parameter_config(), rank, world, D, own_slots=max(2, burst),
                           frames_in_flight=K, window=window, burst=burst)
    D.frame_of = lambda: r.r.frame_index
    for f in range(frames):
        if f >= 3:  # static frames (3-row history reach), then an orbit (the ghost zone's capacity rows)
            r.camera.orbit(1.0, 0.5)
        r.frame()
    r.planes()  # flush: the last window is cut short; every frame's device motion bound verified
    torch.cuda.synchronize()
    r.close()
    logs = [None] * world
    dist.all_gather_object(logs, D.log)
    if rank == 0:
        with open(os.path.join(outdir, "logs.json"), "w") as fh:
            json.dump(logs, fh)
    gl.shutdown()
    dist.destroy_process_group()


@pytest.mark.parametrize("world,window,burst", [(3, 3, 1), (3, 2, 2), (4, 4, 1)])
def test_frame_shard_p2p_issue_order(gpu, world, window, burst):
    """the real FrameShardRenderer's point-to-point traffic over its two communicators — the history
    exchange (halo_exchange on WORLD, issued early on the SVGF stream) and the window exchange (exchange_window on
    scatter_group, on the receive stream) — logged per rank (dist.P2PRecorder) through static and moving frames, full
    windows, a window cut short by flush() and bursts: for every pair of ranks the batches, groups, call sites and
    byte counts match in issue order (dist.check_p2p_logs). gloo's blocking wait() hides a stream dependency RCCL would
    need, but not an issue order that differs between ranks: that is what this checks, for the 8-GPU RCCL run."""
    import json

    import torch.multiprocessing as mp

    from ptsvgf.dist import check_p2p_logs

    frames = 3 * window + 2  # the last window holds 2 frames: cut short by flush()
    with tempfile.TemporaryDirectory() as d:
        mp.spawn(_p2p_worker, args=(world, _port(), d, window, burst, 2 * window + 4, frames), nprocs=world, join=True)
        with open(os.path.join(d, "logs.json")) as fh:
            logs = json.load(fh)
    bad = check_p2p_logs(logs)
    assert not bad, bad[:4]
    calls = {(site, g) for log in logs for site, g, _, _ in log}
    assert calls == {("halo_exchange", "world"), ("exchange_window", "scatter")}, calls
    windows = [sum(1 for site, *_ in log if site == "exchange_window") for log in logs]
    assert min(windows) >= 3, windows
    hist = [n for site, g, f, ops in logs[0] if site == "halo_exchange" for _, _, n in ops]
    assert len(set(hist)) > 1, "static and moving frames exchange different history rows"
