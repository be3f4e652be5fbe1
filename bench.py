#!/usr/bin/env python3
"""Headline benchmark: frames/s of 1 spp path tracing + 5-iteration SVGF on the
table+clock+plant scene (BASELINE.json metric / configs[2]: 3840x2160, 1x MI355X),
plus the a-trous kernel's achieved HBM GB/s against the 8 TB/s roofline.

A "step" is one frame of the hot path: G-buffer, path tracer (depth 2, NEE),
reprojection, variance, 5 a-trous iterations, modulate (TAA and
the output tonemap are excluded there and excluded here). Inputs (scene, BVH,
environment) are resident in HBM before timing starts; the camera orbits by a
fixed step each frame only with --moving.

`value` is the pipelined rate (frames_in_flight front ends overlap);
the line also carries the serial rate (one frame at a time: camera-to-display
latency of one frame), 1080p (configs[1]), the path tracer's rays/s and BVH
visits/s, a surface-dominated view, the a-trous roofline three ways (SURVEY.md's
52 B/px convention, PMC traffic, background-weighted bytes), the CPU oracle on
every usable core and on 1 core, configs[0] (Cornell box + teapot 512x512, SVGF off,
CPU reference traversal), and the dynamic-scene path (GPU LBVH rebuild time, frame
rate over the LBVH).

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
every rank owns one horizontal band of the frame for the SVGF chain and exchanges
its halo rows with the other bands over RCCL (ptsvgf.dist); the G-buffer + path
tracer of frame f run over the whole frame on rank f % N, which sends each band's
rows of colour / emission / albedo to its owner (--shard frames, the default), or
every rank traces its own band of every frame (--shard bands), or the 16x16 tiles
k*N + rank of every frame (--shard tiles). The frame sequence is fixed and N ranks
render it together; "scaling" is "throughput" for --shard frames (frames/s scale,
a frame's camera-to-modulate latency does not: see "latency") and "strong" for
tiles / bands (every frame is split).
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

REPO = os.path.dirname(os.path.abspath(__file__))
# frames in flight use K + 1 streams (K front ends + the SVGF back end; 3K + 1 with the optional G-buffer and
# closest-hit side streams); HIP's default of 4 hardware queues per process would make streams share queues
# and serialise. Set before HIP initialises; the GPU box exports GPU_MAX_HW_QUEUES=4, so it is overridden (PTSVGF_HW_QUEUES to choose).
os.environ["GPU_MAX_HW_QUEUES"] = os.environ.get("PTSVGF_HW_QUEUES", "16")
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

ATROUS_BYTES_PER_PX = 52     # illum 16 + normal/z 16 + depth-fwidth 4 + write 16
ATROUS_BYTES_BG_PX = 36      # a background pixel: depth-fwidth/flag 4 + illum 16 + write 16 (copied)
HBM_PEAK_GBS = 8000.0        # MI355X_MICROARCH.md: 8 TB/s spec
METRIC = "frames/sec @1spp+SVGF, 1080p & 4K; à-trous HBM GB/s vs peak"  # BASELINE.json "metric"
ATROUS_KERNEL = "atrous_tile_kernel"
EXCHANGE_STAGES = ("history", "reproject", "variance", "atrous0", "atrous1", "atrous2", "atrous3", "atrous4", "taa")
# planes compared bitwise between the gathered bands and the one-GPU frame (--gpus N > 1)
PARITY_PLANES = ("color", "albedo", "reproj_illum", "variance", "history_illum", "atrous", "modulate")
# HBM bytes per a-trous launch measured with rocprofv3 PMC passes (tools/gpu_profile.sh), committed under profiles/,
# one file per camera view (the surface view's bytes are its own, not the default view's)
TRAFFIC_FILE = os.path.join(REPO, "profiles", "atrous_traffic_{view}.json")
# configs[2] on a surface-dominated camera (94 % geometry pixels: the plant, a corner of the clock; ~24 % on the
# default view): orbit radius, elevation, azimuth and look-at point (Utils/camera.h:14-38 parameters)
VIEWS = {"default": None, "surface": dict(r_dis=0.8, upAngle=70.0, rotatAngle=180.0, move_vec=(0.4, -0.25, 0.0))}


def atrous_traffic(W, rows, view="default"):
    """PMC-measured HBM bytes per a-trous launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, in KB units as the
    guide prescribes) from the committed profile, when it was taken for this kernel at this frame size on this
    camera view AND of the machine code this process loaded (tools/kernel_hash.py: the a-trous tile kernel's
    instruction bytes in the library, stable across rebuilds); (bytes or None, provenance)."""
    try:
        with open(TRAFFIC_FILE.format(view=view)) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None, {"profile": None}
    prov = {"profile": t.get("source"), "profile_code_sha256": t.get("code_sha256")}
    if t.get("kernel") != ATROUS_KERNEL or t.get("pixels") != W * rows or t.get("view") != view:
        return None, dict(prov, reason="profile of another kernel, frame size or view")
    try:
        sys.path.insert(0, os.path.join(REPO, "tools"))
        from kernel_hash import kernel_code_hash
        from ptsvgf._lib import LIB_DIR
        lib = os.path.join(os.environ.get("PTSVGF_LIB_DIR", LIB_DIR), "libptsvgf.so")
        prov["loaded_code_sha256"] = kernel_code_hash(lib, ATROUS_KERNEL)
    except Exception as e:  # noqa: BLE001 - a failed identity check reports no traffic, never a stale one
        return None, dict(prov, reason=f"code hash failed: {e}")
    if not t.get("code_sha256") or t["code_sha256"] != prov["loaded_code_sha256"]:
        return None, dict(prov, reason="stale: the profile measured other a-trous machine code")
    return t.get("bytes_per_launch"), prov


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--scene", default="table_clock_plant")
    ap.add_argument("--view", default="default", choices=sorted(VIEWS), help="camera of the headline run")
    ap.add_argument("--moving", action="store_true", help="orbit the camera 1 deg/frame (configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="960x540", help="oracle sample frame size for cpu_baseline (all cores)")
    ap.add_argument("--cpu-sample-1core", default="480x270", help="oracle sample frame size on 1 core")
    ap.add_argument("--no-1080p", action="store_true", help="skip the secondary 1080p measurement")
    ap.add_argument("--no-extras", action="store_true", help="skip the serial, surface-view and configs[0] runs")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for --gpus > 1 (nccl = RCCL)")
    ap.add_argument("--no-band-parity", action="store_true",
                    help="multi-GPU: skip the untimed bitwise check of the gathered bands against a one-GPU frame")
    ap.add_argument("--equal-bands", type=int, default=None, choices=(0, 1),
                    help="multi-GPU: 1 = equal band heights (no balancing of the measured band work); default 1 for "
                         "the frame shard on 2 ranks (simulated 357 vs 337 fps at 4K, "
                         "profiles/r05/shard/sim_n2_own4_k12.log), else 0")
    ap.add_argument("--shard", default="frames", choices=("frames", "tiles", "bands"),
                    help="multi-GPU: 'frames' = rank f %% N traces frame f whole and scatters its rows to the band owners, "
                         "the SVGF chain banded (dist.FrameShardRenderer); 'tiles' = every rank traces the 16x16 tiles "
                         "k*N + rank of every frame, one all-to-all per frame to the band owners, the SVGF chain banded "
                         "(dist.TileShardRenderer); 'bands' = every pass banded (dist.BandRenderer)")
    ap.add_argument("--window", type=int, default=None,
                    help="--shard frames: frames whose rows travel in one exchange, = back_lag (default min(N, 4); N: one "
                         "all-to-all per N frames; 1: one-to-all per frame)")
    ap.add_argument("--tile-batch", type=int, default=1,
                    help="--shard tiles: the subsets of this many consecutive frames traced as one batched draw and "
                         "exchanged together (back_lag max(2, B))")
    ap.add_argument("--burst", type=int, default=1,
                    help="--shard frames: consecutive frames one rank traces (frame f on rank (f // burst) %% N)")
    ap.add_argument("--ship-gbuffer", type=int, default=0, choices=(0, 1),
                    help="--shard frames: the tracing rank also sends the bands their G-buffer rows (they draw none)")
    ap.add_argument("--own-slots", type=int, default=None,
                    help="--shard frames / tiles: whole frames / tile subsets a rank traces at once (its path tracer's "
                         "frames in flight); default 2 above 4 ranks, 3 for 3-4, 4 for 2 (4K simulation, "
                         "profiles/r05/shard/, ms per frame for 2 / 3 / 4 slots: 8 ranks K 16 0.856-0.863 / 0.948 / "
                         "0.879; 4 ranks K 12 1.659 / 1.477 / 1.529; 2 ranks K 12 3.851 / - / 2.967)")
    ap.add_argument("--host-pace", type=int, default=1, choices=(0, 1),
                    help="one GPU: the host waits for frame f - K's SVGF before issuing frame f (Renderer host_pace): "
                         "camera-to-modulate 36 -> 18 ms at 4K, same frame rate (profiles/r04/pace/)")
    ap.add_argument("--breakdown", action="store_true", help="print per-pass ms to stderr")
    ap.add_argument("--pt-kernel", type=int, default=0, help="0 wavefront (production), 1 megakernel (A/B)")
    ap.add_argument("--trace-batch", type=int, default=None,
                    help="path tracers of this many frames drawn as one batch (default 1)")
    ap.add_argument("--frames-in-flight", type=int, default=None,
                    help="K > 1: front ends (G-buffer + path tracer) of K frames overlap on K streams "
                         "(default 4 up to 4 GPUs, 8 on 8 bands: thinner bands have relatively longer launch tails)")
    ap.add_argument("--svgf-uniform", action="append", default=[], metavar="NAME=INT",
                    help="extra int uniform on the SVGF passes (A/B switches, e.g. reproj_block=0)")
    ap.add_argument("--fuse-modulate", type=int, choices=(0, 1), default=1,
                    help="1: the last a-trous iteration writes the modulated colour too (Renderer.fuse_modulate); "
                         "0: the separate modulate pass (A/B)")
    ap.add_argument("--pt-uniform", action="append", default=[], metavar="NAME=INT",
                    help="extra int uniform on the path-tracing pass (A/B switches, e.g. shadow_bvh4=0)")
    return ap.parse_args()


def log(msg: str) -> None:
    """Progress on stderr (the JSON line is the only stdout)."""
    print(f"[bench {time.strftime('%H:%M:%S')}] {msg}", file=sys.stderr, flush=True)


def oracle_fps(scene, W, H, threads, seconds, svgf=True):
    """Frames/s of the CPU oracle (the reference algorithm restated, OpenMP over rows) on a W x H frame: the whole
    frame loop (G-buffer + PT + SVGF), or the path tracer alone (svgf=False)."""
    import oracle_ref as O
    from ptsvgf.camera import parameter_config, rigid_inverse

    loop = O.OracleFrameLoop(scene, W, H, parameter_config(), aspect_corrected=W != H, threads=threads, run_taa=False)

    def frame():
        if svgf:
            loop.frame()
            return
        cam = loop.camera
        cam.update()
        loop.os.path_trace(W, H, cam.frameCounter, cam.cam_position, rigid_inverse(cam.cam_view_mat),
                           aspect_corrected=loop.aspect_corrected, threads=threads)
        cam.frameCounter += 1

    frame()  # warm (first frame: young history, full 7x7 variance)
    t0 = time.perf_counter()
    n = 0
    while True:
        frame()
        n += 1
        if time.perf_counter() - t0 > seconds and n >= 3:
            break
    return n / (time.perf_counter() - t0), n


def host_cpus() -> dict:
    """The host's CPUs as this process sees them: nproc (affinity), the machine's count, the cgroup CPU quota and
    lscpu's model line; `usable` = every core this process may run on at once (affinity, capped by the quota)."""
    import subprocess

    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
            quota = None if q == "max" else float(q) / float(per)
    except (OSError, ValueError):
        pass
    model = None
    try:
        out = subprocess.run(["lscpu"], capture_output=True, text=True, timeout=10).stdout
        model = next((ln.split(":", 1)[1].strip() for ln in out.splitlines() if ln.startswith("Model name")), None)
    except (OSError, subprocess.SubprocessError):
        pass
    usable = aff if quota is None else max(1, min(aff, int(quota)))
    # the GPU pool gives a one-GPU box a CPU share and exports it as OMP_NUM_THREADS (16): worker pools stay
    # within it, so the baseline's "all cores" are the cores of that share
    share = os.environ.get("OMP_NUM_THREADS")
    if share and share.isdigit() and int(share) > 0:
        usable = min(usable, int(share))
    return {"nproc": aff, "machine_cpus": os.cpu_count(), "cgroup_cpu_quota": quota, "omp_num_threads": share,
            "lscpu_model": model, "usable": usable}


def cpu_baseline(scene, W, H, sample: str, sample1: str):
    """The CPU oracle on a bounded sample frame (every usable host core, and 1 core), scaled to W x H by pixel
    count (all host cores, nproc / lscpu recorded)."""
    out = {}
    hc = host_cpus()
    for key, smp, threads in (("all", sample, hc["usable"]), ("one", sample1, 1)):
        sw, sh = (int(v) for v in smp.split("x"))
        fps, n = oracle_fps(scene, sw, sh, threads, 10.0)
        scale = (W * H) / (sw * sh)
        out[key] = {"value": fps / scale, "unit": "frames/s", "cores": threads, "kind": "port",
                    "sample": f"oracle frame loop (G-buffer+PT+SVGF) at {sw}x{sh} on {threads} thread(s), {n} frames, "
                              f"{1e3 / fps:.1f} ms/frame, scaled by pixel count to {W}x{H}"}
    line = dict(out["all"])
    line["single_core"] = out["one"]
    line["host"] = hc
    return line


def config0(gl):
    """configs[0]: Cornell box + teapot stand-in, 512x512, 1 spp, SVGF off — the CPU reference traversal (oracle
    path tracer, all usable cores and 1 core), with the GPU path tracer's rate on the same frame beside it."""
    import torch

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer
    from ptsvgf.scene import build_scene

    from ptsvgf._lib import check, pt

    check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
    scene = build_scene("cornell_teapot")
    res = {"workload": "cornell_teapot 512x512 1spp depth2, SVGF off", "triangles": scene.ntris}
    for key, threads in (("cpu_fps_all_cores", host_cpus()["usable"]), ("cpu_fps_1t", 1)):
        fps, n = oracle_fps(scene, 512, 512, threads, 4.0, svgf=False)
        res[key] = round(fps, 3)
    r = Renderer(scene, 512, 512, parameter_config(), mode="fast", run_taa=False, run_output=False)
    for _ in range(3):
        r._path_trace()
        r.camera.frameCounter += 1
    torch.cuda.synchronize()
    n = 200
    t0 = time.perf_counter()
    for _ in range(n):
        r._path_trace()
        r.camera.frameCounter += 1
    torch.cuda.synchronize()
    res["gpu_pt_fps"] = round(n / (time.perf_counter() - t0), 1)
    r.close()
    return res


def dynamic_bvh(scene, W, H, K, steps, warmup, host_ms):
    """SURVEY.md §8(f)2, dynamic scenes: the GPU builder (pt_bvh_build) rebuilding the path tracer's BVH in place —
    a plain LBVH (leaves of <= 8) and with the PLOC-built top (leaves of <= 3, radius 32) — median device and host-wall ms of 10 rebuilds against the
    host SAH build of the same triangles, a rebuild plus the frame that decodes it against a frame alone, and the
    frame rate of the headline configuration rendered over the GPU-built tree instead of the reference's SAH tree."""
    import numpy as np
    import torch

    from ptsvgf.camera import parameter_config
    from ptsvgf.renderer import Renderer

    out = {"triangles": scene.ntris, "host_sah_build_ms": round(host_ms, 1) if host_ms else None}
    for name, leaf_n, radius in (("lbvh", 8, 0), ("ploc", 3, 32)):
        r = Renderer(scene, W, H, parameter_config(), mode="fast", aspect_corrected=True, run_taa=False,
                     run_output=False, frames_in_flight=K)
        dev, wall, nodes, upd, plain = [], [], 0, [], []
        for _ in range(10):
            t0 = time.perf_counter()
            nodes, ms = r.rebuild_bvh(leaf_n=leaf_n, ploc_radius=radius)
            wall.append((time.perf_counter() - t0) * 1e3)
            dev.append(ms)
            r.frame()  # the first draw over the new buffers decodes them (capi get_scene)
            torch.cuda.synchronize()
            upd.append((time.perf_counter() - t0) * 1e3)
        for _ in range(10):
            t0 = time.perf_counter()
            r.frame()
            torch.cuda.synchronize()
            plain.append((time.perf_counter() - t0) * 1e3)
        for _ in range(warmup):
            r.frame()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(steps):
            r.frame()
        torch.cuda.synchronize()
        fps = steps / (time.perf_counter() - t0)
        moved = []  # geometry moved: the path tracer's tree and the K + 1 G-buffer passes' trees, all on the GPU
        for _ in range(5):
            t0 = time.perf_counter()
            r.rebuild_bvh(tri_enc=scene.tri_enc, raster=scene.raster, leaf_n=leaf_n, ploc_radius=radius)
            r.frame()
            torch.cuda.synchronize()
            moved.append((time.perf_counter() - t0) * 1e3)
        r.close()
        out[name] = {"leaf_n": leaf_n, "ploc_radius": radius, "nodes": nodes,
                     "gpu_build_ms": round(float(np.median(dev)), 4),
                     "rebuild_all_trees_plus_frame_ms": round(float(np.median(moved)), 3),
                     "gpu_build_wall_ms": round(float(np.median(wall)), 3),
                     "rebuild_plus_frame_ms": round(float(np.median(upd)), 3),
                     "frame_ms": round(float(np.median(plain)), 3), "fps": round(fps, 3)}
    return out


def main():
    args = parse()
    # stdout carries the one JSON line only: native libraries (gloo's connection messages, HIP) print to file
    # descriptor 1, so it is pointed at stderr for the run and the JSON line goes to the saved descriptor
    sys.stdout.flush()
    json_fd = os.dup(1)
    os.dup2(2, 1)
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = args.gpus if world == 1 and args.gpus == 1 else world
    k1080 = args.frames_in_flight  # 1080p: 6 frames in flight by default on one GPU (4 / 6 / 8: 512 / 538 / 536 fps)
    if args.frames_in_flight is None:
        # simulated bands (tools/band_sim_sweep.sh): 2 bands K = 4 / 8: 303 / 289 fps, 4 bands 524 / 524, 8 bands: 8
        # (thin bands' launch tails need more frames to overlap)
        args.frames_in_flight = 4 if world <= 4 else 8
        k1080 = 6 if world == 1 else 8
        if world > 1 and args.shard == "frames":
            # band slots cover another rank's whole-frame path tracer (a band's SVGF of frame f starts when f's window
            # has arrived), and the host runs as far ahead as they allow, so they also set the camera-to-modulate
            # latency. Simulated at 4K (tools/frame_shard_sim.py, profiles/r04/shard/, DESIGN.md "Which partition"),
            # window 4, N = 8, one box: K = 12 / 16 / 24 925 / 1014 / 1030 fps at 15.0 / 16.6 / 22.3 ms (window 8
            # K = 34, round 3's default: 909 fps at 39 ms); N = 4 K = 12 / 18: 611 / 623 fps at 23.6 / 30.6 ms; N = 2
            # (window 2) K = 12 / 16: 351 / 348 fps at 35 / 45 ms
            args.frames_in_flight = k1080 = 16 if world > 4 else 12
        if world > 1 and args.shard == "tiles":
            # band slots cover back_lag (2) + the subsets' frames in flight
            args.frames_in_flight = k1080 = 8
    if args.trace_batch is None:
        args.trace_batch = 1
    if args.equal_bands is None:
        args.equal_bands = 1 if (world == 2 and args.shard == "frames") else 0
    if args.own_slots is None:
        # a rank's own frames come N frames apart: with few ranks its path tracers overlap only with several slots,
        # with 8 a third or fourth slot only crowds the band's SVGF chain (simulated, see --own-slots)
        args.own_slots = 2 if world > 4 else 3 if world > 2 else 4
    if args.window is None and world > 1 and args.shard == "frames":
        args.window = min(world, 4)  # a back end waits for 4 frames' rows, not N (DESIGN.md "Which partition")
    # every frame slot must have run once before the timed region (a slot's first frame allocates its
    # wavefront state, and hipMalloc stalls the queues): at least K + 1 untimed frames
    args.warmup = max(args.warmup, args.frames_in_flight + 1)
    dist = None
    if world > 1:
        import torch.distributed as dist
        # one GPU per rank; --backend gloo (host-staged halos) rehearses the multi-rank path on fewer GPUs
        local = local % max(1, torch.cuda.device_count())
        torch.cuda.set_device(local)
        if args.backend == "nccl":
            dist.init_process_group("nccl", device_id=torch.device("cuda", local))
        else:
            dist.init_process_group(args.backend)
        # every rank takes part in the first collective (batch_isend_irecv requires it when it comes first)
        dist.barrier()
    else:
        torch.cuda.set_device(0)

    from ptsvgf import gl
    from ptsvgf.camera import parameter_config
    from ptsvgf.scene import build_scene

    scene_timings = {}
    scene = build_scene(args.scene, timings=scene_timings)
    cfg = parameter_config()
    gl.init(local)
    stream = torch.cuda.current_stream()
    from ptsvgf._lib import check, pt
    check(pt().pt_set_stream(stream.cuda_stream))

    def allsum(vals):
        if not dist:
            return vals
        t = torch.tensor(vals, dtype=torch.float64, device="cuda")
        dist.all_reduce(t)
        return t.tolist()

    def run(W, H, K, view="default", probes=True, parity=False, moving=None):
        """Warm up, time exactly args.steps frames (barrier + sync on both sides, max over ranks); then, untimed:
        one frame with the traversal counters on, one profiled frame (per-pass HIP events), the a-trous launches
        replayed between HIP events, and the surface fraction of the frame. moving: orbit the camera 1 deg per
        frame (configs[4]; default --moving), the profiled frame included."""
        moving = args.moving if moving is None else moving
        check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))  # a previous renderer's streams are gone
        log(f"run {W}x{H} K={K} view={view}")
        if world > 1 and args.shard == "frames":
            from ptsvgf.dist import make_frame_shard_renderer
            r = make_frame_shard_renderer(scene, W, H, cfg, rank, world, dist, balance=not args.equal_bands,
                                          own_slots=args.own_slots, frames_in_flight=K,
                                          ship_gbuffer=bool(args.ship_gbuffer), window=args.window,
                                          burst=args.burst)
        elif world > 1 and args.shard == "tiles":
            from ptsvgf.dist import TileShardRenderer, make_frame_shard_renderer
            r = make_frame_shard_renderer(scene, W, H, cfg, rank, world, dist, balance=not args.equal_bands,
                                          cls=TileShardRenderer, own_slots=args.own_slots, frames_in_flight=K,
                                          batch=args.tile_batch)
        elif world > 1:
            from ptsvgf.dist import make_band_renderer
            r = make_band_renderer(scene, W, H, cfg, rank, world, dist, balance=not args.equal_bands,
                                   frames_in_flight=K, trace_batch=min(args.trace_batch, K))
        else:
            from ptsvgf.renderer import Renderer
            r = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                         frames_in_flight=K, trace_batch=min(args.trace_batch, K), host_pace=bool(args.host_pace))
        r.pass_path_tracing.set_uniform_int("pt_kernel", args.pt_kernel)
        for kv in args.pt_uniform:
            name, val = kv.split("=")
            r.pass_path_tracing.set_uniform_int(name, int(val))
        rr = getattr(r, "r", r)  # the band renderer's Renderer
        rr.fuse_modulate = bool(args.fuse_modulate)
        for kv in args.svgf_uniform:
            name, val = kv.split("=")
            # every a-trous draw: the plain iterations and the last one with the fused modulate (atrous_mod_to)
            for sp in [*rr.reproject, rr.variance_compute_pass, *rr.atrous_to.values(), *rr.atrous_mod_to.values(),
                       rr.svgf_modulate_pass]:
                sp.set_uniform_int(name, int(val))
        if VIEWS[view]:
            cam = r.camera
            for k, v in VIEWS[view].items():
                setattr(cam, k, np.array(v, np.float32) if isinstance(v, tuple) else np.float32(v))
            cam.dirty = True

        moves = []  # per frame the band renderer drew: the orbit applied before it (band_parity replays them)

        def step():
            if moving:
                r.camera.orbit(1.0, 0.0)
            moves.append((1.0, 0.0) if moving else None)
            r.frame()

        for _ in range(max(args.warmup, K + 1)):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        if world > 1:
            r.time_exchanges(True)  # HIP events around each halo stage on the back-end stream
        torch.cuda.synchronize()
        torch.arange(3, device="cuda")  # kernel-trace marker: the timed frames start (tools/launch_diff.py)
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        torch.arange(3, device="cuda")  # kernel-trace marker: the timed frames have ended
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([dt], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        out = {"dt": dt, "rows": r.rows_rendered() if hasattr(r, "rows_rendered") else H}
        rr = getattr(r, "r", r)
        if K > 1 and probes:
            # camera-to-modulate latency (untimed frames): from a frame's camera reaching the GPU to the end of its
            # SVGF chain, HIP events; in frames of the timed rate
            rr.latency_events = []
            for _ in range(3 * K):
                step()
            lat = rr.latency_ms()
            rr.latency_events = None
            if dist:
                t = torch.tensor([lat], dtype=torch.float64, device="cuda")
                dist.all_reduce(t, op=dist.ReduceOp.MAX)
                lat = float(t.item())
            out["latency"] = {"camera_to_modulate_ms": round(lat, 3),
                              "frames": round(lat / (dt / args.steps * 1e3), 2), "back_lag": rr.lag}
        if world > 1:  # the band plan the calibration chose: (slowest band ms, bounds) per measured plan
            ex = r.exchange_ms()
            r.time_exchanges(False)
            # per-stage exchange ms per frame, MAX over ranks (the slowest rank's wait sets the frame)
            mx = torch.tensor([ex.get(k, 0.0) for k in EXCHANGE_STAGES], dtype=torch.float64, device="cuda")
            dist.all_reduce(mx, op=dist.ReduceOp.MAX)
            out["bands"] = {"shard": args.shard, "ship_gbuffer": bool(getattr(r, "ship_gbuffer", False)),
                            "window": getattr(r, "window", None), "burst": getattr(r, "burst", None),
                            "tile_batch": getattr(r, "batch", None), "own_slots": getattr(r, "own_slots", None),
                            "bounds": list(r.plan.bounds), "back_lag": r.r.lag,
                            "frames_in_flight": r.r.K,
                            "exchange_ms_per_frame": {k: round(v, 4) for k, v in zip(EXCHANGE_STAGES, mx.tolist())
                                                      if k in ex or v > 0},
                            "exchange_ms_rank0": ex,
                            "calibration": [[round(m, 3), list(b)] for m, b in getattr(r, "calibration", [])]}
            if getattr(r, "scatter_log", None):  # --shard frames: bytes a rank sends per frame it traces (tiles: per frame)
                out["bands"]["scatter_mb_per_traced_frame"] = round(sum(r.scatter_log) / len(r.scatter_log) / 1e6, 3)
        log(f"  {args.steps} frames in {dt:.3f} s = {args.steps / dt:.2f} frames/s")
        if probes:
            st = r.trace_stats()
            moves.append(None)  # trace_stats drew one frame (no camera move)
            out["stats"] = dict(zip(st, allsum([float(v) for v in st.values()])))
            r.profile(True)
            # on N ranks a frame's back end runs back_lag frames after its front end: profile that many more frames, so
            # that at least one SVGF chain is timed (per_frame_passes: each pass per frame it served)
            for _ in range(1 + (rr.lag if world > 1 else 0)):
                step()
            torch.cuda.synchronize()
            out["per_pass"] = per_frame_passes(r)
            r.profile(False)
            if world > 1 and parity:
                # the bands' rows before the a-trous replay below: a band's replay reads ghost rows the frame's later
                # exchanges refilled, so it times the kernels but leaves band planes that are not the frame's
                p = r.plan
                pl = r.planes()
                owned = {k: gl.readback(pl[k])[p.y0 - p.row0:p.y1 - p.row0] for k in PARITY_PLANES}
            # the roofline kernel alone: the last frame's 5 a-trous launches replayed back to back between two
            # HIP events on the library's stream (per-draw events above include launch gaps)
            out["per_pass"]["atrous_avg_ms"] = r.time_atrous(20)
            nd = gl.readback(r.planes()["normal_depth"])
            if world > 1:
                p = r.plan
                nd = nd[p.y0 - p.row0:p.y1 - p.row0]
            bg, px = allsum([float(np.count_nonzero(nd[..., 3] == 1.0)), float(nd.shape[0] * nd.shape[1])])
            out["background_fraction"] = bg / px
            if moving:
                # the profiled frame's history lengths (reproject's OutMoments_HistoryLength.z, svgf_reproject.frag:
                # 189-203): 1 = no valid history (bilinear taps and the 3x3 fallback, :111-141, both failed), < 4 =
                # young history, which svgf_variance.frag:68-96 filters with its 7x7 kernel
                hl = gl.readback(r.planes()["reproj_moments"])[..., 2]
                if world > 1:
                    hl = hl[p.y0 - p.row0:p.y1 - p.row0]
                surf = nd[..., 3] != 1.0
                ns, fresh, young = allsum([float(np.count_nonzero(surf)), float(np.count_nonzero(surf & (hl == 1.0))),
                                           float(np.count_nonzero(surf & (hl < 4.0)))])
                out["history"] = {"surface_px": int(ns), "no_history_px": int(fresh), "young_history_px": int(young),
                                  "no_history_fraction": round(fresh / max(ns, 1.0), 5),
                                  "young_history_fraction": round(young / max(ns, 1.0), 5)}
            if hasattr(r, "motion_log") and r.motion_log:
                out["max_history_rows"] = int(max(n for _, n in r.motion_log))
        if world > 1 and parity and probes:
            r.close()
            out["band_parity"] = band_parity(owned, r.plan, W, H, view, moves)
            return out
        r.close() if hasattr(r, "close") else None
        return out

    def band_parity(owned, p, W, H, view, moves):
        """The bands' owned rows, gathered on rank 0 (P2P: RCCL over xGMI, or gloo), against a one-GPU Renderer
        drawing the same camera path from frame 0: bitwise, per plane (svgf_Atrous.frag:92-97 and
        svgf_reproject.frag:45-156 are what the halo rows carry). Untimed."""
        from ptsvgf.dist import gather_bands
        from ptsvgf.renderer import Renderer

        torch.cuda.synchronize()
        full = gather_bands(owned, p, dist)
        res = None
        if rank == 0:
            log(f"band parity: one-GPU reference, {len(moves)} frames")
            gl.set_band(W, H, 0, H, 0, H)  # the library's band state is process-global: back to the whole frame
            check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
            ref = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False)
            ref.pass_path_tracing.set_uniform_int("pt_kernel", args.pt_kernel)
            for kv in args.pt_uniform:
                name, val = kv.split("=")
                ref.pass_path_tracing.set_uniform_int(name, int(val))
            if VIEWS[view]:
                for k, v in VIEWS[view].items():
                    setattr(ref.camera, k, np.array(v, np.float32) if isinstance(v, tuple) else np.float32(v))
                ref.camera.dirty = True
            for mv in moves:
                if mv:
                    ref.camera.orbit(*mv)
                ref.frame()
            want = {k: gl.readback(ref.planes()[k]) for k in PARITY_PLANES}
            ref.close()
            planes = {}
            for k in PARITY_PLANES:
                a, b = full[k].view(np.uint32), want[k].view(np.uint32)
                diff = np.abs(full[k].astype(np.float64) - want[k].astype(np.float64))
                planes[k] = {"bit_exact": bool(np.array_equal(a, b)),
                             "differing_px": int(np.count_nonzero(np.any(a != b, axis=-1))),
                             "max_abs": float(np.nanmax(diff)) if diff.size else 0.0}
            res = {"bit_exact": all(v["bit_exact"] for v in planes.values()),
                   "max_abs": max(v["max_abs"] for v in planes.values()), "frames": len(moves),
                   "backend": dist.get_backend(), "planes": planes}
            log(f"band parity: bit_exact={res['bit_exact']} max_abs={res['max_abs']}")
        dist.barrier()
        return res

    def atrous_roofline(res, W, rows, view="default"):
        atrous_ms = res["per_pass"].get("atrous_avg_ms")
        if not atrous_ms:
            return None
        t = atrous_ms * 1e-3
        alg = ATROUS_BYTES_PER_PX * W * rows
        achieved = alg / t / 1e9
        bgf = res["background_fraction"]
        weighted = W * rows * (bgf * ATROUS_BYTES_BG_PX + (1.0 - bgf) * ATROUS_BYTES_PER_PX)
        traffic, prov = atrous_traffic(W, rows, view)
        return {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": traffic, "traffic_provenance": prov,
                "kernel": ATROUS_KERNEL, "avg_launch_ms": round(atrous_ms, 4), "algorithmic_bytes_per_launch": alg,
                "frac_pmc_traffic": round(traffic / t / 1e9 / HBM_PEAK_GBS, 4) if traffic else None,
                "frac_background_weighted": round(weighted / t / 1e9 / HBM_PEAK_GBS, 4),
                "background_fraction": round(bgf, 4)}

    def per_frame_passes(r):
        """Per-pass ms per frame of the profiled frames (HIP events per draw): the SVGF passes over the frames whose
        back end was drawn (a-trous: its four plain iterations, atrous_modulate the fused last one), the G-buffer over
        the front ends drawn, the frame shard's whole-frame G-buffer / path tracer (full_*) over the frames this rank
        traced; atrous_avg_ms = one a-trous launch; frame_sum_ms = the per-frame sum."""
        rr = getattr(r, "r", r)
        times = {k: list(v) for k, v in rr._times.items()}
        full = getattr(r, "full", None)
        if full is not None:
            for k in ("gbuffer", "pathtrace"):
                if full._times.get(k):
                    times["full_" + k] = list(full._times[k])
        nback = len(times.get("reproject", [])) or 1
        back = ("reproject", "variance", "atrous", "atrous_modulate", "modulate", "taa")
        out = {k: float(np.sum(v)) / (nback if k in back else max(1, len(v))) for k, v in times.items()}
        if times.get("atrous"):
            out["atrous_avg_ms"] = float(np.mean(times["atrous"]))
        out["frame_sum_ms"] = float(sum(v for k, v in out.items() if k != "atrous_avg_ms"))
        return out

    def shadow_split(st):
        return {"point_rays": int(st.get("shadow_point_rays", 0)), "occluded": int(st.get("shadow_occluded", 0))}

    def pt_rates(res, fps):
        """Rays and BVH node + triangle visits per frame (traversal counters), as rates at the measured frame rate
        and over the path tracer's own (profiled, serial) time."""
        st = res["stats"]
        rays = st["primary_rays"] + st["bounce_rays"] + st["shadow_rays"]
        visits = st["primary_visits"] + st["bounce_visits"] + st["shadow_visits"]
        pt_ms = res["per_pass"].get("pathtrace")
        return {"rays_per_frame": {k: int(st[k]) for k in ("primary_rays", "bounce_rays", "shadow_rays")},
                "visits_per_frame": {k: int(st[k]) for k in ("primary_visits", "bounce_visits", "shadow_visits")},
                "tie_rewalks": int(st["tie_rewalks"]), "primary_retries": int(st["primary_retries"]),
                "traversals_per_pixel": round(rays / st["primary_rays"], 3) if st["primary_rays"] else None,
                "visits_per_ray": round(visits / rays, 2) if rays else None,
                # share of SIMD lanes doing traversal work: a wave runs as long as its longest ray
                "lane_efficiency": {k: round(st[f"{k}_visits"] / st[f"{k}_slots"], 3) if st.get(f"{k}_slots") else None
                                    for k in ("primary", "bounce", "shadow")},
                # shadow rays (lane-refill walks): toward point lights, occluded
                "shadow_split": shadow_split(st),
                "rays_per_s": round(rays * fps, 0), "visits_per_s": round(visits * fps, 0),
                "pt_ms_profiled": round(pt_ms, 4) if pt_ms else None,
                "rays_per_s_pt_only": round(rays / (pt_ms * 1e-3), 0) if pt_ms else None,
                "visits_per_s_pt_only": round(visits / (pt_ms * 1e-3), 0) if pt_ms else None}

    W, H = args.width, args.height
    K = args.frames_in_flight
    res = run(W, H, K, args.view, parity=world > 1 and not args.no_band_parity)
    ms = res["dt"] / args.steps * 1e3
    fps = args.steps / res["dt"]  # whole frames per second (all ranks together render one frame)
    extra = {}
    if not args.no_extras and world == 1 and K > 1:
        ser = run(W, H, 1, args.view, probes=False)
        extra["fps_serial"] = round(args.steps / ser["dt"], 3)
        extra["ms_per_step_serial"] = round(ser["dt"] / args.steps * 1e3, 3)
    if not args.no_1080p and (W, H) == (3840, 2160):
        r2 = run(1920, 1080, k1080, args.view)
        fps2 = args.steps / r2["dt"]
        extra.update({"fps_1080p": round(fps2, 3), "ms_per_step_1080p": round(r2["dt"] / args.steps * 1e3, 3),
                      "frames_in_flight_1080p": k1080,
                      "roofline_1080p": atrous_roofline(r2, 1920, r2["rows"])})
        if not args.no_extras and world == 1 and K > 1:
            s2 = run(1920, 1080, 1, args.view, probes=False)
            extra["fps_1080p_serial"] = round(args.steps / s2["dt"], 3)
    if not args.no_extras and world == 1 and args.view == "default":
        sv = run(W, H, K, "surface")
        sfps = args.steps / sv["dt"]
        extra["surface_view"] = {"camera": VIEWS["surface"], "fps": round(sfps, 3),
                                 "ms_per_step": round(sv["dt"] / args.steps * 1e3, 3),
                                 "surface_fraction": round(1.0 - sv["background_fraction"], 4),
                                 "roofline": atrous_roofline(sv, W, sv["rows"], "surface"),
                                 "path_tracer": pt_rates(sv, sfps),
                                 "passes_ms": {k: round(v, 4) for k, v in sv["per_pass"].items()}}

    if not args.no_extras and not args.moving:
        # configs[4]'s temporal stress: the camera orbits 1 deg every frame (Utils/camera.h:71 resets frameCounter on
        # each move), so reprojection sees real motion, disocclusions fall back to the 3x3 search
        # (svgf_reproject.frag:111-141) and young history takes the 7x7 variance (svgf_variance.frag:68-96). On N
        # ranks (configs[4] names 8) the history exchanges carry the moved camera's rows (dist.MotionCheck) and the
        # gathered bands are checked bitwise against a one-GPU render of the same orbit (band_parity)
        mv = run(W, H, K, args.view, moving=True, parity=world > 1 and not args.no_band_parity)
        mfps = args.steps / mv["dt"]
        extra["moving"] = {"workload": f"{args.scene} {W}x{H} 1spp depth2 + 5-iter SVGF, orbit 1 deg/frame",
                           "fps": round(mfps, 3), "ms_per_step": round(mv["dt"] / args.steps * 1e3, 3),
                           "frames_in_flight": K, "latency": mv.get("latency"), "history": mv.get("history"),
                           # (the orbit sweeps the view; no PMC profile is matched to it: traffic null)
                           "roofline": atrous_roofline(mv, W, mv["rows"], "moving"),
                           "path_tracer": pt_rates(mv, mfps),
                           "passes_ms": {k: round(v, 4) for k, v in mv["per_pass"].items()}}
        for key in ("bands", "band_parity", "max_history_rows"):
            if mv.get(key) is not None:
                extra["moving"][key] = mv[key]
        if world == 1 and not args.no_1080p and (W, H) == (3840, 2160):
            mv2 = run(1920, 1080, k1080, args.view, probes=False, moving=True)
            extra["moving"]["fps_1080p"] = round(args.steps / mv2["dt"], 3)

    if not args.no_extras and world == 1:
        log("dynamic scenes: GPU LBVH rebuilds")
        extra["dynamic_bvh"] = dynamic_bvh(scene, W, H, K, args.steps, args.warmup,
                                           scene_timings.get("host_sah_build_ms"))

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            log("cpu baseline (oracle, all usable cores and 1 core)")
            cpu = cpu_baseline(scene, W, H, args.cpu_sample, args.cpu_sample_1core)
        except Exception as e:  # the baseline is reported, never the target
            cpu = {"value": None, "error": str(e)}
        if not args.no_extras:
            try:
                log("configs[0]: cornell_teapot 512x512, SVGF off")
                extra["config0"] = config0(gl)
            except Exception as e:
                extra["config0"] = {"error": str(e)}

    if rank == 0:
        line = {"metric": METRIC, "value": round(fps, 3),
                "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "vs_baseline": None,
                # --shard frames: every rank traces whole frames, so frames/s scales but a frame's latency does not
                # (the line's "latency"); tiles / bands split every frame (strong scaling)
                "scaling": "throughput" if world > 1 and args.shard == "frames" else "strong",
                "dtype": "f32", "data": "synthetic",
                "config": {"workload": f"{args.scene} {W}x{H} 1spp depth2 + 5-iter SVGF"
                                       + (" moving camera" if args.moving else "")
                                       + (f" {args.view} view" if args.view != "default" else ""),
                           "resolution": [W, H], "spp": 1, "max_tracing_depth": cfg.max_tracing_depth,
                           "atrous_iterations": cfg.num_atrous_iterations, "triangles": scene.ntris,
                           "parallelism": (f"{args.shard}{world}+svgf_bands{world}"
                                           if world > 1 and args.shard in ("frames", "tiles") else f"bands{world}"),
                           "frames_in_flight": K,
                           "trace_batch": min(args.trace_batch, K)},
                "roofline": atrous_roofline(res, W, res["rows"], args.view), "cpu_baseline": cpu,
                "path_tracer": pt_rates(res, fps), **extra,
                "passes_ms": {k: round(v, 4) for k, v in res["per_pass"].items()}}
        if "max_history_rows" in res:
            line["max_history_rows"] = res["max_history_rows"]
        if "latency" in res:
            line["latency"] = res["latency"]
        if "history" in res:
            line["history"] = res["history"]
        if "bands" in res:
            line["bands"] = res["bands"]
        if res.get("band_parity") is not None:
            line["band_parity"] = res["band_parity"]
        sys.stdout.flush()
        os.write(json_fd, (json.dumps(line) + "\n").encode())
    gl.shutdown()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
