#!/usr/bin/env python3
"""Headline benchmark: frames/s of 1 spp path tracing + 5-iteration SVGF on the
table+clock+plant scene (BASELINE.json metric / configs[2]: 3840x2160, 1x MI355X),
plus the a-trous kernel's achieved HBM GB/s against the 8 TB/s roofline.

A "step" is one frame of the hot path: G-buffer, path tracer (depth 2, NEE),
reprojection, variance, 5 a-trous iterations, modulate (TAA and
the output tonemap are excluded there and excluded here). Inputs (scene, BVH,
environment) are resident in HBM before timing starts; the camera orbits by a
fixed step each frame only with --moving.

Multi-GPU (python -m torch.distributed.run --nproc-per-node N bench.py --gpus N):
each rank renders one horizontal band of the SAME 4K frame and exchanges SVGF
halo rows with its neighbours over RCCL (ptsvgf.dist) — strong scaling.
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
# and serialise. Set before HIP initialises.
os.environ.setdefault("GPU_MAX_HW_QUEUES", "16")
sys.path.insert(0, os.path.join(REPO, "path-tracing-svgf_amd"))
sys.path.insert(0, os.path.join(REPO, "tests"))

ATROUS_BYTES_PER_PX = 52  # illum 16 + normal/z 16 + depth-fwidth 4 + write 16
HBM_PEAK_GBS = 8000.0     # MI355X_MICROARCH.md: 8 TB/s spec
METRIC = "frames/sec @1spp+SVGF, 1080p & 4K; \u00e0-trous HBM GB/s vs peak"  # BASELINE.json "metric"
ATROUS_KERNEL = "atrous_tile_kernel"
# HBM bytes per a-trous launch measured with rocprofv3 PMC passes (tools/gpu_profile.sh), committed under profiles/
TRAFFIC_FILE = os.path.join(REPO, "profiles", "atrous_traffic.json")


def atrous_traffic(W, rows):
    """PMC-measured HBM bytes per a-trous launch (FETCH_SIZE x2 gfx950 correction + WRITE_SIZE, in KB units as the
    guide prescribes) from the committed profile, when it was taken for this kernel at this frame size."""
    try:
        with open(TRAFFIC_FILE) as f:
            t = json.load(f)
    except (OSError, ValueError):
        return None
    if t.get("kernel") != ATROUS_KERNEL or t.get("pixels") != W * rows:
        return None
    return t.get("bytes_per_launch")


def parse():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=100)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--width", type=int, default=3840)
    ap.add_argument("--height", type=int, default=2160)
    ap.add_argument("--scene", default="table_clock_plant")
    ap.add_argument("--moving", action="store_true", help="orbit the camera 1 deg/frame (configs[4])")
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--cpu-sample", default="960x540", help="oracle sample frame size for cpu_baseline")
    ap.add_argument("--no-1080p", action="store_true", help="skip the secondary 1080p measurement")
    ap.add_argument("--backend", default="nccl", help="torch.distributed backend for --gpus > 1 (nccl = RCCL)")
    ap.add_argument("--equal-bands", action="store_true", help="multi-GPU: equal band heights (no cost balancing)")
    ap.add_argument("--breakdown", action="store_true", help="print per-pass ms to stderr")
    ap.add_argument("--pt-kernel", type=int, default=0, help="0 wavefront (production), 1 megakernel (A/B)")
    ap.add_argument("--frames-in-flight", type=int, default=None,
                    help="K > 1: front ends (G-buffer + path tracer) of K frames overlap on K streams "
                         "(default 4 on one GPU, 8 on bands: thinner bands have relatively longer launch tails)")
    ap.add_argument("--pt-uniform", action="append", default=[], metavar="NAME=INT",
                    help="extra int uniform on the path-tracing pass (A/B switches, e.g. shadow_bvh4=0)")
    return ap.parse_args()


def cpu_baseline(scene, W, H, sample: str):
    """Time the CPU oracle (the reference algorithm restated, OpenMP over rows) on a bounded sample
    frame and scale to the full frame by pixel count."""
    import oracle_ref as O
    from ptsvgf.camera import parameter_config

    sw, sh = (int(v) for v in sample.split("x"))
    threads = min(16, os.cpu_count() or 1)
    loop = O.OracleFrameLoop(scene, sw, sh, parameter_config(), aspect_corrected=True, threads=threads,
                              run_taa=False)
    loop.frame()  # warm (first frame: young history, full 7x7 variance)
    t0 = time.perf_counter()
    n = 0
    while True:
        loop.frame()
        n += 1
        if time.perf_counter() - t0 > 10.0 and n >= 3:  # ~10 s of CPU work
            break
    dt = (time.perf_counter() - t0) / n
    scale = (W * H) / (sw * sh)
    return {"value": 1.0 / (dt * scale), "unit": "frames/s", "cores": threads, "kind": "port",
            "sample": f"oracle frame loop (G-buffer+PT+SVGF) at {sw}x{sh}, {n} frames, {dt * 1e3:.1f} ms/frame, "
                      f"scaled by pixel count to {W}x{H}"}


def main():
    args = parse()
    import numpy as np
    import torch

    world = int(os.environ.get("WORLD_SIZE", "1"))
    rank = int(os.environ.get("RANK", "0"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        world = args.gpus if world == 1 and args.gpus == 1 else world
    if args.frames_in_flight is None:
        args.frames_in_flight = 4 if world == 1 else 8
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
    else:
        torch.cuda.set_device(0)

    from ptsvgf import gl
    from ptsvgf.camera import parameter_config
    from ptsvgf.scene import build_scene

    scene = build_scene(args.scene)
    cfg = parameter_config()
    gl.init(local)
    stream = torch.cuda.current_stream()
    from ptsvgf._lib import check, pt
    check(pt().pt_set_stream(stream.cuda_stream))

    def run(W, H):
        """Warm up, time exactly args.steps frames (barrier + sync on both sides, max over ranks), then one
        profiled frame for the per-pass HIP-event breakdown."""
        if world > 1:
            from ptsvgf.dist import make_band_renderer
            r = make_band_renderer(scene, W, H, cfg, rank, world, dist, balance=not args.equal_bands,
                                   frames_in_flight=args.frames_in_flight)
        else:
            from ptsvgf.renderer import Renderer
            r = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, run_taa=False, run_output=False,
                         frames_in_flight=args.frames_in_flight)
        r.pass_path_tracing.set_uniform_int("pt_kernel", args.pt_kernel)
        for kv in args.pt_uniform:
            name, val = kv.split("=")
            r.pass_path_tracing.set_uniform_int(name, int(val))

        def step():
            if args.moving:
                r.camera.orbit(1.0, 0.0)
            r.frame()

        for _ in range(args.warmup):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(args.steps):
            step()
        torch.cuda.synchronize()
        if dist:
            dist.barrier()
        torch.cuda.synchronize()
        dt = time.perf_counter() - t0
        if dist:
            t = torch.tensor([dt], device="cuda")
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            dt = float(t.item())
        r.profile(True)
        step()
        torch.cuda.synchronize()
        per_pass = r.pass_times()
        r.profile(False)
        # the roofline kernel alone: the last frame's 5 a-trous launches replayed back to back between two
        # HIP events on the library's stream (per-draw events above include launch gaps)
        per_pass["atrous_avg_ms"] = r.time_atrous(20)
        rows = r.rows_rendered() if hasattr(r, "rows_rendered") else H
        r.close() if hasattr(r, "close") else None
        return dt, per_pass, rows

    W, H = args.width, args.height
    dt, per_pass, rows = run(W, H)
    ms = dt / args.steps * 1e3
    fps = args.steps / dt  # whole frames per second (all ranks together render one frame)
    extra = {}
    if not args.no_1080p and (W, H) == (3840, 2160):
        dt2, _, _ = run(1920, 1080)
        extra = {"fps_1080p": round(args.steps / dt2, 3), "ms_per_step_1080p": round(dt2 / args.steps * 1e3, 3)}

    atrous_ms = per_pass.get("atrous_avg_ms")
    roof = None
    if atrous_ms:
        achieved = ATROUS_BYTES_PER_PX * W * rows / (atrous_ms * 1e-3) / 1e9
        roof = {"bound": "hbm", "achieved": round(achieved, 1), "peak": HBM_PEAK_GBS, "unit": "GB/s",
                "frac": round(achieved / HBM_PEAK_GBS, 4), "traffic": atrous_traffic(W, rows),
                "kernel": ATROUS_KERNEL, "avg_launch_ms": round(atrous_ms, 4),
                "algorithmic_bytes_per_launch": ATROUS_BYTES_PER_PX * W * rows}

    cpu = None
    if rank == 0 and world == 1 and not args.no_cpu_baseline:
        try:
            cpu = cpu_baseline(scene, W, H, args.cpu_sample)
        except Exception as e:  # the baseline is reported, never the target
            cpu = {"value": None, "error": str(e)}

    if rank == 0:
        line = {"metric": METRIC, "value": round(fps, 3),
                "unit": "frames/s", "n_gpus": world, "steps": args.steps, "warmup": args.warmup,
                "ms_per_step": round(ms, 3), "higher_is_better": True, "scaling": "strong", "vs_baseline": None,
                "dtype": "f32", "data": "synthetic",
                "config": {"workload": f"{args.scene} {W}x{H} 1spp depth2 + 5-iter SVGF"
                                       + (" moving camera" if args.moving else ""),
                           "resolution": [W, H], "spp": 1, "max_tracing_depth": cfg.max_tracing_depth,
                           "atrous_iterations": cfg.num_atrous_iterations, "triangles": scene.ntris,
                           "parallelism": f"bands{world}", "frames_in_flight": args.frames_in_flight},
                "roofline": roof, "cpu_baseline": cpu, **extra,
                "passes_ms": {k: round(v, 4) for k, v in per_pass.items()}}
        print(json.dumps(line), flush=True)
    gl.shutdown()
    if dist:
        dist.destroy_process_group()


if __name__ == "__main__":
    main()
