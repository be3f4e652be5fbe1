"""bench.py's multi-GPU line checks itself: at --gpus N > 1 every rank's owned rows
are gathered on rank 0 after the timed region and compared bitwise with a one-GPU
render of the same camera path (band_parity), and the per-stage halo exchange
times are reported. The driver's 8-GPU run (RCCL over xGMI) executes exactly this
code; here it is rehearsed with --backend gloo, N ranks on the one visible GPU
(RCCL refuses two ranks on one device)."""
import json
import os
import socket
import subprocess
import sys

import pytest

pytestmark = pytest.mark.gpu

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize("world,moving,balance,shard", [(2, True, True, "bands"), (4, False, False, "bands"),
                                                        (2, True, False, "frames"), (3, True, True, "frames"),
                                                        (4, True, False, "frames"), (3, True, False, "frames+gbuffer"),
                                                        (2, True, False, "tiles"), (3, True, True, "tiles"),
                                                        (4, False, False, "tiles"), (3, True, False, "frames+w1"),
                                                        (3, True, False, "frames+b2"), (3, True, False, "tiles+b3")])
def test_bench_band_parity_gloo(world, moving, balance, shard):
    """shard = "bands": every rank traces its band; "frames": rank f % N traces frame f whole and scatters the
    path tracer's rows to the band owners (dist.FrameShardRenderer); "frames+gbuffer": and its G-buffer rows, which
    the bands adopt instead of drawing (ship_gbuffer, an option); "frames+w1": each frame's rows sent alone as soon
    as traced (window 1); "frames+b2": each rank traces two consecutive frames (burst 2); "tiles": every rank traces the 16x16 tiles
    k * N + rank of every frame and one all-to-all per frame carries them to the band owners (dist.TileShardRenderer;
    320 / 16 = 20 tiles per row, so at N = 3 the subsets are not column stripes)."""
    ship = shard == "frames+gbuffer"
    w1 = shard == "frames+w1"  # per-frame exchanges (window 1, back_lag 1)
    b2 = shard == "frames+b2"  # two consecutive frames per rank (burst 2): a window holds two frames of one source
    tb3 = shard == "tiles+b3"  # tile subsets of 3 consecutive frames in one batched draw and one exchange
    shard = "frames" if ship or w1 or b2 else "tiles" if tb3 else shard
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--backend", "gloo", "--width", "320", "--height", "256", "--steps", "4",
           "--warmup", "2", "--no-extras", "--no-1080p", "--no-cpu-baseline", "--shard", shard,
           "--ship-gbuffer", "1" if ship else "0"]
    cmd += ["--moving"] if moving else []
    cmd += ["--window", "1", "--frames-in-flight", "6"] if w1 else []
    cmd += ["--burst", "2"] if b2 else []
    cmd += ["--tile-batch", "3"] if tb3 else []
    cmd += ["--equal-bands", "0" if balance else "1"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    bp = line["band_parity"]
    print(json.dumps(bp), json.dumps(line["bands"]["exchange_ms_per_frame"]))
    assert line["n_gpus"] == world
    assert bp["backend"] == "gloo" and bp["frames"] >= 4
    assert bp["bit_exact"], bp
    assert line["bands"]["shard"] == shard and line["bands"].get("ship_gbuffer", False) == ship
    if w1:
        assert line["bands"]["window"] == 1 and line["bands"]["back_lag"] == 1
    if b2:
        assert line["bands"]["burst"] == 2
    if tb3:
        assert line["bands"]["tile_batch"] == 3 and line["bands"]["back_lag"] == 3
    if shard in ("frames", "tiles"):
        assert line["bands"]["scatter_mb_per_traced_frame"] > 0
    assert line["latency"]["camera_to_modulate_ms"] > 0 and line["latency"]["back_lag"] == line["bands"]["back_lag"]
    ex = line["bands"]["exchange_ms_per_frame"]
    if shard == "bands":
        assert {"reproject", "variance", "atrous0", "atrous4"} <= set(ex)
    else:  # ghost zone: the history exchange only, started early (overlapping the previous frame's chain)
        assert "history" in ex and not {"variance", "atrous0", "atrous4"} & set(ex), ex


@pytest.mark.timeout(900)
@pytest.mark.parametrize("W,H,balance", [(1920, 1080, False), (3840, 2160, False), (1920, 1080, True)])
def test_bench_frame_shard_8_ranks_gloo(W, H, balance):
    """the default multi-GPU mode (--shard frames: rank f % 8 traces frame f whole, the SVGF chain
    banded with the ghost zone and the early history exchange) at the BASELINE sizes and rank count — 8 ranks, 1920 x
    1080 (configs[1]) and 3840 x 2160 (configs[3] / [4]), a moving camera, frames_in_flight and the exchange window at
    their 8-rank defaults (16 band slots, window = back_lag 4) — rehearsed with gloo on the one GPU (4K: ≈ 30 s). 16 timed frames = 4 full windows of 4 after the warm-up's windows; the gathered bands must
    equal a one-GPU render of the same camera path bit for bit (reference: main.cpp:436-535 per frame,
    svgf_Atrous.frag:92-97 and svgf_reproject.frag:45-156 for what crosses bands). balance: the bench's exact 8-rank
    default, balanced bands calibrated by make_frame_shard_renderer (round 4's rank-disagreement bug
    lived in that calibration path, dist.agree_bounds)."""
    world = 8
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--backend", "gloo", "--width", str(W), "--height", str(H), "--steps", "16",
           "--warmup", "2", "--no-extras", "--no-1080p", "--no-cpu-baseline", "--shard", "frames", "--moving"]
    cmd += ["--equal-bands", "0" if balance else "1"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=850)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    bp, bands = line["band_parity"], line["bands"]
    print(json.dumps(bp), json.dumps(bands["exchange_ms_per_frame"]), bands["frames_in_flight"], bands["back_lag"],
          line.get("max_history_rows"))
    assert line["n_gpus"] == world and bands["shard"] == "frames"
    assert bands["back_lag"] == bands["window"] == 4 and bands["frames_in_flight"] == 16  # bench.py's 8-rank defaults
    assert bp["backend"] == "gloo" and bp["frames"] >= 2 * world + 16  # warm-up windows + 4 timed windows + probes
    assert bp["bit_exact"], bp
    assert line.get("max_history_rows", 0) > 3  # the orbit moved the history (reprojection reach beyond the taps)
    assert line["scaling"] == "throughput"  # whole frames per rank: frames/s scale, a frame's latency does not
    equal = [(H * k) // world for k in range(world + 1)]
    if balance:
        # make_frame_shard_renderer measured its rounds (equal bands first) and every rank holds rank 0's choice
        assert len(bands["calibration"]) == 3 and bands["calibration"][0][1] == equal, bands
        assert bands["bounds"] in [b for _, b in bands["calibration"]], bands
    else:
        assert bands["bounds"] == equal


def test_bench_moving_extra_on_ranks_gloo():
    """The driver's multi-GPU line carries configs[4] (moving camera, per-pass times) beside the static run: at N ranks
    bench.py (extras on) draws the 1 deg/frame orbit through the frame shard and checks its gathered bands bitwise
    against a one-GPU render of the same orbit (the history exchanges carry the moved camera's rows)."""
    world = 2
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", f"--nproc-per-node={world}",
           "--master-addr", "127.0.0.1", f"--master-port={_port()}", os.path.join(REPO, "bench.py"),
           "--gpus", str(world), "--backend", "gloo", "--width", "320", "--height", "256", "--steps", "4",
           "--warmup", "2", "--no-1080p", "--no-cpu-baseline", "--equal-bands", "1"]
    p = subprocess.run(cmd, cwd=REPO, capture_output=True, text=True, timeout=600)
    assert p.returncode == 0, p.stderr[-4000:]
    line = json.loads(p.stdout.strip().splitlines()[-1])
    mv = line["moving"]
    print(json.dumps({k: mv[k] for k in ("fps", "history", "max_history_rows") if k in mv}), json.dumps(mv["band_parity"]))
    assert line["band_parity"]["bit_exact"] and mv["band_parity"]["bit_exact"], mv["band_parity"]
    assert mv["max_history_rows"] > 3  # the moved camera's history rows crossed ranks
    assert {"reproject", "variance", "atrous"} <= set(mv["passes_ms"]) and mv["fps"] > 0
    assert "history" in mv["bands"]["exchange_ms_per_frame"]
