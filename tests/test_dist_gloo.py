"""Multi-GPU band decomposition, validated on the CPU with gloo (world 2 and 3).

Each rank holds only its band (+ ghost rows) of every plane; everything outside
is poisoned with NaN. The ranks run the SVGF passes (CPU oracle) following
ptsvgf.dist.HALO_SCHEDULE and exchange halos with ptsvgf.dist.halo_exchange —
the same plan/schedule/exchange code the GPU BandRenderer runs over RCCL. The
owned rows must equal the single-process full-frame result bit for bit: a
missing or short halo lets NaN poison into the band.
"""
import os
import socket

import numpy as np
import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(("127.0.0.1", 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _worker(rank, world, port, W, H, frames, moves, bounds=None, ghost=None, shard="bands"):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        import oracle_ref as O
        from ptsvgf.camera import rigid_inverse
        from ptsvgf.dist import (GHOST, GHOST_ZONE_GHOST, BandPlan, P2PRecorder, allreduce_motion, exchange_window,
                                 halo_exchange, run_stage, svgf_margins)
        from ptsvgf.scene import build_scene

        cur = [0]
        D = P2PRecorder(dist, frame_of=lambda: cur[0])  # every P2P batch logged (checked against the peers' below)

        scene = build_scene("table_clock_plant", hdr_size=(128, 64), plant_leaves=20)
        gz = shard == "frames_gz"  # ghost zone: passes draw margins, only the histories cross ranks
        plan = BandPlan(W, H, rank, world, ghost=ghost or (GHOST_ZONE_GHOST if gz else GHOST), bounds=bounds,
                        margins=svgf_margins(5, taa=True) if gz else None)
        rows = (lambda st: plan.stage_rows(st)) if gz else (lambda st: (plan.y0, plan.y1))
        full = O.OracleFrameLoop(scene, W, H, threads=2)
        band = O.OracleFrameLoop(scene, W, H, threads=2)  # same camera path, band-restricted execution
        log = []

        def poison(a, lo, hi):
            a[:lo] = np.nan
            a[hi:] = np.nan
            return a

        def halo(stage, arrays):
            if gz:  # the histories only (BandRenderer ghost_zone)
                t = {k: torch.from_numpy(a)[plan.row0:plan.row1] for k, a in arrays.items()}
                if stage == "reproject":
                    halo_exchange(plan.history_items(t, plan.motion), plan, D)
                elif stage == "taa":
                    halo_exchange([(t["prev_taa"], plan.motion)], plan, D)
                return
            run_stage(stage, {k: torch.from_numpy(a)[plan.row0:plan.row1] for k, a in arrays.items()}, plan, D)

        nan = lambda: np.full((H, W, 4), np.nan, np.float32)  # noqa: E731
        prev_illum, prev_moments, prev_nd, prev_taa = nan(), nan(), nan(), nan()
        for q in (prev_illum, prev_moments, prev_nd, prev_taa):  # history starts as zeros (the build zero-fills)
            q[plan.row0:plan.row1] = 0.0
        for f in range(frames):
            cur[0] = f
            mv = moves[f] if f < len(moves) else None
            if mv:
                full.camera.orbit(*mv)
                band.camera.orbit(*mv)
            want = full.frame()
            cam, cfg = band.camera, band.cfg
            cam.update()
            view, proj = cam.cam_view_mat, cam.cam_proj_mat
            g = O.gbuffer(scene.raster, W, H, view, proj, band.pre_viewproj, 2)
            for k in g:                      # the G-buffer computes the owned rows only (ghost zone: gbuffer_rows)
                poison(g[k], *(plan.gbuffer_rows() if gz else (plan.y0, plan.y1)))
            if shard == "bands":
                col, em, al = band.os.path_trace(W, H, cam.frameCounter, cam.cam_position, rigid_inverse(view),
                                                 cfg.clamp_threshold, cfg.max_tracing_depth, band.aspect_corrected,
                                                 rows=(plan.y0, plan.y1), threads=2)
            elif f % world == rank:  # frame shard: this rank traces frame f whole and sends the other bands' rows
                col, em, al = band.os.path_trace(W, H, cam.frameCounter, cam.cam_position, rigid_inverse(view),
                                                 cfg.clamp_threshold, cfg.max_tracing_depth, band.aspect_corrected,
                                                 threads=2)
                nbytes = exchange_window([(rank, [torch.from_numpy(a) for a in (col, em, al)])], plan, D)
                assert nbytes == 3 * sum(plan.zone(k)[1] - plan.zone(k)[0] for k in range(world) if k != rank) * W * 16
            else:  # ... or receives its band's rows of the planes rank f % world traced
                col, em, al = nan(), nan(), nan()
                z0, z1 = plan.zone(rank)
                exchange_window([(f % world, [torch.from_numpy(a)[z0:z1] for a in (col, em, al)])], plan, D)
            for a in (col, em, al):
                poison(a, *plan.zone(rank))
            # the motion bound the G-buffer kernel reduces (owned surface pixels), MAX over ranks
            own = g["velocity"][plan.y0:plan.y1]
            surf = g["normal_depth"][plan.y0:plan.y1, :, 3] != 1.0
            m = float(np.abs(own[..., 1][surf]).max()) if surf.any() else 0.0
            n = plan.set_motion(allreduce_motion(m, dist))
            log.append(n)
            halo("reproject", dict(prev_illum=prev_illum, prev_moments=prev_moments, prev_nd=prev_nd))
            ri, rm = O.reproject(g["velocity"], col, al, em, prev_illum, prev_moments, g["normal_depth"], prev_nd,
                                 g["fwidth"], np.float32(1.0 / W), np.float32(1.0 / H), 10.0, 16.0, 2)
            poison(ri, *rows("reproject"))
            poison(rm, *rows("reproject"))
            halo("variance", dict(illum=ri, moments=rm, nd=g["normal_depth"]))
            a = poison(O.variance(ri, rm, g["normal_depth"], g["fwidth"], 4.0, 128.0, 2), *rows("variance"))
            for i in range(cfg.num_atrous_iterations):
                halo(f"atrous{i}", dict(atrous_in=a))
                a = poison(O.atrous(a, g["normal_depth"], g["fwidth"], 1 << i, 4.0, 128.0, 2), *rows("atrous"))
                if i == 1:
                    hist = a
            m = poison(O.modulate(al, em, a, g["normal_depth"], 2), *rows("modulate"))
            halo("taa", dict(modulate=m, velocity=g["velocity"], prev_taa=prev_taa))
            t = poison(O.taa(m, prev_taa, g["velocity"], g["normal_depth"], cam.frameCounter, 2), *rows("taa"))
            prev_taa = t
            band.pre_viewproj = band._mat_mul(proj, view)
            cam.frameCounter += 1
            prev_illum, prev_moments, prev_nd = hist, rm, g["normal_depth"]
            got = dict(color=col, reproj_illum=ri, reproj_moments=rm, atrous=a, modulate=m, final=t)
            for k, v in got.items():
                o, w = v[plan.y0:plan.y1], want[k][plan.y0:plan.y1]
                assert np.array_equal(np.isnan(o), np.isnan(w)), (rank, f, k, "NaN leaked into the band")
                assert np.array_equal(np.nan_to_num(o), np.nan_to_num(w)), (rank, f, k)
        _check_p2p(D, world, frames)
        if rank == 0:
            print("history rows per frame:", log)
        return log
    finally:
        dist.destroy_process_group()


SMALL = [(1.5, 0.5)] * 3


@pytest.mark.parametrize("world,moves,bounds", [(2, [], None), (3, SMALL, None), (2, SMALL, (0, 38, 108))])
def test_band_halo_schedule_gloo(world, moves, bounds):
    W, H = 48, 108  # bands of 54 / 36 rows; uneven (balanced) split 38 / 70
    mp.spawn(_worker, args=(world, _free_port(), W, H, 3, moves, bounds), nprocs=world, join=True)


# 5-6 degrees of pitch per frame at 64 x 256 move the surface pixels of rows 0-21 by 11-16 rows (the orbit turns
# about the frame centre, so motion is largest near the frame edges): band boundaries there read history rows far
# beyond round 1's fixed 8-row halo (forcing a fixed 8 rows makes this case fail). The 16-row bands make
# the halos span several ranks (rows from rank r +- 2).
BIG = [(0.0, 5.0), (2.0, -5.0), (-3.0, 6.0)]


@pytest.mark.parametrize("world,bounds", [(2, (0, 20, 256)), (4, (0, 16, 32, 140, 256))])
def test_band_halo_large_motion_gloo(world, bounds):
    W, H = 64, 256
    mp.spawn(_worker, args=(world, _free_port(), W, H, 4, [None] + BIG, bounds), nprocs=world, join=True)


@pytest.mark.parametrize("world,moves,bounds", [(2, SMALL, None), (3, [None] + BIG, (0, 20, 140, 256))])
def test_frame_shard_scatter_gloo(world, moves, bounds):
    """Frame shard (dist.FrameShardRenderer's data path): rank f % N path-traces frame f whole and exchange_window()
    sends each band's rows of colour / emission / albedo to its owner, the SVGF chain stays banded. The bands must
    equal the single-process frame bit for bit (rows not received stay NaN and would leak)."""
    W, H = (48, 108) if bounds is None else (64, 256)
    mp.spawn(_worker, args=(world, _free_port(), W, H, 4, moves, bounds, None, "frames"), nprocs=world, join=True)


def _check_p2p(D, world, frames=None):
    """Every rank's P2P log (dist.P2PRecorder) against its peers': pairwise the same ops, bytes, groups and call sites
    in the same order (dist.check_p2p_logs)."""
    from ptsvgf.dist import check_p2p_logs

    logs = [None] * world
    dist.all_gather_object(logs, D.log)
    bad = check_p2p_logs(logs)
    assert not bad, bad[:4]
    assert all(logs), "a rank issued no P2P batch"
    if frames is not None:
        assert {f for _, _, f, _ in logs[0]} <= set(range(frames))


def _window_worker(rank, world, port, bounds, windows):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ptsvgf.dist import BandPlan, P2PRecorder, exchange_window
        D = P2PRecorder(dist)
        W, H = 8, bounds[-1]
        plan = BandPlan(W, H, rank, world, ghost=4, bounds=bounds, iterations=1)

        def frame(f):  # plane c of frame f as rank f % world traces it
            return [torch.arange(H * W * 4, dtype=torch.float32).reshape(H, W, 4) * (f + 1) + 1000 * c
                    for c in range(3)]

        f0 = 0
        for n in windows:  # consecutive frames f0 .. f0 + n - 1, at most one per source rank
            window, got = [], {}
            for f in range(f0, f0 + n):
                if f % world == rank:
                    window.append((rank, frame(f)))
                else:
                    got[f] = [torch.full((plan.y1 - plan.y0, W, 4), float("nan")) for _ in range(3)]
                    window.append((f % world, got[f]))
            sent = exchange_window(window, plan, D)
            mine = sum(1 for f in range(f0, f0 + n) if f % world == rank)
            assert sent == mine * 3 * (H - (plan.y1 - plan.y0)) * W * 16
            for f, planes in got.items():
                for a, b in zip(planes, frame(f)):
                    assert torch.equal(a, b[plan.y0:plan.y1]), (rank, f)
            f0 += n
        _check_p2p(D, world)
        assert len(D.log) == len(windows) and {s for s, *_ in D.log} == {"exchange_window"}
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bounds,windows", [(3, (0, 5, 9, 16), [3, 3, 1, 3, 2]), (4, (0, 2, 4, 10, 12), [4, 2, 4])])
def test_exchange_window_gloo(world, bounds, windows):
    """exchange_window: a window of consecutive frames (full and cut short, as flush() cuts them) delivers each band's
    rows of every frame another rank traced, and each rank sends exactly its frames' other-band rows."""
    mp.spawn(_window_worker, args=(world, _free_port(), bounds, windows), nprocs=world, join=True)


@pytest.mark.parametrize("world,moves,bounds", [(2, SMALL, None), (3, [None] + BIG, (0, 20, 140, 256)),
                                                (4, [None] + BIG, (0, 16, 32, 140, 256))])
def test_frame_shard_ghost_zone_gloo(world, moves, bounds):
    """Frame shard with the ghost zone (FrameShardRenderer's default): the path tracer's planes arrive with the
    reprojection's margin, the G-buffer covers every stored row, each SVGF pass draws its svgf_margins rows (a-trous
    at iteration 0's), and only the histories cross ranks (prev illumination / moments with margin + motion rows,
    the TAA history with motion rows). Everything outside the rows a pass draws is NaN; the bands must equal the
    single-process frame bit for bit, through 11-16-row motion and 16-row bands."""
    W, H = (48, 108) if bounds is None else (64, 256)
    mp.spawn(_worker, args=(world, _free_port(), W, H, 4, moves, bounds, None, "frames_gz"), nprocs=world, join=True)


def test_band_motion_beyond_ghost_raises():
    from ptsvgf.dist import REPROJ_REACH, BandPlan, motion_rows
    p = BandPlan(64, 400, 0, 2, ghost=40)
    assert p.set_motion(10.0 / 400) == 10 + REPROJ_REACH
    assert p.rows_for("reproj") == 13 and p.rows_for("reproj_nd") == 0
    assert p.rows_for("nd") == 32
    p.set_motion(37.0 / 400)
    assert p.rows_for("reproj_nd") == 40
    with pytest.raises(RuntimeError):
        p.set_motion(37.5 / 400)   # 38 + 3 rows of reach > 40 ghost rows
    with pytest.raises(RuntimeError):
        p.set_motion(float("inf"))
    with pytest.raises(RuntimeError):
        motion_rows(float("nan"), 100)
    with pytest.raises(ValueError):
        BandPlan(64, 400, 0, 2, ghost=40, iterations=6)   # step 32 reads 64 rows
    assert BandPlan(64, 600, 0, 2, ghost=128, iterations=6).nd_rows == 64


def test_host_motion_bound_rows():
    """MotionCheck's host bound: a static camera reaches REPROJ_REACH rows, a moved one the plan's capacity (every ghost
    row the taps can reach); camera_moved compares the matrices bit for bit, as the G-buffer kernel's arithmetic does."""
    import numpy as np

    from ptsvgf.camera import Camera, mat_mul
    from ptsvgf.dist import GHOST_ZONE_GHOST, REPROJ_REACH, BandPlan, camera_moved, svgf_margins
    p = BandPlan(64, 400, 0, 2, ghost=40)
    assert p.capacity() == 40 and p.set_rows(p.capacity()) == 40
    gz = BandPlan(3840, 2160, 3, 8, ghost=GHOST_ZONE_GHOST, margins=svgf_margins(5, False))
    assert gz.capacity() == GHOST_ZONE_GHOST - gz.margins["reproject"] == 63
    assert gz.set_rows(gz.capacity()) == 63
    with pytest.raises(RuntimeError):
        gz.set_rows(64)
    assert gz.set_rows(REPROJ_REACH) == REPROJ_REACH
    cam = Camera(64, 48)
    cam.update()
    pre = mat_mul(cam.cam_proj_mat, cam.cam_view_mat)
    assert not camera_moved(cam, pre)
    cam.update()  # recomputing the same camera gives the same bits
    assert not camera_moved(cam, pre)
    cam.orbit(0.01, 0.0)
    cam.update()
    assert camera_moved(cam, pre)
    pre2 = pre.copy()
    pre2[5] = np.nextafter(pre2[5], np.float32(2))  # one ulp of one entry is a move
    cam2 = Camera(64, 48)
    cam2.update()
    assert camera_moved(cam2, pre2)


def test_frame_shard_burst_needs_own_slots():
    """a window holding more of one rank's frames than it has own slots would overwrite an unsent frame;
    the constructor refuses before touching the GPU."""
    from ptsvgf.camera import parameter_config
    from ptsvgf.dist import FrameShardRenderer
    with pytest.raises(ValueError, match="own_slots"):
        FrameShardRenderer(None, 64, 64, parameter_config(), 0, 4, None, own_slots=2, window=4, burst=3,
                           frames_in_flight=8)


def test_halo_intervals_cover_exactly_what_is_read():
    """need()/owned() bookkeeping: for every rank pair the rows sent equal the rows received, and the union of what
    a rank receives is exactly its n-row halo (minus frame edges)."""
    from ptsvgf.dist import BandPlan, _meet
    for bounds in [(0, 90, 106, 122, 256), (0, 64, 128, 192, 256), (0, 16, 240, 256)]:
        world = len(bounds) - 1
        plans = [BandPlan(40, 256, r, world, ghost=128, bounds=bounds) for r in range(world)]
        for n in (1, 3, 20, 40, 100):
            for me in plans:
                got = set()
                for k in plans:
                    if k.rank == me.rank:
                        continue
                    for part in me.need(me.rank, n):
                        a, b = _meet(k.owned(k.rank), part)
                        got.update(range(a, b))
                want = set(range(max(0, me.y0 - n), me.y0)) | set(range(me.y1, min(256, me.y1 + n)))
                assert got == want, (bounds, n, me.rank)


def test_band_plan_properties():
    from ptsvgf.dist import GHOST, BandPlan
    for world in (1, 2, 4, 8):
        plans = [BandPlan(3840, 2160, r, world) for r in range(world)]
        assert plans[0].y0 == 0 and plans[-1].y1 == 2160
        for a, b in zip(plans, plans[1:]):
            assert a.y1 == b.y0 and a.down == b.rank and b.up == a.rank
        for p in plans:
            assert p.row0 == max(0, p.y0 - GHOST) and p.row1 == min(2160, p.y1 + GHOST)
    with pytest.raises(ValueError):
        BandPlan(64, 40, 0, 4, bounds=(0, 10, 10, 30, 40))  # empty band


def test_balanced_bounds_properties():
    from ptsvgf.dist import MIN_BAND_ROWS, balanced_bounds, fit_row_cost
    rng = np.random.default_rng(3)
    for world in (2, 3, 4, 8):
        cost = rng.uniform(0.0, 1.0, 2160)
        cost[:700] *= 6.0                              # an expensive region
        b = balanced_bounds(cost, world)
        assert b[0] == 0 and b[-1] == 2160 and len(b) == world + 1
        sizes = np.diff(b)
        assert (sizes >= MIN_BAND_ROWS).all() and all(x % 2 == 0 for x in b)
        sums = [cost[x:y].sum() for x, y in zip(b, b[1:])]
        assert max(sums) <= cost.sum() / world * 1.05   # equal cost within row granularity
    # zero cost degenerates to equal bands; a band never shrinks below the halo
    assert balanced_bounds(np.zeros(200), 4) == (0, 50, 100, 150, 200)
    spike = np.zeros(400)
    spike[10] = 1.0
    b = balanced_bounds(spike, 4)
    assert (np.diff(b) >= MIN_BAND_ROWS).all()
    with pytest.raises(ValueError):
        balanced_bounds(np.ones(40), 4)   # 4 bands of >= MIN_BAND_ROWS do not fit
    a, c = fit_row_cost([10.0, 30.0], [100, 100], [2.0, 4.0])
    assert abs(a - 0.1) < 1e-9 and abs(c - 0.01) < 1e-9
    a, c = fit_row_cost([10.0, 30.0], [100, 100], [5.0, 1.0])   # negative slope -> single-term fallback
    assert a >= 0 and c >= 0


def test_band_row_cost_matches_band_times():
    """band_row_cost keeps every band's measured time (rows sum to it) and the model's shape inside a band;
    cutting on it moves rows from a slow band to a fast one."""
    from ptsvgf.dist import balanced_bounds, band_row_cost
    rng = np.random.default_rng(5)
    visits = rng.uniform(0.0, 100.0, 400)
    visits[300:] = 0.0                                   # sky rows
    bounds = (0, 100, 200, 300, 400)
    ms = [3.0, 2.0, 2.0, 0.5]
    c = band_row_cost(visits, bounds, ms)
    for k in range(4):
        assert abs(c[bounds[k]:bounds[k + 1]].sum() - ms[k]) < 1e-9
    assert (c >= 0).all()
    nb = balanced_bounds(c, 4)
    assert nb[1] < 100 and nb[3] < 300                   # the slow first band shrinks, the cheap last one grows
    assert abs(band_row_cost(np.zeros(400), bounds, ms)[350] - 0.5 / 100) < 1e-12


def _gather_worker(rank, world, port, W, H, bounds):
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ptsvgf.dist import BandPlan, gather_bands

        plan = BandPlan(W, H, rank, world, bounds=bounds)
        frame = np.arange(H * W * 4, dtype=np.float32).reshape(H, W, 4)
        owned = {"a": frame[plan.y0:plan.y1].copy(), "b": -frame[plan.y0:plan.y1, :, :2].copy()}
        full = gather_bands(owned, plan, dist)
        if rank == 0:
            assert np.array_equal(full["a"], frame)
            assert np.array_equal(full["b"], -frame[..., :2])
        else:
            assert full is None
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,bounds", [(2, None), (3, (0, 10, 14, 40))])
def test_gather_bands_assembles_full_frame(world, bounds):
    """bench.py's band_parity gathers every rank's owned rows on rank 0 (ptsvgf.dist.gather_bands)."""
    mp.spawn(_gather_worker, args=(world, _free_port(), 6, 40, bounds), nprocs=world, join=True)


def _tile_worker(rank, world, port, W, H, bounds, batches):
    """TileShardRenderer's data path on the CPU: each rank packs its tile subset of every peer band's zone per the
    shared layout (dist.tile_layout / tile_messages; pixel order restated in numpy as test_tiles.subset_index, which is
    pinned there against pt_tiles_copy), the ranks exchange one batch with dist.exchange_tiles over gloo, and each rank
    unpacks every source's block into its zone: the zone rows must equal the frame's, for full batches and a batch cut
    short."""
    import sys
    here = os.path.dirname(os.path.abspath(__file__))
    sys.path.insert(0, here)
    sys.path.insert(0, os.path.join(os.path.dirname(here), "path-tracing-svgf_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from test_tiles import subset_index

        from ptsvgf import gl
        from ptsvgf.dist import BandPlan, exchange_tiles, svgf_margins, tile_layout, tile_messages

        plan = BandPlan(W, H, rank, world, ghost=8, bounds=bounds, iterations=1, margins=svgf_margins(1, False))
        B = max(batches)
        lay = tile_layout(plan, W, B, lambda o, a, b: gl.tiles_count(W, world, o, a, b))
        n_send, send_base, n_recv, recv_base, ns, nr = lay

        def frame(f):  # the frame's three planes (every rank knows them; each packs only its subset)
            return np.stack([np.arange(H * W * 4, dtype=np.float32).reshape(H, W, 4) * (f + 1) + 1000 * c
                             for c in range(3)])

        def block(planes, s, y0, y1):  # one packed block: plane by plane, the subset's pixels in layout order
            ys, xs = subset_index(W, world, s, y0, y1)
            return np.concatenate([planes[j][ys, xs].reshape(-1) for j in range(3)])

        f0 = 0
        z0, z1 = plan.zone(rank)
        for c in batches:
            send = torch.full((max(1, ns) * 12,), float("nan"))
            recv = torch.full((max(1, nr) * 12,), float("nan"))
            for b in range(c):
                pl = frame(f0 + b)
                for k, n in n_send.items():
                    o = (send_base[k] + b * n) * 12
                    send[o:o + n * 12] = torch.from_numpy(block(pl, rank, *plan.zone(k)))
                o = (recv_base[rank] + b * n_recv[rank]) * 12
                recv[o:o + n_recv[rank] * 12] = torch.from_numpy(block(pl, rank, z0, z1))
            sends, recvs = tile_messages(lay, rank, c, 12)
            sent = exchange_tiles(send, sends, recv, recvs, dist)
            assert sent == sum(c * n * 48 for n in n_send.values())
            for b in range(c):
                got = np.full((3, H, W, 4), np.nan, np.float32)
                for s, m in n_recv.items():
                    ys, xs = subset_index(W, world, s, z0, z1)
                    o = (recv_base[s] + b * m) * 12
                    blk = recv[o:o + m * 12].numpy().reshape(3, m, 4)
                    for j in range(3):
                        got[j][ys, xs] = blk[j]
                assert np.array_equal(got[:, z0:z1], frame(f0 + b)[:, z0:z1]), (rank, f0 + b)
            f0 += c
    finally:
        dist.destroy_process_group()


@pytest.mark.parametrize("world,W,bounds,batches", [(2, 80, None, [1, 1]), (3, 80, (0, 20, 36, 64), [3, 2]),
                                                    (4, 48, (0, 8, 30, 40, 64), [2, 2, 1])])
def test_tile_exchange_gloo(world, W, bounds, batches):
    """The tile shard's all-to-all (dist.exchange_tiles with the tile_layout / tile_messages layout): every rank's zone
    (its band widened by the ghost zone's reprojection margin) is assembled from the N subsets bit for bit; 80 / 16 = 5
    tiles per row, so the subsets are not column stripes; batches of 1-3 frames, one cut short as flush() cuts it."""
    mp.spawn(_tile_worker, args=(world, _free_port(), W, 64, bounds, batches), nprocs=world, join=True)


def _agree_worker(rank, world, port):
    import sys
    sys.path.insert(0, os.path.join(os.path.dirname(os.path.dirname(os.path.abspath(__file__))), "path-tracing-svgf_amd"))
    os.environ.update(MASTER_ADDR="127.0.0.1", MASTER_PORT=str(port))
    dist.init_process_group("gloo", rank=rank, world_size=world)
    try:
        from ptsvgf.dist import agree_bounds

        mine = (0, 100 + 8 * rank, 180 + rank, 256)  # each rank's own (diverging) calibration choice
        got = agree_bounds(tuple(np.int64(v) for v in mine), dist)
        assert got == (0, 100, 180, 256) and all(type(v) is int for v in got), (rank, got)
    finally:
        dist.destroy_process_group()


def test_agree_bounds_gloo():
    """A band calibration ends in rank 0's plan on every rank (dist.agree_bounds): ranks whose own choices differ
    (their timings raced) would otherwise cut different bands and exchange halo rows their peers do not hold."""
    mp.spawn(_agree_worker, args=(3, _free_port()), nprocs=3, join=True)


def test_check_p2p_logs_finds_mismatches():
    """dist.check_p2p_logs: matched logs pass; a byte count, a group, a call site or a cross-group order that differs
    between two peers is reported."""
    from ptsvgf.dist import check_p2p_logs

    r0 = [("halo_exchange", "world", 0, [("send", 1, 64), ("recv", 1, 32)]),
          ("exchange_window", "scatter", 0, [("send", 1, 96), ("send", 2, 96)])]
    # (within a batch the send / receive interleaving is free: one group call)
    r1 = [("halo_exchange", "world", 0, [("send", 0, 32), ("recv", 0, 64)]),
          ("exchange_window", "scatter", 0, [("recv", 0, 96)])]
    r2 = [("exchange_window", "scatter", 0, [("recv", 0, 96)])]
    assert check_p2p_logs([r0, r1, r2]) == []
    bytes_off = [r0, [r1[0], ("exchange_window", "scatter", 0, [("recv", 0, 80)])], r2]
    assert check_p2p_logs(bytes_off)
    wrong_group = [r0, [("halo_exchange", "scatter", 0, r1[0][3]), r1[1]], r2]
    assert check_p2p_logs(wrong_group)
    swapped_sizes = [r0, [("halo_exchange", "world", 0, [("send", 0, 64), ("recv", 0, 32)]), r1[1]], r2]
    assert check_p2p_logs(swapped_sizes)
    split = [r0, [("halo_exchange", "world", 0, [("send", 0, 32)]), ("halo_exchange", "world", 0, [("recv", 0, 64)]),
                  r1[1]], r2]  # the same ops in two batches: not one group call on both sides
    assert check_p2p_logs(split)
    reordered = [r0, [r1[1], r1[0]], r2]  # rank 1 issues the scatter receive before the world halo: cross-group order
    assert any("0<->1" in m for m in check_p2p_logs(reordered))
    missing = [r0, r1, []]
    assert any("0<->2" in m for m in check_p2p_logs(missing))


def test_motion_check_names_first_bad_frame():
    """MotionCheck verifies after the fact; MotionCheckError names the first frame whose exchanged history
    rows fell short of its measured motion (that frame on is to be discarded), and verify() reports the earliest."""
    import numpy as np

    from ptsvgf.dist import REPROJ_REACH, BandPlan, MotionCheck, MotionCheckError

    class Ev:
        def query(self):
            return True

        def synchronize(self):
            pass

    mc = MotionCheck.__new__(MotionCheck)  # (the pinned host ring needs a device; a plain tensor stands in)
    mc.plan = BandPlan(64, 400, 0, 2, ghost=40)
    mc.host = torch.zeros(MotionCheck.RING, dtype=torch.int32)
    mc.ev, mc.slot_frame = [None] * MotionCheck.RING, [None] * MotionCheck.RING
    mc.pending, mc.moved, mc.used, mc.log, mc.first_bad = [], {}, {}, [], None

    def frame(f, moved, motion_rows_measured):
        j = f % MotionCheck.RING
        mc.host[j:j + 1] = torch.from_numpy(np.array([motion_rows_measured / 400.0], np.float32).view(np.int32))
        mc.ev[j], mc.slot_frame[j] = Ev(), f
        mc.pending.append(j)
        mc.note_camera(f, moved)

    frame(0, False, 0.0)
    frame(1, True, 30.0)  # moved: capacity rows, enough
    assert mc.rows(0) == REPROJ_REACH and mc.rows(1) == mc.plan.capacity()
    frame(2, False, 10.0)  # the host saw no move but the G-buffer measured 10 rows: short
    frame(3, False, 12.0)
    with pytest.raises(MotionCheckError) as e:
        mc.rows(2)
        mc.rows(3)
    assert e.value.frame == 2 and e.value.need >= 10 + REPROJ_REACH and e.value.used == REPROJ_REACH
    with pytest.raises(MotionCheckError) as e:
        mc.verify()
    assert e.value.frame == 2
