"""Screen-band sharding of one frame across GPUs.

One process per GPU; rank r renders the horizontal band of global rows
[y0, y1). The path tracer is embarrassingly parallel (RNG seeds use global pixel
coordinates, path_tracing.frag:433-436), so it runs on owned rows only. The SVGF
passes are bounded stencils; before each one the ranks swap halo rows with
their up/down neighbours (torch.distributed P2P: RCCL over xGMI on the GPU,
gloo on the CPU tests). The G-buffer ghost rows are recomputed locally (a
primary-ray cast is cheaper than shipping 2 planes).

Every frame-sized plane is stored with GHOST rows either side of the band:
rows [row0, row1) = [y0 - GHOST, y1 + GHOST) clipped to the frame.

HALO_SCHEDULE is the single source of truth for which planes are exchanged
before which pass and how many rows; BandRenderer (GPU) and
tests/test_dist_gloo.py (CPU, oracle) both execute it.
"""
from __future__ import annotations

from dataclasses import dataclass

# a-trous radius 2*step (svgf_Atrous.frag:92-97) up to step 16; variance radius 3
# (svgf_variance.frag:273); reprojection taps within |motion|+2 rows (svgf_reproject.frag:63,116)
ATROUS_HALO = [2 * (1 << i) for i in range(8)]
VARIANCE_HALO = 3
GHOST = 34

# (stage, planes, rows): executed before `stage`
HALO_SCHEDULE = (
    ("reproject", ("prev_illum", "prev_moments"), "reproj"),
    ("variance", ("illum", "moments"), VARIANCE_HALO),
    *((f"atrous{i}", ("atrous_in",), ATROUS_HALO[i]) for i in range(8)),
    # taa.frag: 3x3 neighbourhood of the current colour, history fetched at uv - velocity (:88-98, :137-139)
    ("taa", ("modulate", "prev_taa"), "reproj"),
)


@dataclass
class BandPlan:
    W: int
    H: int
    rank: int
    world: int
    ghost: int = GHOST
    reproj_halo: int = 8
    bounds: tuple | None = None  # world+1 row boundaries (balanced_bounds); None = equal bands

    def __post_init__(self):
        b = list(self.bounds) if self.bounds is not None else [(self.H * k) // self.world for k in range(self.world + 1)]
        if len(b) != self.world + 1 or b[0] != 0 or b[-1] != self.H or any(x >= y for x, y in zip(b, b[1:])):
            raise ValueError(f"bad band bounds {b}")
        self.bounds = tuple(b)
        self.y0, self.y1 = b[self.rank], b[self.rank + 1]
        if self.y1 - self.y0 < max(ATROUS_HALO[4], self.reproj_halo):
            raise ValueError(f"band of {self.y1 - self.y0} rows is thinner than the largest halo")
        if self.reproj_halo + 1 > self.ghost:
            raise ValueError("reprojection halo exceeds the ghost rows")
        self.row0 = max(0, self.y0 - self.ghost)
        self.row1 = min(self.H, self.y1 + self.ghost)
        self.rows = self.row1 - self.row0
        self.up = self.rank - 1 if self.rank > 0 else None
        self.down = self.rank + 1 if self.rank < self.world - 1 else None

    def rows_for(self, n) -> int:
        return self.reproj_halo if n == "reproj" else int(n)


MIN_BAND_ROWS = max(ATROUS_HALO[4], 8) + 4  # a band must hold the widest halo it ships (5-iteration a-trous)


def balanced_bounds(row_cost, world: int, min_rows: int = MIN_BAND_ROWS, align: int = 2) -> tuple:
    """Row boundaries splitting a frame into `world` bands of equal summed cost.

    row_cost[y] is the estimated time of row y (measure_row_cost). Boundary k is the first row where the
    cumulative cost reaches k/world of the total, rounded to `align` rows and pushed so that every band keeps
    at least `min_rows` rows. Pure function of its inputs, so every rank computes the same plan."""
    import numpy as np

    c = np.asarray(row_cost, dtype=np.float64)
    H = c.size
    if world * min_rows > H:
        raise ValueError(f"{world} bands of >= {min_rows} rows do not fit {H} rows")
    cum = np.concatenate([[0.0], np.cumsum(np.maximum(c, 0.0))])
    total = cum[-1]
    b = [0]
    for k in range(1, world):
        y = int(np.searchsorted(cum, total * k / world)) if total > 0 else (H * k) // world
        y = int(round(y / align) * align)
        lo = b[-1] + min_rows                   # previous band keeps min_rows
        hi = H - (world - k) * min_rows         # the remaining bands still fit
        b.append(min(max(y, lo), hi))
    b.append(H)
    return tuple(b)


def halo_exchange(tensors, plan: BandPlan, n: int, dist, group=None) -> None:
    """Swap n halo rows with both neighbours for each (rows, W, C) tensor holding rows [row0, row1)."""
    if plan.world == 1 or n <= 0:
        return
    if tensors and tensors[0].is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device P2P: stage through host memory (tests run 2 ranks on one GPU this way)
        host = [t.cpu() for t in tensors]
        halo_exchange(host, plan, n, dist, group)
        for t, h in zip(tensors, host):
            t.copy_(h)
        return
    ops = []
    lo = plan.y0 - plan.row0  # local index of the first owned row
    hi = plan.y1 - plan.row0  # one past the last owned row
    for t in tensors:
        if plan.up is not None:
            k = min(n, lo)
            ops.append(dist.P2POp(dist.isend, t[lo:lo + k], plan.up, group))  # row slices are contiguous
            ops.append(dist.P2POp(dist.irecv, t[lo - k:lo], plan.up, group))
        if plan.down is not None:
            k = min(n, plan.rows - hi)
            ops.append(dist.P2POp(dist.isend, t[hi - k:hi], plan.down, group))
            ops.append(dist.P2POp(dist.irecv, t[hi:hi + k], plan.down, group))
    if ops:
        for req in dist.batch_isend_irecv(ops):
            req.wait()


class BandRenderer:
    """One rank's share of a frame: the fast Renderer on band storage + HALO_SCHEDULE exchanges."""

    def __init__(self, scene, W, H, cfg, rank, world, dist, reproj_halo: int = 8, bounds=None, **kw):
        import torch

        from . import gl
        from .renderer import Renderer

        self.plan = BandPlan(W, H, rank, world, reproj_halo=reproj_halo, bounds=bounds)
        self.dist = dist
        self.exchange = True  # False only while calibrating (make_band_renderer): ranks time their bands alone
        self._tensors = {}
        gl.set_band(W, H, self.plan.y0, self.plan.y1, self.plan.row0, self.plan.rows)
        dev = torch.device("cuda", torch.cuda.current_device())

        def factory(w, h):
            t = torch.zeros((self.plan.rows, w, 4), dtype=torch.float32, device=dev)
            handle = gl.wrap_device_texture(t.data_ptr(), w, h)
            self._tensors[handle] = t
            return handle

        kw.setdefault("run_taa", False)
        kw.setdefault("run_output", False)
        self.r = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, tex_factory=factory,
                          halo=self._halo, gbuffer_rows=(self.plan.row0, self.plan.row1), **kw)
        self.camera = self.r.camera
        self.pass_path_tracing = self.r.pass_path_tracing

    def _halo(self, stage: str, handles) -> None:
        if not self.exchange:
            return
        for st, _, n in HALO_SCHEDULE:
            if st == stage:
                halo_exchange([self._tensors[h] for h in handles], self.plan, self.plan.rows_for(n), self.dist)
                return

    def frame(self) -> None:
        self.r.frame()

    def profile(self, on: bool) -> None:
        self.r.profile(on)

    def pass_times(self) -> dict:
        return self.r.pass_times()

    def time_atrous(self, reps: int = 20) -> float:
        return self.r.time_atrous(reps)

    def rows_rendered(self) -> int:
        return self.plan.y1 - self.plan.y0

    def planes(self) -> dict:
        return self.r.planes()

    def close(self) -> None:
        self.r.close()
        self._tensors.clear()

    def measure_row_cost(self, frames: int = 24):
        """Estimated time (ms) of every frame row, identical on all ranks.

        One probed frame counts each row's BVH visits (pt_pass_set_row_cost). Then every rank times `frames`
        frames of its band ALONE (halo exchanges off, so a rank's time is its own work, not its wait for the
        slowest neighbour) with the renderer's frames in flight: per-launch tails that overlap other frames'
        work cost nothing, which a serial per-pass timing would count. The per-rank times are spread back onto
        rows by band_row_cost. Calibration frames are discarded (the renderer is rebuilt afterwards)."""
        import time

        import numpy as np
        import torch

        p, H = self.plan, self.r.H
        dev = torch.device("cuda", torch.cuda.current_device())
        counts = torch.zeros(p.y1 - p.y0, dtype=torch.int32, device=dev)
        self.exchange = False
        try:
            self.pass_path_tracing.set_row_cost(counts.data_ptr())
            self.r.frame()
            torch.cuda.synchronize()
            self.pass_path_tracing.set_row_cost(0)
            for _ in range(max(1, self.r.K)):  # every frame slot once: first use allocates (hipMalloc syncs)
                self.r.frame()
            torch.cuda.synchronize()
            t0 = time.perf_counter()
            for _ in range(frames):
                self.r.frame()
            torch.cuda.synchronize()
            frame_ms = (time.perf_counter() - t0) * 1e3 / frames
        finally:
            self.exchange = True
        visits = torch.zeros(H, dtype=torch.float64, device=dev)
        visits[p.y0:p.y1] = counts.to(torch.float64)
        per_rank = torch.zeros(p.world, dtype=torch.float64, device=dev)
        per_rank[p.rank] = frame_ms
        self.dist.all_reduce(visits)
        self.dist.all_reduce(per_rank)
        return band_row_cost(visits.cpu().numpy(), p.bounds, per_rank.cpu().numpy())


def band_row_cost(visits, bounds, ms):
    """Per-row cost (ms) from per-row BVH visits and the measured time of each band [bounds[k], bounds[k+1]).

    A global model T = a*visits + b*rows (fit_row_cost over the bands) shapes the cost inside a band; each
    band's rows are then scaled so that they sum to that band's measured time, so the model's misfit (tails,
    sky rows) cannot move a boundary away from where the measurements put it."""
    import numpy as np

    v = np.asarray(visits, np.float64)
    t = np.asarray(ms, np.float64)
    segs = [(bounds[k], bounds[k + 1]) for k in range(len(bounds) - 1)]
    a, b = fit_row_cost([v[y0:y1].sum() for y0, y1 in segs], [y1 - y0 for y0, y1 in segs], t)
    model = a * v + b
    out = np.empty_like(v)
    for k, (y0, y1) in enumerate(segs):
        m = model[y0:y1]
        s = m.sum()
        out[y0:y1] = m * (t[k] / s) if s > 0 else t[k] / max(y1 - y0, 1)
    return out


def fit_row_cost(visits, rows, ms):
    """Least-squares T = a*visits + b*rows with a, b >= 0 (falls back to a single term when the 2-term fit
    goes negative or is singular)."""
    import numpy as np

    A = np.stack([np.asarray(visits, np.float64), np.asarray(rows, np.float64)], 1)
    t = np.asarray(ms, np.float64)
    try:
        (a, b), *_ = np.linalg.lstsq(A, t, rcond=None)
    except np.linalg.LinAlgError:
        a = b = -1.0
    if a >= 0 and b >= 0 and a + b > 0:
        return float(a), float(b)
    if A[:, 0].sum() > 0:
        return float(t.sum() / A[:, 0].sum()), 0.0
    return 0.0, float(t.sum() / max(A[:, 1].sum(), 1.0))


def make_band_renderer(scene, W, H, cfg, rank, world, dist, balance: bool = True, rounds: int = 2, **kw):
    """BandRenderer whose band heights equalise the measured per-row cost (sky rows are cheap, the plant
    and clock rows expensive). Each calibration round renders on the current bands, measures every rank's
    band time and visits (measure_row_cost) and cuts new bands at equal quantiles of the mean of all rounds'
    per-row cost estimates; the renderer is then rebuilt on the final plan. Every rank derives the same bounds
    from all-reduced data."""
    import numpy as np

    r = BandRenderer(scene, W, H, cfg, rank, world, dist, **kw)
    if not balance or world == 1:
        return r
    est = []
    for _ in range(max(rounds, 1)):
        r.frame()
        est.append(r.measure_row_cost())
        bounds = balanced_bounds(np.mean(est, axis=0), world)
        r.close()
        r = BandRenderer(scene, W, H, cfg, rank, world, dist, bounds=bounds, **kw)
    return r
