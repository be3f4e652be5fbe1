"""Screen-band sharding of one frame across GPUs.

One process per GPU; rank r renders the horizontal band of global rows
[y0, y1). The path tracer is embarrassingly parallel (RNG seeds use global pixel
coordinates, path_tracing.frag:433-436), and so is the G-buffer: both compute the
owned rows only. The SVGF passes are bounded stencils; before each one the ranks
exchange the rows it reads outside their bands (torch.distributed P2P: RCCL over
xGMI on the GPU, gloo on the CPU tests).

Every frame-sized plane is stored with `ghost` rows either side of the band:
rows [row0, row1) = [y0 - ghost, y1 + ghost) clipped to the frame. Ghost rows are
storage only: nothing computes them, an exchange fills the ones a pass reads.

How many rows each pass reads beyond the band (HALO_SCHEDULE):
  * reprojection (svgf_reproject.frag:45-156): the history is fetched at uv - motion,
    bilinearly, with +1-texel taps and a 3x3 fallback: at most ceil(M*H) + 3 rows,
    M = the largest |motion.y| (UV units) over the frame's surface pixels THIS
    frame. The G-buffer kernel reduces M on the device (pt_pass_set_motion_bound);
    the ranks all-reduce MAX on the host (a gloo group), so every pair of ranks
    agrees on the count. History planes: previous a-trous iteration-1 output and
    moments; the previous normal/depth plane only where M reaches past the rows
    the previous frame already exchanged;
  * variance (svgf_variance.frag:39-117): 3 rows of illumination + moments; the
    G-buffer normal/depth plane once per frame, as many rows as the widest a-trous
    iteration reads (2 * 2^(n-1), svgf_Atrous.frag:92-97), for variance and every
    a-trous iteration;
  * a-trous iteration i: 2 * 2^i rows of its input;
  * TAA (taa.frag:19-39, 88-98, 137-139): 2 rows of the modulated colour and the
    velocity (3x3 neighbourhood and closest-depth tap, each a LINEAR fetch whose
    zero-weight neighbour row the sampler still reads), ceil(M*H) + 3 rows of the
    TAA history (fetched at the pixel's own uv - velocity).
A row is exchanged between ANY two ranks whose intervals meet (a halo may span
several thin bands). A motion beyond the ghost rows raises instead of reading
stale or clamped rows.

HALO_SCHEDULE is the single source of truth; BandRenderer (GPU) and
tests/test_dist_gloo.py (CPU, oracle) both execute it through run_stage().
"""
from __future__ import annotations

import math
import os
from dataclasses import dataclass

# a-trous radius 2*step (svgf_Atrous.frag:92-97) for step 1 << i; the reference allows up to 8 iterations
# (main.cpp:383); variance radius 3 (svgf_variance.frag:68)
ATROUS_HALO = [2 * (1 << i) for i in range(8)]
VARIANCE_HALO = 3
REPROJ_REACH = 3  # rows beyond |motion| the history taps reach: bilinear + 1-texel tap / 3x3 fallback + rounding
TAA_NEIGHBOURS = 2  # rows of the TAA 3x3 neighbourhood: +-1 texel, plus the LINEAR sampler's zero-weight row
GHOST = 96        # default stored rows either side of a band (storage only); motion up to GHOST - 3 rows per frame
GHOST_ZONE_GHOST = 128  # ghost zone: storage for 65 margin rows + up to 63 rows of history reach per frame
MIN_BAND_ROWS = 16
BAND_VISIT_BUDGET = 256  # shadow / closest-hit visits before a band's ray goes to the cooperative walk (the renderer's
                         # default since round 5, renderer.VISIT_BUDGET)
BAND_REFILL_WAVES = 1280  # resident waves a band's lane-refill launch is sized for (the chip: 5120)

# stage -> ((plane, rows), ...) exchanged before that stage; rows: int, or "reproj" / "reproj_nd" (set from this
# frame's motion bound) / "nd" (the widest a-trous halo of the configured iterations)
HALO_SCHEDULE = (
    ("reproject", (("prev_illum", "reproj"), ("prev_moments", "reproj"), ("prev_nd", "reproj_nd"))),
    ("variance", (("illum", VARIANCE_HALO), ("moments", VARIANCE_HALO), ("nd", "nd"))),
    *((f"atrous{i}", (("atrous_in", ATROUS_HALO[i]),)) for i in range(8)),
    ("taa", (("modulate", TAA_NEIGHBOURS), ("velocity", TAA_NEIGHBOURS), ("prev_taa", "reproj"))),
)
STAGES = {st: planes for st, planes in HALO_SCHEDULE}


def nd_halo(iterations: int) -> int:
    """Rows of the G-buffer normal/depth plane the SVGF passes read beyond the band."""
    return max([VARIANCE_HALO] + ATROUS_HALO[:max(0, int(iterations))])


def svgf_margins(iterations: int, taa: bool) -> dict:
    """Ghost zone (FrameShardRenderer): rows beyond a band each SVGF pass draws so that the band's rows need no halo
    exchange but the history's. Going backwards from what must be right: modulate on the band (+ TAA's 2-row
    neighbourhood), a-trous iteration i valid on its input's margin minus 2 * 2^i rows (svgf_Atrous.frag:92-97),
    variance 3 rows inside reproject (svgf_variance.frag:68). The a-trous iterations all draw iteration 0's rows (one
    per-tile flag set for all five; a later iteration's extra rows are never read)."""
    m = TAA_NEIGHBOURS if taa else 0
    v = m + sum(ATROUS_HALO[:max(0, int(iterations))])  # the variance output's margin
    out = {"taa": 0, "modulate": m, "atrous": v - ATROUS_HALO[0] if iterations > 0 else m, "variance": v,
           "reproject": v + VARIANCE_HALO}
    _check_early_history(out, int(iterations))
    return out


def _check_early_history(margins: dict, iterations: int) -> None:
    """The invariant the early history exchange (BandRenderer._early_history, issued on the RCCL stream while the back
    end still runs a-trous iterations 2..n-1) relies on. The exchange overwrites the rows of the iteration-1 output
    (hist_illum) and of this frame's normal/depth (prev_nd) outside the band with the owners' bits. Those rows may
    change under a running iteration only where nothing the band's final rows depend on reads them, or where the
    local bits equal the owner's:
      * iteration i >= 2 is exact on margin_i = v - sum(ATROUS_HALO[:i+1]) rows and reads its input (iteration i-1's
        output) ATROUS_HALO[i] rows further out, i.e. within margin_{i-1}: for i = 2 that is the iteration-1 output's
        own exact rows, whose local bits equal the owner's (same kernels, same inputs);
      * every iteration reads normal/depth at most ATROUS_HALO[i] rows beyond its exact rows, within the variance
        margin v, which the G-buffer draws (reproject margin + REPROJ_REACH > v): again the owner's bits.
    Raises if a change to the margins breaks either."""
    if iterations < 2:
        return
    v = margins["variance"]
    exact = [v - sum(ATROUS_HALO[:i + 1]) for i in range(iterations)]
    if exact[-1] < margins["modulate"]:
        raise AssertionError(f"a-trous margins {exact} leave the band's modulated rows inexact")
    for i in range(2, iterations):
        if exact[i] + ATROUS_HALO[i] > exact[i - 1]:
            raise AssertionError(f"a-trous iteration {i} reads beyond its input's exact rows: early history unsafe")
    if max(exact[i] + ATROUS_HALO[i] for i in range(iterations)) > margins["reproject"] + REPROJ_REACH:
        raise AssertionError("a-trous iterations read normal/depth rows the G-buffer does not draw")


def motion_rows(m: float, H: int) -> int:
    """Rows the history taps reach beyond a band for a largest |motion.y| of m (UV units) in an H-row frame."""
    if not math.isfinite(m):
        raise RuntimeError(f"non-finite G-buffer motion ({m}): the history rows a band needs are unbounded")
    return int(math.ceil(m * H)) + REPROJ_REACH


@dataclass
class BandPlan:
    W: int
    H: int
    rank: int
    world: int
    ghost: int = GHOST
    bounds: tuple | None = None  # world+1 row boundaries (balanced_bounds); None = equal bands
    iterations: int = 5          # a-trous iterations the bands serve (sizes the normal/depth halo)
    margins: dict | None = None  # ghost zone (svgf_margins): per-pass rows drawn beyond the band; None = HALO_SCHEDULE

    def __post_init__(self):
        b = list(self.bounds) if self.bounds is not None else [(self.H * k) // self.world for k in range(self.world + 1)]
        if len(b) != self.world + 1 or b[0] != 0 or b[-1] != self.H or any(x >= y for x, y in zip(b, b[1:])):
            raise ValueError(f"bad band bounds {b}")
        self.bounds = tuple(b)
        self.y0, self.y1 = b[self.rank], b[self.rank + 1]
        self.nd_rows = nd_halo(self.iterations)
        if self.margins is not None and self.margins["reproject"] + REPROJ_REACH > self.ghost:
            raise ValueError(f"a ghost zone of {self.margins['reproject']} rows needs more than {self.ghost} ghost rows")
        if self.nd_rows > self.ghost:
            raise ValueError(f"{self.iterations} a-trous iterations read {self.nd_rows} rows beyond a band, more than "
                             f"its {self.ghost} ghost rows (BandPlan(ghost=...))")
        self.row0 = max(0, self.y0 - self.ghost)
        self.row1 = min(self.H, self.y1 + self.ghost)
        self.rows = self.row1 - self.row0
        self.up = self.rank - 1 if self.rank > 0 else None
        self.down = self.rank + 1 if self.rank < self.world - 1 else None
        self.motion = 0  # history rows of the current frame (set_motion)

    def set_motion(self, m: float) -> int:
        """This frame's all-reduced largest |motion.y| (UV) -> rows the history exchanges carry."""
        return self.set_rows(motion_rows(m, self.H))

    def set_rows(self, n: int) -> int:
        """Rows the history exchanges carry this frame (n = motion_rows of a bound on the frame's motion)."""
        # ghost zone: the reprojection's margin rows read the previous G-buffer's normal/depth n rows further out
        reach = n + (self.margins["reproject"] if self.margins is not None else 0)
        if reach > self.ghost:
            raise RuntimeError(f"the camera moved {n - REPROJ_REACH} rows in one frame; a band holds {self.ghost} "
                               f"ghost rows (history reach {reach}): build the band renderer with a larger ghost")
        self.motion = int(n)
        return self.motion

    def capacity(self) -> int:
        """The most history rows a frame can exchange: every ghost row the reprojection's taps may reach (a camera
        moving capacity() - REPROJ_REACH rows or fewer per frame fits)."""
        return self.ghost - (self.margins["reproject"] if self.margins is not None else 0)

    def stage_rows(self, stage: str) -> tuple:
        """Ghost zone: the rows the SVGF pass `stage` draws (the band widened by its margin, clipped to the frame)."""
        m = self.margins[stage]
        return max(0, self.y0 - m), min(self.H, self.y1 + m)

    def gbuffer_rows(self, k: int | None = None) -> tuple:
        """Ghost zone: the rows band k's G-buffer draws (default this rank's) — the reprojection's rows and the reach
        of its taps into the previous normal/depth at rest (REPROJ_REACH); a moving camera's further rows arrive with
        the history (history_items)."""
        a, b = self.owned(self.rank if k is None else k)
        r = self.margins["reproject"] + REPROJ_REACH
        return max(0, a - r), min(self.H, b + r)

    def history_items(self, planes: dict, n: int) -> list:
        """Ghost zone: the exchanges before the reprojection for a motion reach of n rows (motion_rows): the previous
        a-trous iteration-1 output and moments over the reprojection's margin + n rows, and the previous normal/depth
        over as many when n reaches past the G-buffer's own rows."""
        rows = self.margins["reproject"] + n
        items = [(planes["prev_illum"], rows), (planes["prev_moments"], rows)]
        if n > REPROJ_REACH and "prev_nd" in planes:
            items.append((planes["prev_nd"], rows))
        return items

    def zone(self, k: int) -> tuple:
        """Ghost zone: rows of rank k's band the path tracer's planes must hold (its reprojection's rows)."""
        a, b = self.owned(k)
        m = self.margins["reproject"] if self.margins is not None else 0
        return max(0, a - m), min(self.H, b + m)

    def rows_for(self, spec) -> int:
        if spec == "reproj":
            return self.motion
        if spec == "reproj_nd":  # the previous frame's normal/depth already holds nd_rows exchanged ghost rows
            return self.motion if self.motion > self.nd_rows else 0
        if spec == "nd":
            return self.nd_rows
        return int(spec)

    def owned(self, k: int) -> tuple:
        return self.bounds[k], self.bounds[k + 1]

    def halo_parts(self, n: int) -> list:
        """The point-to-point transfers of an n-row halo, in the order every rank issues them (so sends and
        receives pair up): (send?, first row, end row, peer) per part, peers ascending, this rank's sends to a peer
        before its receives from it. Pure function of the plan and n; cached (a frame issues it per SVGF stage)."""
        cache = self.__dict__.setdefault("_halo_parts", {})
        if n not in cache:
            me, mine, parts = self.rank, self.owned(self.rank), []
            for k in range(self.world):
                if k == me:
                    continue
                for part in self.need(k, n):       # rows of my band that rank k reads
                    a, b = _meet(mine, part)
                    if b > a:
                        parts.append((True, a, b, k))
                for part in self.need(me, n):      # rows of rank k's band that I read
                    a, b = _meet(self.owned(k), part)
                    if b > a:
                        parts.append((False, a, b, k))
            cache[n] = parts
        return cache[n]

    def need(self, k: int, n: int) -> tuple:
        """Rows rank k reads outside its band for a halo of n rows: ((above), (below)), clipped to the frame."""
        a, b = self.owned(k)
        return (max(0, a - n), a), (b, min(self.H, b + n))


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


def _meet(a: tuple, b: tuple) -> tuple:
    return max(a[0], b[0]), min(a[1], b[1])


def halo_exchange(items, plan: BandPlan, dist, group=None, wait: bool = True):
    """Fill the ghost rows each (tensor, n) item reads: every rank sends the rows of its band that another rank's
    n-row halo covers. Tensors are (rows, W, C) holding global rows [row0, row1) of this rank. wait=False (RCCL):
    return the works instead of making the current stream wait for them (gloo is host-blocking either way)."""
    items = [(t, int(n)) for t, n in items if int(n) > 0]
    if plan.world == 1 or not items:
        return []
    if max(n for _, n in items) > plan.ghost:
        raise RuntimeError(f"halo of {max(n for _, n in items)} rows exceeds the {plan.ghost} ghost rows")
    if items[0][0].is_cuda and dist.get_backend(group) == "gloo":
        # gloo has no device P2P: stage through host memory (tests run several ranks on one GPU this way)
        host = [(t.cpu(), n) for t, n in items]
        halo_exchange(host, plan, dist, group)
        for (t, _), (h, _) in zip(items, host):
            t.copy_(h)
        return []
    ops = []
    for t, n in items:
        for send, a, b, k in plan.halo_parts(n):
            ops.append(dist.P2POp(dist.isend if send else dist.irecv, t[a - plan.row0:b - plan.row0], k, group))
    works = dist.batch_isend_irecv(ops) if ops else []
    if wait:
        for req in works:
            req.wait()
        return []
    return works


def run_stage(stage: str, planes: dict, plan: BandPlan, dist, group=None) -> None:
    """Execute HALO_SCHEDULE's exchanges before `stage`; planes maps plane names to (rows, W, C) tensors."""
    items = [(planes[name], plan.rows_for(spec)) for name, spec in STAGES.get(stage, ()) if name in planes]
    halo_exchange(items, plan, dist, group)


_HOST_GROUP = {}


def host_group(dist):
    """A gloo group for the per-frame motion all-reduce (host values: no device stream is involved, so it cannot
    interleave with the RCCL halo traffic). Collective: every rank creates it at the same point."""
    if dist.get_backend() == "gloo":
        return None
    world = dist.group.WORLD
    key = (id(world), dist.get_rank(), dist.get_world_size())
    hit = _HOST_GROUP.get(key)
    # the cache holds the WORLD object it was made for, so its id cannot be reused while cached; a re-initialised
    # default group is a new object and gets a new gloo group
    if hit is None or hit[0] is not world:
        _HOST_GROUP[key] = hit = (world, dist.new_group(backend="gloo"))
    return hit[1]


def allreduce_motion(m: float, dist, group=None) -> float:
    """MAX over ranks of the per-rank largest |motion.y| (host float). (The CPU oracle tests size their halos with
    it; the GPU band renderers use a bound the host already holds, MotionCheck, and no per-frame collective.)"""
    import torch

    t = torch.tensor([m], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX, group=group)
    return float(t.item())


def camera_moved(cam, pre_viewproj) -> bool:
    """True unless this frame's projection * view equals the previous frame's pre_viewproj bit for bit. The G-buffer
    kernel forms both clip positions of a surface point with the same float arithmetic from those two matrices
    (kernels_pt.hip: motion = now - prev, capi.hip builds projection * view as camera.mat_mul does), so a camera that
    did not move gives motion exactly 0 at every pixel."""
    import numpy as np

    from .camera import mat_mul

    cur = mat_mul(cam.cam_proj_mat, cam.cam_view_mat)
    return not np.array_equal(cur.view(np.uint32), np.asarray(pre_viewproj, np.float32).reshape(16).view(np.uint32))


class MotionCheckError(RuntimeError):
    """A frame's measured motion needed more history rows than its exchange carried. `frame` is the first such frame:
    its SVGF output and every later frame's (the history carries it forward) are not the one-GPU frame's; discard them.
    Raised after the fact (MotionCheck verifies once the device bound's copy has landed, frames later)."""

    def __init__(self, frame: int, need: int, used: int):
        super().__init__(f"frame {frame}: the G-buffer's motion needs {need} history rows but {used} were exchanged "
                         f"(camera moved without the host seeing it: pre_viewproj and projection * view disagree); "
                         f"frames {frame} and later are not the one-GPU frames")
        self.frame, self.need, self.used = frame, need, used


class MotionCheck:
    """The history rows of each frame from a bound the host holds when it issues the frame's back end — no wait for
    the G-buffer and no per-frame collective (round 4 synchronised on the G-buffer's motion bound and all-reduced it
    over gloo on every frame, a host round trip on every rank's critical path):
      * a camera that did not move (camera_moved False): motion is 0 at every pixel, the taps reach REPROJ_REACH rows;
      * a moved camera: the plan's capacity() — every ghost row the taps can reach (a camera moving further than that
        in one frame was already an error).
    Every rank derives the same count from the same camera path, so the exchanges pair up without communicating. The
    device bound the G-buffer kernel reduces (pt_pass_set_motion_bound) is still copied to pinned host memory behind
    each G-buffer and checked later, once its copy has landed (poll; never waited for unless a ring slot comes round
    again), against the rows the frame used: a frame whose motion exceeded them raises MotionCheckError (verify) — the
    bound is verified, not trusted. The check runs AFTER the fact: by the time it raises, that frame and possibly
    several later ones have been drawn with the short history; the error names the first bad frame (`frame`), from
    which on the output is to be discarded. A moved camera exchanges capacity() rows (63 with the ghost zone, 96
    without) whatever it actually moved: a host bound from the camera delta alone is not finite (a point at the near
    plane moves without limit under any translation), so the rows are sized for the worst the ghost can hold."""

    RING = 64

    def __init__(self, plan: BandPlan):
        import torch

        self.plan = plan
        self.host = torch.zeros(self.RING, dtype=torch.int32).pin_memory()
        self.ev = [None] * self.RING
        self.slot_frame = [None] * self.RING
        self.pending = []   # ring slots with a copy in flight, capture order
        self.moved = {}     # frame -> camera moved (host)
        self.used = {}      # frame -> history rows its exchange carried
        self.log = []       # (frame, rows the measured motion needs, rows used)
        self.first_bad = None  # the first frame whose motion needed more rows than it exchanged (MotionCheckError)

    def note_camera(self, f: int, moved: bool) -> None:
        self.moved[f] = bool(moved)

    def capture(self, f: int, dev_word, stream) -> None:
        """Copy frame f's device motion bound (its G-buffer wrote it on `stream`) to the host ring."""
        import torch

        j = f % self.RING
        if self.slot_frame[j] is not None:
            self._check(j, block=True)
        with torch.cuda.stream(stream):
            self.host[j:j + 1].copy_(dev_word, non_blocking=True)
            ev = torch.cuda.Event()
            ev.record(stream)
        self.ev[j], self.slot_frame[j] = ev, f
        self.pending.append(j)

    def rows(self, f: int) -> int:
        """History rows for frame f (host bound; plan.set_rows checks the ghost)."""
        moved = self.moved.pop(f, True)
        n = self.plan.capacity() if moved else REPROJ_REACH
        self.used[f] = n
        if len(self.used) > 2 * self.RING:  # frames whose bound another rank captures (shipped G-buffer)
            for old in sorted(self.used)[:len(self.used) - self.RING]:
                del self.used[old]
        self.poll()
        return n

    def poll(self, block: bool = False) -> None:
        """Check every captured bound whose copy has landed (block: wait for all of them)."""
        keep = []
        for j in self.pending:
            f = self.slot_frame[j]
            if f in self.used and (block or self.ev[j].query()):
                self._check(j, block=block)
            else:
                keep.append(j)
        self.pending = keep

    def _check(self, j: int, block: bool) -> None:
        import numpy as np

        f, ev = self.slot_frame[j], self.ev[j]
        if block:
            ev.synchronize()
        self.slot_frame[j] = self.ev[j] = None
        if j in self.pending:
            self.pending.remove(j)
        n = self.used.pop(f, None)
        if n is None:  # the frame's back end never exchanged a history (calibration frames, a renderer closed early)
            return
        m = float(self.host[j:j + 1].numpy().view(np.float32)[0])
        need = motion_rows(m, self.plan.H)
        self.log.append((f, need, n))
        if need > n:
            if self.first_bad is None or f < self.first_bad[0]:
                self.first_bad = (f, need, n)
            raise MotionCheckError(*self.first_bad)

    def verify(self) -> None:
        """Wait for every captured bound and check it (flush / close: the frames drawn so far); raises
        MotionCheckError naming the first frame whose exchange fell short."""
        self.poll(block=True)
        if self.first_bad is not None:
            raise MotionCheckError(*self.first_bad)


class _StageFilter:
    """A halo callback with the set of stages it acts on (Renderer._halo skips the rest)."""

    def __init__(self, fn, stages):
        self.fn = fn
        self.stages = frozenset(stages)

    def __call__(self, stage, handles):
        return self.fn(stage, handles)


class BandRenderer:
    """One rank's share of a frame: the fast Renderer on band storage + HALO_SCHEDULE exchanges."""

    def __init__(self, scene, W, H, cfg, rank, world, dist, bounds=None, ghost=None, ghost_zone: bool = False, **kw):
        """ghost_zone: every SVGF pass draws its margin beyond the band (svgf_margins) over inputs that hold those
        rows — the G-buffer on every stored row, the path tracer's planes on the reprojection's rows (pt_source must
        provide them: FrameShardRenderer) — so the only rows that cross ranks are the history's, once per frame,
        before the reprojection (and the TAA history's before TAA)."""
        import torch

        from . import gl
        from .renderer import Renderer

        if ghost_zone and kw.get("pt_source") is None:
            # the margin rows the SVGF passes draw read colour / emission / albedo the band's own path tracer never
            # draws (it covers the band only): without a source of those rows the band silently differs from a frame
            raise ValueError("ghost_zone needs a pt_source that provides the path tracer's planes on plan.zone() rows "
                             "(FrameShardRenderer)")
        iters = cfg.num_atrous_iterations
        margins = svgf_margins(iters, kw.get("run_taa", False)) if ghost_zone else None
        if ghost is None:
            ghost = max(GHOST, nd_halo(iters)) if not ghost_zone else GHOST_ZONE_GHOST
        self.plan = BandPlan(W, H, rank, world, ghost=int(ghost), bounds=bounds, iterations=iters, margins=margins)
        self.ghost_zone = bool(ghost_zone)
        self.dist = dist
        self.exchange = True  # False only while calibrating (make_band_renderer): ranks time their bands alone
        self.stage_events = None  # (stage, event, event) per exchange while time_exchanges(True)
        self._group = host_group(dist) if world > 1 else None
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
        # frames in flight: the host issues frame f once frame f - K's SVGF is done (Renderer host_pace), which frame
        # f's front end waits for on the GPU anyway. The host no longer blocks on anything per frame otherwise
        # (MotionCheck), so unpaced it would queue frames without bound and each camera would reach the GPU long
        # before its frame's result
        kw.setdefault("host_pace", True)
        # frames in flight: issue the back end one frame behind the front end, so the host's wait for the motion
        # bound (before the reprojection exchange) finds a G-buffer issued a frame earlier (Renderer back_lag)
        if kw.get("frames_in_flight", 1) > 1:
            kw.setdefault("back_lag", min(int(os.environ.get("PTSVGF_BAND_LAG", "2")), kw["frames_in_flight"] - 1))
        if kw.get("frames_in_flight", 1) == 1:  # exchanges run on torch's stream: the draws must too
            from ._lib import check, pt
            check(pt().pt_set_stream(torch.cuda.current_stream().cuda_stream))
        self._hist_works = None  # ghost zone: the next frame's history exchange, started early
        if ghost_zone:
            kw["gbuffer_rows"] = self.plan.gbuffer_rows()
            kw["stage_rows"] = self.plan.stage_rows
            kw["early_history"] = self._early_history
        halo = self._halo
        if ghost_zone:  # only these stages exchange (the Renderer skips the others without a stream context)
            halo = _StageFilter(self._halo, ("reproject", "taa"))
        self.r = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, tex_factory=factory,
                          halo=halo, after_gbuffer=self._after_gbuffer, **kw)
        if ghost_zone:  # the G-buffer marks the a-trous tiles of the rows the a-trous passes draw
            a0, a1 = self.plan.stage_rows("atrous")
            for p in self.r.init_pass:
                p.set_uniform_int("atrous_rows_begin", a0)
                p.set_uniform_int("atrous_rows_end", a1)
        # per G-buffer set: the device motion bound the G-buffer kernel writes (checked later, MotionCheck)
        ng = len(self.r.gbuf)
        self._mb_dev = torch.zeros(ng, dtype=torch.int32, device=dev)
        for b, p in enumerate(self.r.init_pass):
            p.set_motion_bound(self._mb_dev[b:b + 1].data_ptr())
        self.mcheck = MotionCheck(self.plan)
        self._set_frame = {}  # G-buffer set -> the frame whose front end last used it
        self.camera = self.r.camera
        self.pass_path_tracing = self.r.pass_path_tracing
        if self.r.K > 1:
            # a band's traversal launches end on a few long rays: past 256 visits a ray is finished by a
            # wave-cooperative walk (same bits; simulated 8-band frame 1.22 -> 1.08 ms; the one-GPU frame, whose
            # launches are full, keeps them off)
            self.pass_path_tracing.set_uniform_int("shadow_budget", BAND_VISIT_BUDGET)
            self.pass_path_tracing.set_uniform_int("closest_budget", BAND_VISIT_BUDGET)
            # a band's refill launches are small and share the chip with the other frames in flight: sized for the
            # whole chip they get one chunk per wave (no refill); sized for a quarter of it they keep refilling
            # (8 simulated bands, same box: slowest non-edge band 1.35 -> 1.27 ms, profiles/r03/band_sim_r03.log)
            self.pass_path_tracing.set_uniform_int("refill_waves", BAND_REFILL_WAVES)

    @property
    def motion_log(self) -> list:
        """Per checked frame: (history rows its measured motion needs, rows exchanged)."""
        return [(need, n) for _, need, n in self.mcheck.log]

    def _note_frame(self, b: int) -> None:
        """Frame r.frame_index's front end uses G-buffer set b: remember whether its camera moved (host)."""
        f = self.r.frame_index
        self._set_frame[b] = f
        self.mcheck.note_camera(f, camera_moved(self.r.camera, self.r.pre_viewproj))

    def _after_gbuffer(self, b: int, stream) -> None:
        """The G-buffer of set b was issued on `stream`: copy its motion bound to the host behind it (checked later)."""
        self._note_frame(b)
        self.mcheck.capture(self.r.frame_index, self._mb_dev[b:b + 1], stream)

    def _motion(self, b: int | None = None) -> int:
        """History reach of the frame whose back end is being issued (or of G-buffer set b), from the bound the host
        holds (MotionCheck: no wait, no collective)."""
        b = self.r.back_set if b is None else b
        return self.plan.set_rows(self.mcheck.rows(self._set_frame[b]))

    def verify_motion(self) -> None:
        """Check every frame's device motion bound against the history rows it exchanged (waits for the frames)."""
        self.mcheck.verify()

    def _early_history(self, handles: dict, next_set) -> None:
        """Ghost zone, Renderer early_history: the a-trous iteration that writes the next frame's history has been
        issued (frame f); when the next frame's front end is issued too (G-buffer set next_set), size its history
        exchange from that G-buffer's motion bound and start it now, so it overlaps the rest of frame f's chain.
        Frame f + 1's reprojection waits for it."""
        if not self.exchange or next_set is None or self._hist_works is not None:
            return
        import torch

        cur = self.plan.motion
        n = self._motion(next_set)
        self.plan.motion = cur  # frame f's TAA stage still reads frame f's reach
        planes = {k: self._tensors[h] for k, h in handles.items()}
        e0 = None
        if self.stage_events is not None:
            e0 = torch.cuda.Event(enable_timing=True)
            e0.record()
        works = halo_exchange(self.plan.history_items(planes, n), self.plan, self.dist, wait=False)
        self._hist_works = (works, n, e0)

    def _halo(self, stage: str, handles: dict) -> None:
        if not self.exchange:
            return
        if stage == "reproject" and self._hist_works is not None:  # started early (_early_history): wait for it
            import torch

            works, n, e0 = self._hist_works
            self._hist_works = None
            self.plan.motion = n
            for w in works:
                w.wait()
            if e0 is not None and self.stage_events is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record()
                self.stage_events.append(("history", e0, e1))
            return
        if stage == "reproject":
            self._motion()
        planes = {k: self._tensors[h] for k, h in handles.items()}
        if self.ghost_zone:  # only the histories cross ranks (BandRenderer ghost_zone)
            p = self.plan
            if stage == "reproject":
                items = p.history_items(planes, p.motion)
            elif stage == "taa":
                items = [(planes["prev_taa"], p.motion)]
            else:
                return
            self._exchange_items(stage, items)
            return
        items = [(planes[name], self.plan.rows_for(spec)) for name, spec in STAGES.get(stage, ()) if name in planes]
        self._exchange_items(stage, items)

    def _exchange_items(self, stage: str, items) -> None:
        if self.stage_events is None:
            halo_exchange(items, self.plan, self.dist)
            return
        import torch

        # exchange time on the stream the SVGF passes run on: the exchange's rows are waited for there (RCCL's own
        # stream joins it at req.wait()), so the event pair spans the stage as the back end sees it
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
        e0.record()
        halo_exchange(items, self.plan, self.dist)
        e1.record()
        self.stage_events.append((stage, e0, e1))

    def time_exchanges(self, on: bool) -> None:
        """Record HIP events around every halo stage from now on (on) / stop (off); exchange_ms() reads them."""
        self.stage_events = [] if on else None

    def exchange_ms(self) -> dict:
        """Per stage: mean ms per frame between the events around its exchanges (after the frames finished), and
        the frames counted. Synchronises."""
        import torch

        torch.cuda.synchronize()
        tot, n = {}, {}
        for stage, e0, e1 in self.stage_events or []:
            tot[stage] = tot.get(stage, 0.0) + e0.elapsed_time(e1)
            n[stage] = n.get(stage, 0) + 1
        return {s: round(tot[s] / n[s], 4) for s in tot}

    def frame(self) -> None:
        self.r.frame()

    def profile(self, on: bool) -> None:
        self.r.profile(on)

    def pass_times(self) -> dict:
        return self.r.pass_times()

    def time_atrous(self, reps: int = 20) -> float:
        """The a-trous kernels' average launch time (Renderer.time_atrous). The replay runs without exchanges, so
        iterations 1-4 read ghost rows that the frame's LATER exchanges refilled: the band planes it leaves are not
        the frame's (read what a frame produced before calling this)."""
        return self.r.time_atrous(reps)

    def trace_stats(self) -> dict:
        return self.r.trace_stats()

    def rows_rendered(self) -> int:
        return self.plan.y1 - self.plan.y0

    def planes(self) -> dict:
        pl = self.r.planes()
        self.verify_motion()
        return pl

    def close(self) -> None:
        self.verify_motion()  # the frames whose back end was issued
        self.r.close()
        self._tensors.clear()

    def measure_row_cost(self, frames: int = 32):
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
        torch.cuda.synchronize()  # zeroed before the path tracer adds to it on the renderer's front-end stream
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
        # host tensors over the host group (gloo): every rank must read the same sums, since they cut the next bands
        visits = torch.zeros(H, dtype=torch.float64)
        visits[p.y0:p.y1] = counts.cpu().to(torch.float64)
        per_rank = torch.zeros(p.world, dtype=torch.float64)
        per_rank[p.rank] = frame_ms
        self.dist.all_reduce(visits, group=self._group)
        self.dist.all_reduce(per_rank, group=self._group)
        self.last_band_ms = per_rank.numpy()  # every rank's band time alone (ms per frame)
        return band_row_cost(visits.cpu().numpy(), p.bounds, self.last_band_ms)


_SCATTER_GROUP = {}


def scatter_group(dist):
    """A second process group (same backend) for the frame-shard scatter: its RCCL communicator has its own stream,
    so a receive waiting for another rank's path tracer never queues the band halo exchanges behind it.
    Collective: every rank creates it at the same point."""
    import torch

    world = dist.group.WORLD
    key = (id(world), dist.get_rank(), dist.get_world_size())
    hit = _SCATTER_GROUP.get(key)
    if hit is None or hit[0] is not world:
        backend = dist.get_backend()
        g = dist.new_group(backend=backend)
        if backend == "gloo":
            dist.barrier(group=g)
        else:  # the first operation on a group involves every rank (batch_isend_irecv requires it when it comes first)
            dist.barrier(group=g, device_ids=[torch.cuda.current_device()])
        _SCATTER_GROUP[key] = hit = (world, g)
    return hit[1]


def exchange_window(window, plan: BandPlan, dist, group=None, rows=None) -> int:
    """The point-to-point transfers of one frame-shard window: consecutive frames (frame f is traced by rank
    (f // burst) % N, so a source holds up to min(burst, window) of them, each in its own slot). window = [(src,
    planes)] in frame order: for a frame this rank traced, planes are its whole-frame
    (H, W, C) tensors and every other band's rows (plan.zone: the band, widened by the ghost zone's reprojection
    margin) go to that band's owner; for a frame rank src traced, planes are this band's zone rows, received from src. Every rank builds the same window, so the batch is symmetric: an
    all-to-all over the window's sources, every link busy at once, one communicator. rows[j](k) (default plan.zone):
    the rows of band k plane j carries. RCCL: the current stream waits for the batch; gloo (tests): blocking, device
    tensors staged through host memory. Returns the bytes sent."""
    import torch

    gloo = dist.get_backend(group) == "gloo"
    ops, staged, nbytes = [], [], 0
    for src, planes in window:
        if src == plan.rank:
            for k in range(plan.world):
                if k == plan.rank:
                    continue
                for j, t in enumerate(planes):
                    y0, y1 = (rows[j] if rows else plan.zone)(k)
                    part = t[y0:y1]
                    if gloo and part.is_cuda:
                        part = part.cpu()
                    ops.append(dist.P2POp(dist.isend, part, k, group))
                    nbytes += part.numel() * part.element_size()
        else:
            for t in planes:
                buf = t
                if gloo and t.is_cuda:
                    buf = torch.empty(t.shape, dtype=t.dtype)
                    staged.append((t, buf))
                ops.append(dist.P2POp(dist.irecv, buf, src, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for t, h in staged:
        t.copy_(h)
    return nbytes


class FrameShardRenderer(BandRenderer):
    """Frames interleaved across ranks for the path tracer, bands for the SVGF chain.

    The G-buffer + path tracer of frame f (the front end: camera in, colour / emission / albedo out, no history) are
    traced over the WHOLE frame by rank f % N, so every traversal launch is a full frame's (a band's launches are an
    N-th of that and end on the same longest rays: DESIGN.md "What limits strong scaling"). The SVGF chain is
    sequential through its history, so it stays banded exactly as in BandRenderer: every rank draws its band's
    G-buffer (per pixel, nothing to exchange), receives its rows of the path tracer's planes and runs reproject /
    variance / a-trous / modulate with the HALO_SCHEDULE exchanges. Same kernels on the same inputs: the bands equal
    a one-GPU frame bit for bit.

    The SVGF passes draw a ghost zone (BandRenderer ghost_zone, svgf_margins): the G-buffer covers every stored row
    and the path tracer's planes arrive with the reprojection's margin, so per frame only the history rows cross
    ranks, once, before the reprojection (7 halo stages per frame become 1).

    The path tracer's rows travel once per window of N consecutive frames (exchange_window on a group of their own, scatter_group:
    RCCL over xGMI): each rank sends its traced frame's rows to every other band and receives its band's rows of the
    other N - 1 frames, all links at once. A frame's back end waits for its window, so the back end runs back_lag = N
    frames behind the front end, and frames_in_flight (band slots) must cover that plus a path tracer's latency.
    Per rank and N frames: one full-frame front end + N band G-buffers and SVGF chains. own_slots = whole frames this
    rank traces at once (the path tracer's streams)."""

    GBUF_PLANES = (1, 2, 3)  # G-buffer attachments the SVGF chain reads: normal/depth, motion, depth-fwidth

    def __init__(self, scene, W, H, cfg, rank, world, dist, own_slots: int = 2, ship_gbuffer: bool | None = None,
                 window: int | None = None, burst: int = 1, own_budget: int = 0, own_refill_waves: int = 0, **kw):
        """burst (default 1): consecutive frames one rank traces, frame f on rank (f // burst) % N. With 2 a rank's
        two path tracers are issued one frame apart and overlap (their launch tails fill each other's idle CUs, as frames
        in flight do on one GPU) instead of starting N frames apart.

        window (default N): frames whose rows travel in one exchange. N: one all-to-all per N frames (every rank
        sends its traced frame and receives the N - 1 others, all links at once), and a frame's back end waits for its
        window: back_lag = N. 1: frame f's rows go out from rank f % N alone as soon as they are traced (one-to-all per
        frame), back_lag = 1, so fewer band slots (frames_in_flight) cover the same path-tracer latency and the
        camera-to-modulate latency falls with them.

        ship_gbuffer (default off): the frame's tracing rank also sends each band the rows of its G-buffer
        (normal/depth, motion, depth-fwidth on the band's G-buffer rows), which the band adopts (pt_raster_pass_adopt)
        instead of drawing its own. A band's G-buffer draw costs 0.06-0.25 ms per frame (the plant's rows dominate)
        against 0.01 for the adoption, for twice the window's bytes (≈ 150 MB per window and link at 8 ranks); the
        8-rank simulation measured it within noise (0.93-1.11 vs 0.90-0.99 ms per frame,
        profiles/r03/frame_shard/fs_ship*.log), so it stays an option.

        own_budget / own_refill_waves (0: the one-GPU settings, renderer.VISIT_BUDGET and the whole chip): the
        whole-frame path tracer's cooperative-walk visit budget (shadow_budget / closest_budget) and the resident waves
        its lane-refill launches are sized for (refill_waves) — the tail tools; a rank's own frames are N frames apart,
        so its path tracer runs nearly alone, as one frame at a time does on one GPU (8-rank simulation, window 4, K 16:
        0.962 ms equal bands without budgets, 0.913 balanced with them; K 24 balanced 0.890 / 0.887 without / with,
        profiles/r05/shard/)."""
        import torch

        from . import gl
        from .renderer import Renderer, acquire_stream

        K = kw.get("frames_in_flight", 1)
        self.window = int(window) if window else world
        self.burst = int(burst)
        if self.burst < 1:
            raise ValueError(f"burst must be >= 1, got {burst}")
        if not 1 <= self.window <= world:
            raise ValueError(f"window must be in [1, {world}], got {window}")
        # a window may hold min(burst, window) frames this rank traces; each needs its own slot until the window's
        # exchange has sent it (_render_own waits only for the exchange that sent a slot's previous frame)
        if max(2, int(own_slots)) < min(self.burst, self.window):
            raise ValueError(f"own_slots = {own_slots} < min(burst, window) = {min(self.burst, self.window)}: a window "
                             f"would reuse a slot whose frame it has not sent yet")
        kw.setdefault("back_lag", self.window)  # a frame's back end is issued after its window's exchange
        if K <= kw["back_lag"]:
            raise ValueError(f"FrameShardRenderer needs frames_in_flight > back_lag = {kw['back_lag']}, got {K}")
        self._full_tensors = {}
        dev = torch.device("cuda", torch.cuda.current_device())

        def full_factory(w, h):
            t = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
            handle = gl.wrap_device_texture(t.data_ptr(), w, h)
            self._full_tensors[handle] = t
            return handle

        gl.set_band(W, H, 0, H, 0, H)  # the library's band state is process-global: the full renderer's planes are whole
        self.full = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, tex_factory=full_factory,
                             run_taa=False, run_output=False, frames_in_flight=max(2, int(own_slots)))
        for p in self.full.init_pass:
            p.set_rows(0, H)
        for p, _ in self.full.pt_slots:
            p.set_rows(0, H)
        self.own_slots = self.full.K
        # experiment (PTSVGF_OWN_CU_RESERVE = R): the whole-frame path tracer's streams never use R CUs spread over the
        # XCDs, so the band's G-buffer and SVGF chain (sequential through its history, a chain of short launches) always
        # find free CUs beside the long traversal launches
        self._masked = []
        reserve = int(os.environ.get("PTSVGF_OWN_CU_RESERVE", "0"))
        if reserve > 0:
            import ctypes as C

            from ._lib import check, pt
            from .renderer import masked_stream, release_stream, reserved_cus

            n = C.c_int()
            check(pt().pt_device_cus(C.byref(n)))
            excl = reserved_cus(n.value, reserve)
            for i in range(len(self.full._streams)):
                st, h = masked_stream(excl)
                release_stream(self.full._streams[i])  # the pool's stream goes back unused
                self.full._streams[i] = st
                self._masked.append(h)
        # experiment (PTSVGF_OWN_PRIORITY = P, e.g. 1 = HIP's low): the whole-frame path tracer's streams at queue
        # priority P, below the band's G-buffer (normal) and SVGF chain (high)
        own_prio = os.environ.get("PTSVGF_OWN_PRIORITY")
        if own_prio is not None and reserve <= 0:
            from .renderer import priority_stream, release_stream

            for i in range(len(self.full._streams)):
                st, h = priority_stream(int(own_prio))
                release_stream(self.full._streams[i])  # the pool's stream goes back unused
                self.full._streams[i] = st
                self._masked.append(h)
        self._own_free = [None] * self.own_slots  # event: the window exchange that sent the slot's last frame is done
        self._win = []  # frames registered since the last window exchange
        kw.setdefault("front_streams", 1)  # band front ends are a G-buffer each: one stream, in order
        kw.setdefault("ghost_zone", True)
        self.ship_gbuffer = bool(ship_gbuffer)
        if self.ship_gbuffer and not kw["ghost_zone"]:
            raise ValueError("ship_gbuffer needs the ghost zone")
        if self.ship_gbuffer:
            kw["draw_gbuffer"] = False
            # the tracing rank's whole-frame G-buffer reduces the frame's motion bound (the bands draw none); that rank
            # checks it against the rows every band exchanged (MotionCheck)
            nb = len(self.full.init_pass)
            self._fmb_dev = torch.zeros(nb, dtype=torch.int32, device=dev)
            for b, p in enumerate(self.full.init_pass):
                p.set_motion_bound(self._fmb_dev[b:b + 1].data_ptr())
        super().__init__(scene, W, H, cfg, rank, world, dist, pt_source=self._pt_source, pt_flush=self._exchange,
                         **kw)
        self.full.camera = self.r.camera  # one camera: the full front end draws the band renderer's frame
        self.pass_path_tracing = self.full.pass_path_tracing
        if own_budget > 0:
            self.pass_path_tracing.set_uniform_int("shadow_budget", int(own_budget))
            self.pass_path_tracing.set_uniform_int("closest_budget", int(own_budget))
        if own_refill_waves > 0:
            self.pass_path_tracing.set_uniform_int("refill_waves", int(own_refill_waves))
        self._sgroup = scatter_group(dist) if world > 1 else None
        self._recv_stream = acquire_stream()
        self.scatter_log = []  # per exchange that carried a frame of this rank: bytes sent
        self.own_events = None  # a list: (frame, start, end) HIP events of each own front end (diagnostics)

    def source(self, f: int) -> int:
        """The rank that traces frame f."""
        return (f // self.burst) % self.plan.world

    def own_index(self, f: int) -> int:
        """Ordinal of frame f among the frames its rank traces."""
        return (f // (self.burst * self.plan.world)) * self.burst + f % self.burst

    def _band_rows(self, handle):
        p = self.plan
        a, b = p.zone(p.rank)
        return self._tensors[handle][a - p.row0:b - p.row0]

    def _pt_source(self, f: int, slot: int, stream):
        """Renderer pt_source: register frame f in the current window (exchanging the previous window when it is
        full); when f is this rank's, trace the whole frame and copy its own band's rows. Returns the holder whose
        "ev" the back end of f waits for (set when f's window is exchanged)."""
        import torch

        r, p = self.r, self.plan
        if len(self._win) == self.window:
            self._exchange()
        holder = {}
        gset = f % len(r.gbuf)
        if self.ship_gbuffer:  # (drawn G-buffers note their frame in _after_gbuffer)
            self._note_frame(gset)
        item = dict(src=self.source(f), outs=[self._band_rows(h) for h in r.pt_slots[slot][1]],
                    free=r._slot_free[f % r.K], holder=holder, gset=gset)
        if self.ship_gbuffer:
            g0, g1 = p.gbuffer_rows()
            ip = r.init_pass[gset]
            item["outs"] += [self._tensors[ip.colorAttachments[j]][g0 - p.row0:g1 - p.row0] for j in self.GBUF_PLANES]
        if item["src"] == p.rank:
            o, pt_done = self._render_own(f)
            r._stream_to(stream)  # the library's stream is process-global: back to the band's front-end stream
            full = [self._full_tensors[h] for h in self.full.pt_slots[o][1]]
            if self.ship_gbuffer:
                full += [self._full_tensors[self.full.init_pass[o].colorAttachments[j]] for j in self.GBUF_PLANES]
            rs = self._recv_stream
            if item["free"] is not None:
                rs.wait_event(item["free"])
            rs.wait_event(pt_done)
            rows = self._plane_rows()
            with torch.cuda.stream(rs):
                for j, (a, b) in enumerate(zip(item["outs"], full)):
                    z0, z1 = rows[j](p.rank)
                    a.copy_(b[z0:z1])
            if self.ship_gbuffer:
                self._adopt(gset, rs)
                r._stream_to(stream)
            ev = torch.cuda.Event()
            ev.record(rs)
            holder["ev"] = ev
            item.update(o=o, full=full)
        self._win.append(item)
        return holder

    def _plane_rows(self):
        """Per window plane, the rows of band k it carries: the path tracer's planes on the band's zone, the
        G-buffer's on the band's G-buffer rows."""
        p = self.plan
        return [p.zone] * 3 + ([p.gbuffer_rows] * len(self.GBUF_PLANES) if self.ship_gbuffer else [])

    def _adopt(self, gset: int, stream) -> None:
        """The band's G-buffer set holds its rows of a frame drawn by the tracing rank: make the a-trous side data
        (pt_raster_pass_adopt) on `stream`, behind the rows' arrival."""
        r = self.r
        r._stream_to(stream)
        r.init_pass[gset].adopt(*self.plan.gbuffer_rows())

    def _exchange(self) -> None:
        """Send / receive the rows of the registered window (every rank registers the same frames, so every rank
        calls this at the same point: when a window is full, and on flush)."""
        import torch

        win, self._win = self._win, []
        if not win:
            return
        p, rs = self.plan, self._recv_stream
        for it in win:  # receives overwrite band slots: the SVGF chains that read them K frames ago are done
            if it["src"] != p.rank and it["free"] is not None:
                rs.wait_event(it["free"])
        window = [(it["src"], it["full"] if it["src"] == p.rank else it["outs"]) for it in win]
        with torch.cuda.stream(rs):
            nbytes = exchange_window(window, p, self.dist, self._sgroup, rows=self._plane_rows()) if p.world > 1 else 0
        if self.ship_gbuffer:
            cur = self.r._lib_stream
            for it in win:
                if it["src"] != p.rank:
                    self._adopt(it["gset"], rs)
            if cur is not None:
                self.r._stream_to(cur)
        ev = torch.cuda.Event()
        ev.record(rs)
        for it in win:
            if it["src"] != p.rank:
                it["holder"]["ev"] = ev
            else:
                self._own_free[it["o"]] = ev  # the slot's frame has been sent
                self.scatter_log.append(nbytes)

    def _render_own(self, f: int):
        """G-buffer + path tracer of frame f over the whole frame on an own stream. Returns (own slot, event after
        the path tracer)."""
        import torch

        fr, p = self.full, self.plan
        o = self.own_index(f) % self.own_slots
        st = fr._streams[o]
        if self._own_free[o] is not None:
            st.wait_event(self._own_free[o])
        t0 = None
        if self.own_events is not None:  # diagnostics: when this own front end starts and ends on its stream
            t0 = torch.cuda.Event(enable_timing=True)
            t0.record(st)
        fr._use_slot(o)
        fr._stream_to(st)
        fr.pre_viewproj = self.r.pre_viewproj
        fr.frame_index = f
        fr._gbuffer(o)
        if self.ship_gbuffer:  # the whole frame's motion bound, checked here for every band (MotionCheck)
            self.mcheck.capture(f, self._fmb_dev[o:o + 1], st)
        fr._path_trace(fr.gbuf[o])
        done = torch.cuda.Event(enable_timing=t0 is not None)
        done.record(st)
        if t0 is not None:
            self.own_events.append((f, t0, done))
        return o, done

    def trace_stats(self) -> dict:
        """Traversal counters of one frame: the rank tracing it counts the whole frame, the others nothing (bench
        sums over ranks)."""
        import torch

        buf = torch.zeros(len(self.r.STAT_KEYS), dtype=torch.int64, device="cuda")
        self.r.flush()
        torch.cuda.synchronize()
        for p, _ in self.full.pt_slots:
            p.set_trace_stats(buf.data_ptr(), buf.numel())
        try:
            self.r.frame()
            self.r.flush()
            torch.cuda.synchronize()
        finally:
            for p, _ in self.full.pt_slots:
                p.set_trace_stats(0)
        return dict(zip(self.r.STAT_KEYS, (int(v) for v in buf.cpu().tolist())))

    def profile(self, on: bool) -> None:
        self.r.profile(on)
        self.full.profile(on)

    def band_ms(self, frames: int | None = None) -> float:
        """This rank's band work per frame (its G-buffer and SVGF passes, each draw timed alone with HIP events;
        the whole-frame path tracer, the same on every rank, is not counted). Collective: every rank draws the same
        frames. Calibration only (make_frame_shard_renderer)."""
        import torch

        frames = frames or 2 * self.plan.world
        for _ in range(self.r.K + self.plan.world):  # every slot once: first use allocates
            self.frame()
        self.r.flush()
        torch.cuda.synchronize()
        self.profile(True)
        try:
            for _ in range(frames):
                self.frame()
            self.r.flush()
            torch.cuda.synchronize()
            ms = self.r.pass_times().get("frame_sum_ms", 0.0) / frames
        finally:
            self.profile(False)
        return ms

    def pass_times(self) -> dict:
        out = self.r.pass_times()
        for k, v in self.full.pass_times().items():
            if k in ("gbuffer", "pathtrace"):
                out["full_" + k] = v
        return out

    def close(self) -> None:
        from .renderer import release_stream

        super().close()
        self.full.close()
        self._full_tensors.clear()
        release_stream(self._recv_stream)
        self._recv_stream = None
        if self._masked:
            from ._lib import check, pt

            for h in self._masked:
                check(pt().pt_stream_destroy(h))
            self._masked = []


def tile_layout(plan: BandPlan, W: int, batch: int, count):
    """The tile shard's message layout (pixels, every plane of a pixel together), fixed per plan: send [peer k][frame b]
    blocks of this rank's tiles of band k's zone (n_send[k] pixels per frame), recv [source s][frame b] blocks of s's
    tiles of this band's zone (n_recv[s] per frame; this rank's own block included: the pack writes it, the unpack reads
    it with the others). count(offset, y0, y1): pixels of the subset `offset` in rows [y0, y1) (pt_tiles_count).
    Returns (n_send, send_base, n_recv, recv_base, send pixels, recv pixels)."""
    me = plan.rank
    n_send, send_base, off = {}, {}, 0
    for k in range(plan.world):
        if k != me:
            n_send[k] = count(me, *plan.zone(k))
            send_base[k] = off
            off += batch * n_send[k]
    n_recv, recv_base, off2 = {}, {}, 0
    for s in range(plan.world):
        n_recv[s] = count(s, *plan.zone(me))
        recv_base[s] = off2
        off2 += batch * n_recv[s]
    return n_send, send_base, n_recv, recv_base, off, off2


def tile_messages(layout, me: int, frames: int, elems: int):
    """(peer, first, end) element ranges of one batch of `frames` frames (elems elements per pixel): one message per
    peer each way, its frames contiguous. Both ends derive a pair's sizes from the same counts (my tiles of k's zone ==
    k's count of source me in its zone), so the batch pairs up."""
    n_send, send_base, n_recv, recv_base = layout[:4]
    sends = [(k, send_base[k] * elems, (send_base[k] + frames * n) * elems) for k, n in n_send.items()]
    recvs = [(s, recv_base[s] * elems, (recv_base[s] + frames * n) * elems) for s, n in n_recv.items() if s != me]
    return sends, recvs


def exchange_tiles(send, sends, recv, recvs, dist, group=None) -> int:
    """One tile-shard frame's all-to-all: sends = [(peer, first, end)] element ranges of the flat device buffer `send`
    (this rank's tiles of peer's band rows, every plane), recvs = [(source, first, end)] of `recv` (the source's tiles
    of this band's rows). One symmetric batch (every rank pairs its sends with its peers' receives), every link at
    once. RCCL: the current stream waits for the batch; gloo (tests): blocking, staged through host memory. Returns the
    bytes sent."""
    import torch

    gloo = dist.get_backend(group) == "gloo"
    ops, staged, nbytes = [], [], 0
    hsend = send.cpu() if gloo and send.is_cuda else send
    for k, a, b in sends:
        ops.append(dist.P2POp(dist.isend, hsend[a:b], k, group))
        nbytes += (b - a) * send.element_size()
    for s, a, b in recvs:
        buf = recv[a:b]
        if gloo and recv.is_cuda:
            h = torch.empty(buf.shape, dtype=buf.dtype)
            staged.append((buf, h))
            buf = h
        ops.append(dist.P2POp(dist.irecv, buf, s, group))
    if ops:
        for w in dist.batch_isend_irecv(ops):
            w.wait()
    for t, h in staged:
        t.copy_(h)
    return nbytes


class TileShardRenderer(BandRenderer):
    """Screen tiles across ranks for the path tracer, bands for the SVGF chain (north_star: "frames shard by
    screen-tile across the 8 GPUs").

    Every frame, rank r traces the 16 x 16 tiles t = k * N + r of the WHOLE frame (the path tracer's tile_stride /
    tile_offset subset; RNG seeds use global pixel coordinates, path_tracing.frag:433-436, so the N subsets compose to
    the one-GPU frame bit for bit): every rank holds an even share of the expensive tiles, and each traversal launch
    carries an N-th of the frame's rays. The SVGF chain is sequential through its history, so it stays banded exactly
    as in FrameShardRenderer (ghost zone, BandRenderer ghost_zone): every rank draws its band's G-buffer and runs
    reproject / variance / a-trous with the modulate fused, and only the histories cross ranks.

    Between the two, one all-to-all per batch of frames (exchange_tiles, on a communicator of its own, scatter_group):
    each rank packs its tiles of every other band's zone rows (plan.zone: the band widened by the reprojection's margin)
    into one contiguous message per peer (pt_tiles_copy, one launch per frame for all peers and planes), the messages
    travel over every xGMI link at once, and the band unpacks the N subsets of its zone into its colour / emission /
    albedo planes (one launch per frame).

    batch = B (default 1): the subsets of B consecutive frames are traced as one batched draw (pt_pass_draw_batch: each
    traversal launch carries B subsets' rays, so it fills the chip B times better — a lone subset's launches end on the
    frame's longest walks like a whole frame's) and exchanged as one message per peer. A frame's back end waits for its
    batch, so it runs back_lag = max(2, B) frames behind its front end (2: the host's motion-bound wait finds a G-buffer
    issued two frames earlier). own_slots = subsets this rank holds at once (at least 2B: one batch in flight while the
    next registers)."""

    PT_PLANES = 3  # colour, emission, albedo (the path tracer's outputs the SVGF chain reads)

    def __init__(self, scene, W, H, cfg, rank, world, dist, own_slots: int = 2, batch: int = 1, **kw):
        import torch

        from . import gl
        from .renderer import Renderer, acquire_stream

        if W % 16:
            raise ValueError(f"the tile shard needs a frame width that is a multiple of 16 (the path tracer's tiles), got {W}")
        self.batch = int(batch)
        if not 1 <= self.batch <= 8:
            raise ValueError(f"batch must be in [1, 8] (pt_pass_draw_batch), got {batch}")
        K = kw.get("frames_in_flight", 1)
        kw.setdefault("back_lag", min(max(2, self.batch), max(0, K - 1)))
        if K < 2 or kw["back_lag"] < self.batch - 1:
            raise ValueError(f"TileShardRenderer needs frames_in_flight >= 2 and back_lag >= batch - 1, got K = {K}, "
                             f"back_lag = {kw['back_lag']}")
        self._full_tensors = {}
        dev = torch.device("cuda", torch.cuda.current_device())

        def full_factory(w, h):
            t = torch.zeros((h, w, 4), dtype=torch.float32, device=dev)
            handle = gl.wrap_device_texture(t.data_ptr(), w, h)
            self._full_tensors[handle] = t
            return handle

        gl.set_band(W, H, 0, H, 0, H)  # process-global band state: the subset's planes are whole frames
        slots = max(2, int(own_slots), 2 * self.batch if self.batch > 1 else 1)
        self.full = Renderer(scene, W, H, cfg, mode="fast", aspect_corrected=True, tex_factory=full_factory,
                             run_taa=False, run_output=False, frames_in_flight=slots, trace_batch=self.batch)
        for p, _ in self.full.pt_slots:
            p.set_rows(0, H)
            p.set_uniform_int("tile_stride", world)
            p.set_uniform_int("tile_offset", rank)
        self.own_slots = self.full.K
        self._own_free = [None] * self.own_slots  # event: the pack that read the slot's last subset is done
        self._open = []  # frames of the batch being registered: (f, own slot, band slot, holder)
        kw.setdefault("front_streams", 1)
        kw["ghost_zone"] = True
        super().__init__(scene, W, H, cfg, rank, world, dist, pt_source=self._pt_source, pt_flush=self._flush_batch,
                         **kw)
        self.full.camera = self.r.camera
        self.pass_path_tracing = self.full.pass_path_tracing
        if self.r.K > 1 and self.batch == 1:
            # a lone subset's launches carry an N-th of the rays: the band's traversal settings (BandRenderer)
            self.pass_path_tracing.set_uniform_int("shadow_budget", BAND_VISIT_BUDGET)
            self.pass_path_tracing.set_uniform_int("closest_budget", BAND_VISIT_BUDGET)
            self.pass_path_tracing.set_uniform_int("refill_waves", BAND_REFILL_WAVES)
        self._sgroup = scatter_group(dist) if world > 1 else None
        self._recv_stream = acquire_stream()
        lay = tile_layout(self.plan, W, self.batch, lambda o, a, b: gl.tiles_count(W, world, o, a, b))
        self._n_send, self._send_base, self._n_recv, self._recv_base, ns, nr = lay
        self._send = torch.empty(max(1, ns) * self.PT_PLANES * 4, dtype=torch.float32, device=dev)
        self._recv = torch.empty(max(1, nr) * self.PT_PLANES * 4, dtype=torch.float32, device=dev)
        self.scatter_log = []  # bytes sent per frame

    def _ptr(self, buf, pixels: int) -> int:
        return buf.data_ptr() + pixels * self.PT_PLANES * 16

    def _pt_source(self, f: int, slot: int, stream):
        """Renderer pt_source: register frame f in the open batch (its subset's uniforms on own slot f % own_slots) and,
        when the batch is full, trace, exchange and unpack it. Returns the holder whose "ev" the back end of f waits
        for (set when f's batch is flushed)."""
        fr = self.full
        o = f % self.own_slots
        fr._use_slot(o)
        fr.frame_index = f
        holder = {}
        self._open.append((f, o, slot, holder))
        if self.batch == 1:  # a lone subset: drawn now, on its own stream
            st = fr._streams[o]
            if self._own_free[o] is not None:
                st.wait_event(self._own_free[o])
            fr._stream_to(st)
            fr._path_trace(None)  # the subset's primaries come from its own tile-binned raster (no G-buffer hint)
            self._flush_batch(drawn=st)
        else:
            fr._path_trace(None)  # uniforms only (trace_batch > 1): drawn with its batch
            if len(self._open) == self.batch:
                self._flush_batch()
        self.r._stream_to(stream)
        return holder

    def _flush_batch(self, drawn=None) -> None:
        """Trace the open batch (one pt_pass_draw_batch on the stream of its last own slot, unless `drawn` holds the
        lone subset's stream), pack every frame's tiles per peer, exchange them in one batch, unpack this band's zone.
        Every rank registers the same frames, so every rank flushes at the same point (batch full, or flush())."""
        import torch

        from . import gl

        items, self._open = self._open, []
        if not items:
            return
        r, p, fr = self.r, self.plan, self.full
        st = drawn
        if st is None:
            st = fr._streams[items[-1][1]]
            for _, o, _, _ in items:
                if self._own_free[o] is not None:
                    st.wait_event(self._own_free[o])
            fr._stream_to(st)
            gl.draw_batch([fr.pt_slots[o][0] for _, o, _, _ in items])
        done = torch.cuda.Event()
        done.record(st)
        rs = self._recv_stream
        rs.wait_event(done)
        for f, _, _, _ in items:
            free = r._slot_free[f % r.K]  # the band slot's planes: read by the SVGF chain of frame f - K
            if free is not None:
                rs.wait_event(free)
        r._stream_to(rs)
        me, c = p.rank, len(items)
        for b, (_, o, _, _) in enumerate(items):
            # my tiles: every other band's zone into the send buffer, my own band's zone straight into my recv slot
            segs = [(*p.zone(k), me, self._ptr(self._send, self._send_base[k] + b * n)) for k, n in self._n_send.items()]
            segs.append((*p.zone(me), me, self._ptr(self._recv, self._recv_base[me] + b * self._n_recv[me])))
            gl.tiles_copy(list(fr.pt_slots[o][1]), p.world, segs, unpack=False)
        packed = torch.cuda.Event()
        packed.record(rs)
        for _, o, _, _ in items:
            self._own_free[o] = packed
        sends, recvs = tile_messages((self._n_send, self._send_base, self._n_recv, self._recv_base), me, c,
                                     self.PT_PLANES * 4)
        with torch.cuda.stream(rs):
            nbytes = exchange_tiles(self._send, sends, self._recv, recvs, self.dist, self._sgroup) if p.world > 1 else 0
        r._stream_to(rs)
        for b, (_, _, slot, _) in enumerate(items):
            segs = [(*p.zone(me), s_, self._ptr(self._recv, self._recv_base[s_] + b * n)) for s_, n in self._n_recv.items()]
            gl.tiles_copy(list(r.pt_slots[slot][1]), p.world, segs, unpack=True)
        ev = torch.cuda.Event()
        ev.record(rs)
        for _, _, _, holder in items:
            holder["ev"] = ev
        self.scatter_log += [nbytes / c] * c

    def trace_stats(self) -> dict:
        """Traversal counters of one frame: each rank counts its tiles (bench sums over ranks)."""
        import torch

        buf = torch.zeros(len(self.r.STAT_KEYS), dtype=torch.int64, device="cuda")
        self.r.flush()
        torch.cuda.synchronize()
        for q, _ in self.full.pt_slots:
            q.set_trace_stats(buf.data_ptr(), buf.numel())
        try:
            self.r.frame()
            self.r.flush()
            torch.cuda.synchronize()
        finally:
            for q, _ in self.full.pt_slots:
                q.set_trace_stats(0)
        return dict(zip(self.r.STAT_KEYS, (int(v) for v in buf.cpu().tolist())))

    def profile(self, on: bool) -> None:
        self.r.profile(on)
        self.full.profile(on)

    band_ms = FrameShardRenderer.band_ms

    def pass_times(self) -> dict:
        out = self.r.pass_times()
        for k, v in self.full.pass_times().items():
            if k == "pathtrace":
                out["tiles_" + k] = v
        return out

    def close(self) -> None:
        from .renderer import release_stream

        super().close()
        self.full.close()
        self._full_tensors.clear()
        release_stream(self._recv_stream)
        self._recv_stream = None


class P2PRecorder:
    """A torch.distributed stand-in that forwards everything and logs each batch_isend_irecv call: (site, group, frame,
    ops) with ops = [(kind, peer, bytes)] in issue order. site = the function that issued the batch (halo_exchange,
    exchange_window, exchange_tiles), group = "world" / "scatter" / "host" / "group", frame = frame_of() at the call
    (the frame the host is issuing). check_p2p_logs compares the ranks' logs: what RCCL needs of point-to-point
    traffic spread over two communicators (DESIGN.md "RCCL issue order")."""

    def __init__(self, dist, frame_of=None):
        self._dist = dist
        self.frame_of = frame_of or (lambda: -1)
        self.log = []

    def __getattr__(self, name):
        return getattr(self._dist, name)

    def _group_name(self, group) -> str:
        if group is None or group is self._dist.group.WORLD:
            return "world"
        if any(g is group for _, g in _SCATTER_GROUP.values()):
            return "scatter"
        if any(g is group for _, g in _HOST_GROUP.values()):
            return "host"
        return "group"

    def batch_isend_irecv(self, ops):
        import sys

        site = sys._getframe(1).f_code.co_name
        groups = {self._group_name(o.group) for o in ops}
        if len(groups) != 1:
            raise RuntimeError(f"a P2P batch spans several groups: {sorted(groups)}")
        rec = [("send" if getattr(o.op, "__name__", "") == "isend" else "recv", int(o.peer),
                int(o.tensor.numel() * o.tensor.element_size())) for o in ops]
        self.log.append((site, groups.pop(), int(self.frame_of()), rec))
        return self._dist.batch_isend_irecv(ops)


def check_p2p_logs(logs) -> list:
    """logs[r] = rank r's P2PRecorder.log. Returns the violations (empty: none) of the rule that keeps point-to-point
    traffic on several communicators deadlock-free and correctly paired whatever the streams overlap: for every pair of
    ranks (r, q), the batches in which r addresses q are, in issue order and over every group, the batches in which q
    addresses r — same call site, same group, and r's sends to q (in order, by bytes) are q's receives from r and vice
    versa. (Within one batch, one group call, sends and receives pair up in order among themselves: their interleaving
    does not matter.)"""
    bad = []
    n = len(logs)

    def batches(log, me, peer):
        out = []
        for site, g, _, ops in log:
            snd = tuple(nb for kind, p, nb in ops if p == peer and kind == "send")
            rcv = tuple(nb for kind, p, nb in ops if p == peer and kind == "recv")
            if snd or rcv:
                out.append((site, g, snd, rcv))
        return out

    for r in range(n):
        for q in range(r + 1, n):
            a = batches(logs[r], r, q)
            b = [(site, g, rcv, snd) for site, g, snd, rcv in batches(logs[q], q, r)]
            if a != b:
                i = next((i for i, (x, y) in enumerate(zip(a, b)) if x != y), min(len(a), len(b)))
                bad.append(f"ranks {r}<->{q}: batch {i} differs: {a[i] if i < len(a) else None} (rank {r}: site, group, "
                           f"sends, receives) vs {b[i] if i < len(b) else None} (rank {q}, as seen from {r}); "
                           f"{len(a)} vs {len(b)} batches")
    return bad


def gather_bands(owned: dict, plan: BandPlan, dist, dst: int = 0) -> dict | None:
    """Assemble full frames on rank `dst` from every rank's owned rows: owned maps plane names to (y1 - y0, W, C)
    float32 numpy arrays; returns {name: (H, W, C)} on dst, None elsewhere. Point-to-point sends of device tensors
    (RCCL over xGMI) or host tensors (gloo); for checking and dumps, outside any timed region."""
    import numpy as np
    import torch

    dev = torch.device("cuda", torch.cuda.current_device()) if dist.get_backend() != "gloo" else torch.device("cpu")
    names = sorted(owned)
    if plan.rank != dst:
        for k in names:
            dist.send(torch.from_numpy(np.ascontiguousarray(owned[k])).to(dev), dst)
        return None
    full = {}
    for k in names:
        a = owned[k]
        out = np.empty((plan.H,) + a.shape[1:], a.dtype)
        out[plan.y0:plan.y1] = a
        full[k] = out
    for src in range(plan.world):
        if src == dst:
            continue
        y0, y1 = plan.owned(src)
        for k in names:
            t = torch.empty((y1 - y0,) + full[k].shape[1:], dtype=torch.float32, device=dev)
            dist.recv(t, src)
            full[k][y0:y1] = t.cpu().numpy()
    return full


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


def agree_bounds(bounds, dist, group=None) -> tuple:
    """Rank 0's band bounds on every rank. A calibration must end in ONE plan: ranks that cut their bands differently
    each still trace their own rows right, but exchange halo rows for bands their peers do not hold, so the SVGF
    chain silently leaves the one-GPU frame (seen once with the every-pass bands, whose calibration all-reduced
    device tensors over gloo). Collective over `group` (the host group: a CPU tensor)."""
    import torch

    t = torch.tensor([int(b) for b in bounds], dtype=torch.int64)
    dist.broadcast(t, src=0, group=group)
    return tuple(int(v) for v in t.tolist())


def make_frame_shard_renderer(scene, W, H, cfg, rank, world, dist, balance: bool = True, rounds: int = 2, cls=None,
                              **kw):
    """FrameShardRenderer whose bands equalise the band work (G-buffer + SVGF chain: the plant's rows cost several
    times a sky row; every rank's whole-frame path tracer is the same). Each round measures every rank's band work
    (band_ms), spreads it evenly over the band's rows and cuts new bands at equal quantiles of the mean of the rounds'
    per-row estimates; the measured plan with the smallest slowest band wins and the renderer is rebuilt on it
    (calibration frames are discarded). Every rank derives the same bounds from all-reduced times. cls: the renderer
    (FrameShardRenderer, or TileShardRenderer, whose path tracer is the same share of every frame on every rank)."""
    import numpy as np
    import torch

    cls = cls or FrameShardRenderer
    r = cls(scene, W, H, cfg, rank, world, dist, **kw)
    if not balance or world == 1:
        return r
    est, tried = [], []
    for i in range(max(rounds, 1) + 1):
        t = torch.zeros(world, dtype=torch.float64)
        t[rank] = r.band_ms()
        dist.all_reduce(t, group=r._group)  # host values: the gloo group (the default group under gloo)
        times = t.numpy()
        tried.append((float(times.max()), r.plan.bounds))
        if i == max(rounds, 1):
            break
        b = r.plan.bounds
        cost = np.empty(H)
        for k in range(world):
            cost[b[k]:b[k + 1]] = times[k] / (b[k + 1] - b[k])
        est.append(cost)
        bounds = agree_bounds(balanced_bounds(np.mean(est, axis=0), world), dist, r._group)
        r.close()
        r = cls(scene, W, H, cfg, rank, world, dist, bounds=bounds, **kw)
    best = agree_bounds(min(tried, key=lambda x: x[0])[1], dist, r._group)
    r.close()
    r = cls(scene, W, H, cfg, rank, world, dist, bounds=best, **kw)
    r.calibration = tried  # (slowest band's work ms per frame, bounds) per measured plan
    return r


def make_band_renderer(scene, W, H, cfg, rank, world, dist, balance: bool = True, rounds: int = 3, **kw):
    """BandRenderer whose band heights equalise the measured per-row cost (sky rows are cheap, the plant
    and clock rows expensive). Each calibration round renders on the current bands, measures every rank's
    band time and visits (measure_row_cost) and cuts new bands at equal quantiles of the mean of all rounds'
    per-row cost estimates. A band's time is not additive in its rows (a band holding the plant's longest rays
    has a latency floor set by their walks) and single timings are noisy, so the last cut is measured too and the
    plan with the smallest measured slowest band wins; the renderer is rebuilt on it. Every rank derives the same
    bounds from all-reduced data."""
    import numpy as np

    r = BandRenderer(scene, W, H, cfg, rank, world, dist, **kw)
    if not balance or world == 1:
        return r
    est, tried = [], []
    for i in range(max(rounds, 1) + 1):
        r.frame()
        cost = r.measure_row_cost()
        tried.append((float(np.max(r.last_band_ms)), r.plan.bounds))
        if i == max(rounds, 1):
            break
        est.append(cost)
        bounds = agree_bounds(balanced_bounds(np.mean(est, axis=0), world), dist, r._group)
        r.close()
        r = BandRenderer(scene, W, H, cfg, rank, world, dist, bounds=bounds, **kw)
    best = agree_bounds(min(tried, key=lambda x: x[0])[1], dist, r._group)
    r.close()  # calibration frames are discarded: the renderer starts fresh (frame 0, empty history)
    r = BandRenderer(scene, W, H, cfg, rank, world, dist, bounds=best, **kw)
    r.calibration = tried  # (slowest band ms, bounds) per measured plan
    return r
