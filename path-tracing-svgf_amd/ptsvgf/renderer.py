"""Headless ``main.cpp``: the reference's startup (main.cpp:65-338) and frame
loop (main.cpp:436-602) driven through the drop-in C ABI.

Two drivers over the same kernels:

* :class:`Renderer` (``mode="reference"``) issues the reference's exact call
  sequence — every pass, every ping-pong ``bilt`` copy, the iteration-1 history
  copy and the 5-target ``save_frame_data`` copy (main.cpp:499-553). This is
  what a C++ ``main.cpp`` linked against libptsvgf.so does.
* ``mode="fast"`` keeps the identical math but replaces the copies with
  double-buffered targets (pointer swaps, SURVEY.md §2 "build replaces with
  pointer swaps"): same outputs bit for bit (tests/test_gpu_frame.py), fewer
  HBM bytes per frame. This is the benchmarked path.

TAA and the output tonemap run in both modes (main.cpp:537-590).
"""
from __future__ import annotations

import os
import time

import numpy as np

from . import gl
from .camera import Camera, mat_mul, parameter_config, rigid_inverse
from .gl import GL_TEXTURE_2D, GL_TEXTURE_2D_ARRAY, GL_TEXTURE_BUFFER, RenderPass, Rasterize_RenderPass, getShaderProgram, getTextureRGB32F
from .scene import Scene

SHADERS = "./shaders/"
VISIT_BUDGET = 256  # node + triangle visits before a ray goes to the wave-cooperative walk (_ensure_slots)


def _prog(frag: str, vert: str = "vert.vert") -> int:
    return getShaderProgram(SHADERS + frag, SHADERS + vert)


class PassGroup:
    """Several passes of one program driven as one: a call applies to each (returns the first result)."""

    def __init__(self, passes):
        self.passes = list(passes)

    def __getattr__(self, name):
        fns = [getattr(p, name) for p in self.passes]

        def call(*a, **k):
            return [f(*a, **k) for f in fns][0]

        return call


def _set_stream(stream) -> None:
    from ._lib import check, pt

    check(pt().pt_set_stream(stream.cuda_stream))


_FREE_STREAMS: dict = {}  # (device, priority) -> streams a closed renderer gave back


def acquire_stream(priority: int = 0):
    """A stream no live renderer holds. torch.cuda.Stream() hands out its fixed per-priority pool (32 streams)
    round-robin, so after 32 of them two live objects share one queue: a renderer's streams, or a renderer's and a
    process group's communication stream (taken from the same pool). Recycling what closed renderers held keeps
    the allocations far below the pool's size over a run of many renderers (bench calibration, several views)."""
    import torch

    key = (torch.cuda.current_device(), priority)
    pool = _FREE_STREAMS.setdefault(key, [])
    if pool:
        return pool.pop()
    stream = torch.cuda.Stream(priority=priority)
    stream._ptsvgf_key = key  # the bucket it returns to (the priority torch reports may be clamped)
    return stream


def release_stream(stream) -> None:
    """Give a stream back to the pool; the library first drops what it holds for it (pt_stream_release: the
    trace_fork side stream, merged-environment reader events), so the next holder starts afresh."""
    from ._lib import check, pt

    key = getattr(stream, "_ptsvgf_key", None)
    if key is None:
        return  # not from the pool
    handle = getattr(stream, "cuda_stream", None)
    if handle is not None:
        rc = pt().pt_stream_release(handle)
        if rc != -9:  # PT_ERR_STATE: the library was never initialised, so it holds nothing for the stream
            check(rc)
    _FREE_STREAMS.setdefault(key, []).append(stream)


def reserved_cus(ncu: int, reserve: int, xcds: int = 8) -> list:
    """`reserve` CU indices spread evenly over the XCDs whether the CU mask numbers CUs XCD by XCD (XCD = i // (ncu /
    xcds)) or round-robin (XCD = i % xcds): the j-th reserved CU sits in block j % xcds at residue j % xcds."""
    per = ncu // xcds
    out = []
    for j in range(reserve):
        b, k = j % xcds, j // xcds
        out.append(b * per + (b + xcds * k) % per)
    return sorted(set(out))


def masked_stream(exclude: list):
    """A stream whose kernels never run on the CUs in `exclude` (pt_stream_create_cu_masked), as a torch external
    stream; returns (stream, raw handle) — destroy the handle with pt_stream_destroy after the last use."""
    import ctypes as C

    import torch

    from ._lib import check, pt

    n = C.c_int()
    check(pt().pt_device_cus(C.byref(n)))
    words = (n.value + 31) // 32
    mask = (C.c_uint32 * words)(*([0xFFFFFFFF] * words))
    for i in range(n.value, words * 32):
        mask[i // 32] &= ~(1 << (i % 32)) & 0xFFFFFFFF
    for i in exclude:
        mask[i // 32] &= ~(1 << (i % 32)) & 0xFFFFFFFF
    h = C.c_void_p()
    check(pt().pt_stream_create_cu_masked(words, mask, C.byref(h)))
    return torch.cuda.ExternalStream(h.value), h.value


def priority_stream(priority: int):
    """A stream at HIP queue priority `priority` (pt_stream_create_priority: lower = higher; torch's pool stops at
    0 and -1, this reaches HIP's low priority too), as a torch external stream; returns (stream, raw handle) — destroy
    the handle with pt_stream_destroy after the last use."""
    import ctypes as C

    import torch

    from ._lib import check, pt

    h = C.c_void_p()
    check(pt().pt_stream_create_priority(int(priority), C.byref(h)))
    return torch.cuda.ExternalStream(h.value), h.value


class Renderer:
    def __init__(self, scene: Scene, width: int, height: int, config: parameter_config | None = None,
                 mode: str = "fast", aspect_corrected: bool | None = None, band=None, prune: bool = True,
                 atrous_exact: bool = False, run_taa: bool = True, run_output: bool = True, tex_factory=None,
                 halo=None, gbuffer_rows=None, frames_in_flight: int = 1, after_gbuffer=None, back_lag: int = 0,
                 trace_batch: int = 1, front_streams: int | None = None, pt_source=None, pt_flush=None,
                 stage_rows=None, early_history=None, draw_gbuffer: bool = True, fuse_modulate: bool = True,
                 host_pace: bool = False):
        """band = (y0, y1, row0, rows) for screen-band sharding; tex_factory(w, h) -> handle allocates the
        frame-sized planes (ptsvgf.dist wraps torch tensors); halo(stage, {plane name: handle}) is called before
        the SVGF passes that read rows beyond the band (dist.HALO_SCHEDULE names the planes); after_gbuffer(set,
        torch stream) right after a G-buffer draw is issued; gbuffer_rows = (y0, y1) rows the G-buffer computes
        (default: the band).

        frames_in_flight = K > 1 (fast driver): the G-buffer + path tracer of frame f (the front end, which
        depends on nothing but the camera) run on stream f % K while the SVGF chain (sequential: each frame
        reads the previous frame's history) runs on one back-end stream. Frame f's front end waits only for
        the SVGF of frame f-K, whose buffers it reuses. The front end's launches end in long tails (a few
        rays through dense geometry); with K frames in flight another frame's work fills them. Same
        kernels, same inputs, same bits as K = 1 (tests/test_gpu_parity.py); throughput rises, latency
        from camera to finished frame is up to K frames.

        back_lag = D (0 <= D < K, frames in flight only): frame() issues the front end of frame f and the SVGF
        back end of frame f - D, so a host wait before a back-end pass (the band renderer's motion bound, read
        from the G-buffer before the reprojection exchange is sized) finds a G-buffer issued D frames earlier
        instead of stalling the issue of the next front end. planes() and time_atrous() first issue the back
        ends still pending (flush); results are those of D = 0.

        trace_batch = B (2..8, at most K, frames in flight only): the path tracer of B consecutive frames runs as
        one batched draw (pt_pass_draw_batch) issued with the last of them — its list-driven traversal launches
        trace all B frames' rays at once, so a thin band's launches carry B times the rays. The back lag is raised
        to at least B - 1 (a frame's back end needs its batch). Same bits.

        front_streams = S (frames in flight only, default K): the front ends of frame f run on stream f % S (the K
        frame slots are unchanged). pt_source(f, slot, stream) (fast driver, frames in flight): instead of drawing
        the path tracer, fill frame f's colour / emission / albedo planes of `slot` from elsewhere
        (dist.FrameShardRenderer: some rank traced the whole frame) once the slot is free; it is called right after the
        G-buffer of f is issued on `stream` and returns a holder dict whose "ev" (a torch event, set by the time the
        back end of f is issued) the back end waits for; pt_flush() is called by flush() before the pending back
        ends are issued.

        host_pace (frames in flight only): before issuing frame f's front end the host waits for the back end of
        frame f - K, which that front end waits for on the GPU anyway. Without it the host queues frames as fast as it
        can issue them and each frame's camera reaches the GPU long before its G-buffer runs (camera-to-modulate ≈ 8
        frames at K = 4); with it at most K frames are queued."""
        if mode not in ("fast", "reference"):
            raise ValueError(mode)
        self.mode = mode
        self.W, self.H = int(width), int(height)
        self.cfg = config or parameter_config()
        self.camera = Camera(self.W, self.H)
        self.aspect_corrected = (self.W != self.H) if aspect_corrected is None else bool(aspect_corrected)
        self.prune = prune
        self.atrous_exact = atrous_exact
        self.run_taa = run_taa
        self.run_output = run_output
        self.scene = scene
        self._after_gbuffer = after_gbuffer
        self._lib_stream = None  # torch stream the library draws on (None: torch's current stream)
        if band is not None:
            y0, y1, row0, rows = band
            gl.set_band(self.W, self.H, y0, y1, row0, rows)
        self.band = band
        self._halo_cb = halo
        W, H = self.W, self.H
        self._owned: list[int] = []   # every texture this renderer created (close() destroys them)
        make = tex_factory or getTextureRGB32F

        def tex(w, h):
            t = make(w, h)
            self._owned.append(t)
            return t

        self._tex = tex

        # scene buffers (main.cpp:136-181)
        self.trianglesTextureBuffer = gl.texture_buffer(scene.tri_enc)
        self.nodesTextureBuffer = gl.texture_buffer(scene.node_enc)
        self.pointLightBuffer = gl.texture_buffer(scene.lights)
        hh, hw, _ = scene.hdr.shape
        self.hdrMap = getTextureRGB32F(hw, hh)
        gl.upload_rgb32f(self.hdrMap, scene.hdr)
        self.hdrCache = getTextureRGB32F(hw, hh)
        gl.upload_rgb32f(self.hdrCache, scene.cache)
        self._owned += [self.trianglesTextureBuffer, self.nodesTextureBuffer, self.pointLightBuffer, self.hdrMap,
                        self.hdrCache]
        self.materials_array = None                            # main.cpp:184-205
        if getattr(scene, "textures", None) is not None:
            self.materials_array = gl.texture_array(scene.textures)
            self._owned.append(self.materials_array)
        self.hdrResolution = hw

        self.K = int(frames_in_flight)
        if self.K < 1 or (self.K > 1 and mode != "fast"):
            raise ValueError("frames_in_flight must be >= 1, and > 1 only with the fast driver")
        self.B = int(trace_batch)
        if not 1 <= self.B <= min(self.K, 8) or (self.B > 1 and mode != "fast"):
            raise ValueError(f"trace_batch must be in [1, min(frames_in_flight, 8)] (fast driver), got {trace_batch}")
        self.lag = max(int(back_lag), self.B - 1)
        self.host_pace = bool(host_pace) and self.K > 1
        self.pace_wait_s = 0.0  # host time spent in host_pace's waits (diagnostics)
        if not 0 <= self.lag < self.K:
            raise ValueError(f"back_lag must be in [0, frames_in_flight) = [0, {self.K}), got {back_lag}")
        self._nfs = self.K if front_streams is None else int(front_streams)
        if not 1 <= self._nfs <= self.K:
            raise ValueError(f"front_streams must be in [1, frames_in_flight], got {front_streams}")
        if pt_source is not None and (mode != "fast" or self.K < 2 or self.B > 1):
            raise ValueError("pt_source needs the fast driver with frames in flight and no trace batching")
        self._pt_source = pt_source
        self._pt_flush = pt_flush
        self._stage_rows = stage_rows
        self._draw_gbuffer = bool(draw_gbuffer)
        if not draw_gbuffer and pt_source is None:
            raise ValueError("draw_gbuffer=False needs a pt_source that provides the G-buffer planes")
        self._early_history = early_history
        # fast driver: the last a-trous iteration also writes the modulated colour (svgf_modulate.frag) from its
        # epilogue, saving the modulate pass's launch and its re-read of the a-trous output and normal/depth
        # (same arithmetic, same bits: tests/test_gpu_parity.py::test_fused_modulate_equals_modulate_pass)
        self.fuse_modulate = bool(fuse_modulate) and mode == "fast"
        self._ready = None  # pt_source's event for the front end being issued
        self._batch: list = []  # path-tracing passes of the open batch: (pass, G-buffer-done event, stream, holder)
        self._pending: list = []  # front ends whose back end is not issued yet (back_lag)
        # a serial renderer draws on torch's stream of its construction, whatever stream another renderer in the
        # process left the library on (the library's stream is process-global, pt_set_stream)
        self._serial_stream = None
        if self.K == 1:
            import torch

            self._serial_stream = torch.cuda.current_stream()
        self.back_set = 0         # G-buffer set of the back end being issued (halo / after_gbuffer users)
        # G-buffer sets: the reference has one; fast mode alternates two (this frame / previous frame);
        # with K frames in flight, frame f writes set f % (K+1) once SVGF(f-K) has read it (as "previous")
        nbuf = (self.K + 1 if self.K > 1 else 2) if mode == "fast" else 1
        # G-buffer (main.cpp:208-226); fast mode double-buffers it (prev normal/depth = other parity)
        self.init_pass = []
        self.gbuf = []
        raster_prog = _prog("rasterize_frag.frag", "rasterize_vert.vert")
        for b in range(nbuf):
            g = dict(world=tex(W, H), normal_depth=tex(W, H), velocity=tex(W, H), fwidth=tex(W, H))
            p = Rasterize_RenderPass(raster_prog, W, H)
            p.colorAttachments += [g["world"], g["normal_depth"], g["velocity"], g["fwidth"]]
            p.bindData(scene.raster)
            p.set_uniform_int("screen_width", W)
            p.set_uniform_int("screen_height", H)
            if gbuffer_rows is not None:
                p.set_rows(*gbuffer_rows)
            self.init_pass.append(p)
            self.gbuf.append(g)

        # path tracer (main.cpp:229-248)
        # (one pass + output set per frame in flight: each owns its wavefront state)
        # accumulate mode (path_tracing.frag:1116-1119) reads the previous frame's colour: the fast driver keeps
        # at least two slots so lastFrame is the other slot's colour output (the reference copies it,
        # save_frame_data.frag), and with frames in flight each front end then waits for the previous one
        self.accumulate = bool(self.cfg.accumulate_color)
        nslots = max(self.K, 2) if (self.accumulate and mode == "fast") else self.K
        self.pt_slots = []
        self._pt_prune = prune
        self._ensure_slots(nslots)
        self._use_slot(0)
        self._streams = None
        if self.K > 1:
            import torch  # streams and events are torch plumbing (the kernels are the library's)

            self._streams = [acquire_stream() for _ in range(self._nfs)]
            # the SVGF back end is a chain of short launches (and, on bands, exchanges) beside the front ends' long
            # traversal launches: on a high-priority queue its kernels take CUs as soon as waves retire instead of
            # queueing behind resident traversal waves (PTSVGF_BACK_PRIORITY=0: normal priority, A/B)
            hi = os.environ.get("PTSVGF_BACK_PRIORITY", "1") != "0"
            self._back = acquire_stream(-1 if hi else 0)
            self._slot_free = [None] * self.K  # event: SVGF of the frame that last used the slot is done
            self._fe_prev = None

        # SVGF targets
        if mode == "reference":
            self._build_reference_passes()
        else:
            self._build_fast_passes()
        # output / tonemap (main.cpp:336-338); a readable target instead of the default framebuffer
        self.output_tex = tex(W, H)
        self.output_pass = RenderPass(_prog("output_pass.frag"), W, H)
        self.output_pass.colorAttachments.append(self.output_tex)
        self.output_pass.bindData(True)
        self.pre_viewproj = mat_mul(self.camera.cam_proj_mat, self.camera.cam_view_mat)  # main.h:48
        self.frame_index = 0
        self._profile = False
        self._times: dict = {}
        self.back_events = None  # [start, end] HIP events per back end when set to a list (frames in flight only)
        # (camera, modulate done) HIP events per frame when set to a list (frames in flight only): latency_ms()
        self.latency_events = None
        self._clock = None  # the stream camera-time events are recorded on (idle)
        if self.K > 1:
            # the planes were zero-filled on the stream current at their creation (the library's memset, a tex_factory's
            # torch.zeros) and frames draw on the renderer's own streams, which do not wait for that one: a first frame
            # could read (or be overwritten by) a late fill. Memory a closed renderer freed still holds its old values,
            # so this showed as a history differing from the one-GPU frame after band calibration.
            import torch

            torch.cuda.synchronize()

    # ------------------------------------------------------------ passes ---
    def _svgf_pass(self, frag: str, atts) -> RenderPass:
        p = RenderPass(_prog(frag), self.W, self.H)
        p.colorAttachments += list(atts)
        p.bindData(False)
        return p

    def _build_reference_passes(self):
        W, H, tex = self.W, self.H, self._tex
        self.tmp_atrous_result = tex(W, H)
        self.bilt_pass = self._svgf_pass("bilt.frag", [self.tmp_atrous_result])
        self.next_frame_color_input = tex(W, H)
        self.save_next_frame_pass = self._svgf_pass("bilt.frag", [self.next_frame_color_input])
        self.taa_output = tex(W, H)
        self.pass_taa = self._svgf_pass("taa.frag", [self.taa_output])
        self.pass_taa.set_uniform_int("screen_width", W)
        self.pass_taa.set_uniform_int("screen_height", H)
        self.curIllumination, self.curMomentHistory = tex(W, H), tex(W, H)
        self.reproject_pass = self._svgf_pass("svgf_reproject.frag", [self.curIllumination, self.curMomentHistory])
        self.variance_compute_illumination = tex(W, H)
        self.variance_compute_pass = self._svgf_pass("svgf_variance.frag", [self.variance_compute_illumination])
        self.atrous_output = tex(W, H)
        self.atrous_pass = self._svgf_pass("svgf_Atrous.frag", [self.atrous_output])
        self.modulate_color = tex(W, H)
        self.svgf_modulate_pass = self._svgf_pass("svgf_modulate.frag", [self.modulate_color])
        self.lastIllumination, self.last_normal_depth = tex(W, H), tex(W, H)
        self.last_Moments_HistoryLength, self.last_acc_color, self.last_taa_color = tex(W, H), tex(W, H), tex(W, H)
        self.next_frame_input = self._svgf_pass("save_frame_data.frag", [
            self.lastIllumination, self.last_normal_depth, self.last_Moments_HistoryLength, self.last_acc_color,
            self.last_taa_color])
        for p in (self.reproject_pass, self.variance_compute_pass, self.atrous_pass):
            p.set_uniform_float("inv_screen_width", 1.0 / W)
            p.set_uniform_float("inv_screen_height", 1.0 / H)

    def _build_fast_passes(self):
        W, H, tex = self.W, self.H, self._tex
        self.illum = tex(W, H)                                  # reproject out 0
        self.moments = [tex(W, H), tex(W, H)]                   # reproject out 1 (history, by parity)
        self.hist_illum = [tex(W, H), tex(W, H)]                # a-trous iteration 1 output (history)
        self.var_out = tex(W, H)
        self.ping, self.pong = tex(W, H), tex(W, H)
        self.modulate_color = tex(W, H)
        self.taa = [tex(W, H), tex(W, H)]
        self.reproject = [self._svgf_pass("svgf_reproject.frag", [self.illum, self.moments[b]]) for b in (0, 1)]
        self.variance_compute_pass = self._svgf_pass("svgf_variance.frag", [self.var_out])
        self.atrous_to = {"ping": self._svgf_pass("svgf_Atrous.frag", [self.ping]),
                          "pong": self._svgf_pass("svgf_Atrous.frag", [self.pong]),
                          "hist0": self._svgf_pass("svgf_Atrous.frag", [self.hist_illum[0]]),
                          "hist1": self._svgf_pass("svgf_Atrous.frag", [self.hist_illum[1]])}
        self.svgf_modulate_pass = self._svgf_pass("svgf_modulate.frag", [self.modulate_color])
        # the last iteration with the modulate fused (colour attachment 1, "fuse_modulate"), per destination
        self.atrous_mod_to = {k: self._svgf_pass("svgf_Atrous.frag", [self._atrous_tex(k), self.modulate_color])
                              for k in self.atrous_to}
        for p in self.atrous_mod_to.values():
            p.set_uniform_int("fuse_modulate", 1)
        self.pass_taa = [self._svgf_pass("taa.frag", [self.taa[b]]) for b in (0, 1)]
        for p in self.pass_taa:
            p.set_uniform_int("screen_width", W)
            p.set_uniform_int("screen_height", H)
        for p in self.reproject + [self.variance_compute_pass, *self.atrous_to.values(), *self.atrous_mod_to.values()]:
            p.set_uniform_float("inv_screen_width", 1.0 / W)
            p.set_uniform_float("inv_screen_height", 1.0 / H)

    # ------------------------------------------------------------- frame ---
    def _ensure_slots(self, n: int) -> None:
        """Path-tracing passes + colour/emission/albedo outputs, one per frame slot (main.cpp:229-248)."""
        W, H, scene = self.W, self.H, self.scene
        while len(self.pt_slots) < n:
            p = RenderPass(_prog("path_tracing.frag"), W, H)
            outs = (self._tex(W, H), self._tex(W, H), self._tex(W, H))  # color, emission, albedo
            p.colorAttachments += list(outs)
            p.bindData(False)
            p.set_uniform_int("nTriangles", scene.ntris)
            p.set_uniform_int("nNodes", scene.node_enc.shape[0])
            p.set_uniform_int("width", W)
            p.set_uniform_int("height", H)
            p.set_uniform_int("pointLightSize", scene.lights.shape[0])
            p.set_uniform_int("aspect_corrected", int(self.aspect_corrected))
            p.set_uniform_int("prune", int(self._pt_prune))
            # lane-refill traversal waves: +8 % frames/s with frames in flight, -6 % serial (kernels_wavefront.hip)
            # share of each bounce / shadow list traced by lane-refill waves (frames in flight only); with up to 12
            # chunk rounds per wave 75 / 85 / 90 / 95 % measured 183.1 / 184.3 / 183.7 / 183.9 fps at 4K and 57.2 / 58.7 /
            # 59.5 / 60.6 fps on the surface view, 1080p and 8 bands within noise (tools/refill_pct_sweep.sh)
            # (round 4, 8 waves per SIMD, 26 resident waves per CU: 100 % gave 4K 220.9 / 221.2 against 221.4 / 220.3 for
            # 90 and the surface view 74.4 / 74.2 against 71.3 / 72.1, profiles/r04/refill_pct_ab.log)
            # (round 5: also one frame at a time, now that the visit budgets below cut the refill waves' tails)
            p.set_uniform_int("trace_refill", 100)
            # one frame at a time: the bounce-0 shadow walk on a side stream beside the bounce-1 closest-hit walk
            # (their launch tails overlap): 4K serial 131.3 -> 145.4 fps, surface view 48.3 -> 49.3; with frames in
            # flight the other frames already fill those tails (215.7 / 215.6 fps at K = 4, profiles/r04/fork/)
            p.set_uniform_int("trace_fork", 1 if self.K == 1 else 0)
            # a ray still walking past VISIT_BUDGET node + triangle visits is finished by the wave-cooperative walk
            # (same bits): the launches no longer end on a few long walks. Round 5, same box (profiles/r05/serial/):
            # one frame at a time with lane refill 145.2 -> 160.8 fps at 4K (budgets 128 / 512: 151.3 / 151.8; refill
            # without budgets 146.6; without the fork 133.6); K = 4 219.8 / 220.7 -> 223.9 (512 / 1024: 222.1 / 220.0)
            p.set_uniform_int("shadow_budget", VISIT_BUDGET)
            p.set_uniform_int("closest_budget", VISIT_BUDGET)
            p.set_uniform_int("trace_batch", self.B)
            self.pt_slots.append((p, outs))
        self.pass_path_tracing = PassGroup([p for p, _ in self.pt_slots])  # settings apply to every slot

    VIEWS = ("path_tracing_pic_1spp", "svgf_reprojected_pic", "svgf_variance_pic", "svgf_atrous_pic",
             "svgf_modulate_pic", "taa_pic", "final_pic", "accumulate_color")  # gui_config.h:7-17

    def set_view(self, view: str) -> None:
        """The debug-view switch (main.cpp:398-415 radio buttons + gui_config.h:37-45): selects the plane the
        output pass shows (main.cpp:558-586); accumulate_color turns accumulation on, every other view off, and
        any change restarts the frame counter."""
        if view not in self.VIEWS:
            raise ValueError(f"unknown view {view!r}; one of {self.VIEWS}")
        self.view = view
        self.cfg.accumulate_color = view == "accumulate_color"
        self.accumulate = self.cfg.accumulate_color
        if self.accumulate and self.mode == "fast":
            self._ensure_slots(max(self.K, 2))
        self.camera.frameCounter = 0

    def _view_plane(self, f: int) -> int:
        v = getattr(self, "view", "final_pic")
        pl = self._planes_of(f)
        return {"path_tracing_pic_1spp": pl["color"], "accumulate_color": pl["color"],
                "svgf_reprojected_pic": pl["reproj_illum"], "svgf_variance_pic": pl["variance"],
                "svgf_atrous_pic": pl["atrous"], "svgf_modulate_pic": pl["modulate"],
                "taa_pic": pl["final"], "final_pic": pl["final"]}[v]

    def _use_slot(self, s: int) -> None:
        """Path-tracing pass and outputs of frame slot s (frame f uses slot f % K)."""
        self._slot = s
        self.pt_pass, (self.curColor, self.Emission, self.Albedo) = self.pt_slots[s]

    def _gbuffer_and_pt(self, b: int):
        self._gbuffer(b)
        if self._pt_source is not None:
            self._ready = self._pt_source(self.frame_index, self._slot, self._lib_stream)
            return
        self._path_trace(self.gbuf[b] if self.mode == "fast" else None)

    def _gbuffer(self, b: int):
        cam = self.camera
        view, proj = cam.cam_view_mat, cam.cam_proj_mat
        ip = self.init_pass[b]
        ip.set_uniform_mat4("view", view)                      # main.cpp:436-443
        ip.set_uniform_mat4("projection", proj)
        ip.set_uniform_mat4("pre_viewproj", self.pre_viewproj)
        ip.set_uniform_uint("frameCounter", cam.frameCounter)
        if not self._draw_gbuffer:  # its planes come with the path tracer's (pt_source)
            return
        self._draw(ip, "gbuffer")
        if self._after_gbuffer is not None:
            import torch

            self._after_gbuffer(b, self._lib_stream or torch.cuda.current_stream())

    def _path_trace(self, hint=None):
        """hint: this frame's G-buffer set (drawn before on the same stream); its world position and normal/depth
        planes bound the primary rays' walk (a result-preserving hint with no GL counterpart, kernels_wavefront.hip
        wf_primary). The reference driver binds none, as main.cpp."""
        cam, cfg = self.camera, self.cfg
        view = cam.cam_view_mat
        self.cameraRotate = rigid_inverse(view)                # main.cpp:445
        pt = self.pt_pass                                      # main.cpp:447-470
        pt.set_uniform_vec3("eye", cam.cam_position)
        pt.set_uniform_mat4("cameraRotate", self.cameraRotate)
        pt.set_uniform_uint("frameCounter", cam.frameCounter)
        pt.set_uniform_int("hdrResolution", self.hdrResolution)
        pt.set_uniform_bool("use_normal_map", cfg.use_normal_texture)
        pt.set_uniform_bool("accumulate", cfg.accumulate_color)
        pt.set_uniform_float("clamp_threshold", cfg.clamp_threshold)
        pt.set_uniform_int("max_tracing_depth", cfg.max_tracing_depth)
        pt.reset_texture_slot()
        pt.set_texture_uniform(GL_TEXTURE_BUFFER, self.trianglesTextureBuffer, "triangles")
        pt.set_texture_uniform(GL_TEXTURE_BUFFER, self.nodesTextureBuffer, "nodes")
        if cfg.accumulate_color:
            last_acc = (self.last_acc_color if self.mode == "reference"
                        else self.pt_slots[(self.frame_index - 1) % len(self.pt_slots)][1][0])
            pt.set_texture_uniform(GL_TEXTURE_2D, last_acc, "lastFrame")
        if self.materials_array is not None:
            pt.set_texture_uniform(GL_TEXTURE_2D_ARRAY, self.materials_array, "material_array")
        pt.set_texture_uniform(GL_TEXTURE_2D, self.hdrMap, "hdrMap")
        pt.set_texture_uniform(GL_TEXTURE_2D, self.hdrCache, "hdrCache")
        pt.set_texture_uniform(GL_TEXTURE_BUFFER, self.pointLightBuffer, "pointLights")
        if hint is not None:
            pt.set_texture_uniform(GL_TEXTURE_2D, hint["world"], "gWorldPos")
            pt.set_texture_uniform(GL_TEXTURE_2D, hint["normal_depth"], "gNormalAndLinearZ")
        if self._batching():
            return  # drawn with its batch (_front_fast)
        self._draw(pt, "pathtrace")

    def _batching(self) -> bool:
        return self.B > 1 and self.mode == "fast" and not self.cfg.accumulate_color

    def _issue_batch(self) -> None:
        """Draw the open batch's path tracers on the stream of its last frame, after all its G-buffers."""
        if not self._batch:
            return
        import torch

        stream = self._batch[-1][2]
        for _, ev, _, _ in self._batch:
            stream.wait_event(ev)
        self._stream_to(stream)
        passes = [p for p, _, _, _ in self._batch]
        gl.draw_batch(passes)
        if self._profile:
            self._times.setdefault("pathtrace", []).append(passes[0].last_ms())
        done = torch.cuda.Event()
        done.record(stream)
        for _, _, _, holder in self._batch:
            holder["ev"] = done
        self._batch = []

    def _frame_reference(self):
        cfg = self.cfg
        g = self.gbuf[0]
        self._gbuffer_and_pt(0)
        rp = self.reproject_pass                               # main.cpp:474-486
        rp.reset_texture_slot()
        rp.set_uniform_float("depth_threshold", cfg.reproj_depth_threshold)
        rp.set_uniform_float("normal_threshold", cfg.reproj_normal_threshold)
        rp.set_texture_uniform(GL_TEXTURE_2D, g["velocity"], "gMotion")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.curColor, "gColor")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.Albedo, "gAlbedo")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.Emission, "gEmission")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.lastIllumination, "gPrevIllum")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.last_Moments_HistoryLength, "gPrevMoments_HistoryLength")
        rp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.last_normal_depth, "gPrevNormalAndLinearZ")
        rp.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
        self._draw(rp, "reproject")
        vp = self.variance_compute_pass                        # main.cpp:488-495
        vp.reset_texture_slot()
        vp.set_uniform_float("gPhiColor", cfg.sigma_l)
        vp.set_uniform_float("gPhiNormal", cfg.sigma_n)
        vp.set_texture_uniform(GL_TEXTURE_2D, self.curIllumination, "gIllumination")
        vp.set_texture_uniform(GL_TEXTURE_2D, self.curMomentHistory, "gMoments_HistoryLength")
        vp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
        vp.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
        self._draw(vp, "variance")
        ap = self.atrous_pass                                  # main.cpp:499-526
        for i in range(cfg.num_atrous_iterations):
            ap.reset_texture_slot()
            ap.set_uniform_float("gPhiColor", cfg.sigma_l)
            ap.set_uniform_float("gPhiNormal", cfg.sigma_n)
            ap.set_uniform_int("gStepSize", 1 << i)
            ap.set_uniform_int("exact", int(self.atrous_exact))
            ap.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
            ap.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
            src = self.variance_compute_illumination if i == 0 else self.tmp_atrous_result
            ap.set_texture_uniform(GL_TEXTURE_2D, src, "gIllumination")
            self._draw(ap, "atrous")
            self.bilt_pass.reset_texture_slot()
            self.bilt_pass.set_texture_uniform(GL_TEXTURE_2D, self.atrous_output, "in_texture")
            self._draw(self.bilt_pass, "copy")
            if i == 1:
                self.save_next_frame_pass.reset_texture_slot()
                self.save_next_frame_pass.set_texture_uniform(GL_TEXTURE_2D, self.atrous_output, "in_texture")
                self._draw(self.save_next_frame_pass, "copy")
        mp = self.svgf_modulate_pass                           # main.cpp:530-535
        mp.reset_texture_slot()
        mp.set_texture_uniform(GL_TEXTURE_2D, self.Albedo, "gAlbedo")
        mp.set_texture_uniform(GL_TEXTURE_2D, self.Emission, "gEmission")
        mp.set_texture_uniform(GL_TEXTURE_2D, self.atrous_output, "gIllumination")
        mp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
        self._rows(mp, "modulate")
        self._draw(mp, "modulate")
        if self.run_taa:                                       # main.cpp:537-544
            tp = self.pass_taa
            tp.reset_texture_slot()
            tp.set_texture_uniform(GL_TEXTURE_2D, self.modulate_color, "currentColor")
            tp.set_texture_uniform(GL_TEXTURE_2D, self.last_taa_color, "previousColor")
            tp.set_texture_uniform(GL_TEXTURE_2D, g["velocity"], "velocityTexture")
            tp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "normal_depth")
            tp.set_uniform_uint("frameCounter", self.camera.frameCounter)
            self._draw(tp, "taa")
        nf = self.next_frame_input                             # main.cpp:546-553
        nf.reset_texture_slot()
        nf.set_texture_uniform(GL_TEXTURE_2D, self.next_frame_color_input, "texPass0")
        nf.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "texPass1")
        nf.set_texture_uniform(GL_TEXTURE_2D, self.curMomentHistory, "texPass2")
        nf.set_texture_uniform(GL_TEXTURE_2D, self.curColor, "accColor")
        nf.set_texture_uniform(GL_TEXTURE_2D, self.taa_output, "taaOutput")
        self._draw(nf, "copy")
        self.final = self.taa_output if self.run_taa else self.modulate_color

    def _front_fast(self) -> dict:
        """G-buffer + path tracer of frame f (the front end); returns what its back end needs."""
        f = self.frame_index
        ng = len(self.gbuf)
        s = f % len(self.pt_slots)
        self._use_slot(s)
        done = None
        t_cam = None
        if self.latency_events is not None and self.K > 1:
            # camera time: an event on a stream nothing else uses completes as soon as it is issued, so its timestamp is
            # the moment this frame's camera went to the GPU (a busy front-end stream would record it later)
            import torch

            if self._clock is None:
                self._clock = acquire_stream()
            t_cam = torch.cuda.Event(enable_timing=True)
            t_cam.record(self._clock)
        if self.K > 1:                                         # front end on stream s, after SVGF(f - K)
            import torch

            fe = self._streams[f % self._nfs]
            if self._slot_free[f % self.K] is not None:
                fe.wait_event(self._slot_free[f % self.K])
            if self.accumulate and self._fe_prev is not None:  # lastFrame = the previous front end's colour
                fe.wait_event(self._fe_prev)
            self._ready = None
            self._stream_to(fe)
            self._gbuffer_and_pt(f % ng)
            done = torch.cuda.Event()
            done.record(fe)
            self._fe_prev = done
            if self._batching():  # the path tracer waits for its batch; the back end for the batch's draw
                holder = {}
                self._batch.append((self.pt_pass, done, fe, holder))
                done = holder
                if len(self._batch) == self.B:
                    self._issue_batch()
        else:
            self._gbuffer_and_pt(f % ng)
        return dict(f=f, slot=s, done=done, ready=self._ready, frame_counter=self.camera.frameCounter, t_cam=t_cam)

    def _back_fast(self, ctx: dict):
        """The SVGF chain of the frame whose front end made ctx (back-end stream, sequential over frames)."""
        cfg = self.cfg
        f = ctx["f"]
        b = f & 1                                              # history parity (back end, sequential)
        pb = 1 - b
        ng = len(self.gbuf)
        g, gp = self.gbuf[f % ng], self.gbuf[(f - 1) % ng]
        _, (color, emission, albedo) = self.pt_slots[ctx["slot"]]
        self.back_set = f % ng
        if self.K > 1:
            done = ctx["done"]
            if isinstance(done, dict):  # batched path tracer: its batch must have been drawn
                if "ev" not in done:
                    self._issue_batch()
                done = done["ev"]
            self._back.wait_event(done)
            if ctx.get("ready") is not None:  # pt_source: the colour / emission / albedo planes have arrived
                if "ev" not in ctx["ready"]:
                    raise RuntimeError(f"pt_source has not delivered frame {f} by its back end (back_lag too small)")
                self._back.wait_event(ctx["ready"]["ev"])
            self._stream_to(self._back)
            if self.back_events is not None:  # diagnostics: when each frame's SVGF chain starts and ends on its stream
                import torch

                e0 = torch.cuda.Event(enable_timing=True)
                e0.record(self._back)
                self.back_events.append([e0, None])
        self._halo("reproject", {"prev_illum": self.hist_illum[pb], "prev_moments": self.moments[pb],
                                 "prev_nd": gp["normal_depth"]})
        rp = self.reproject[b]
        rp.reset_texture_slot()
        rp.set_uniform_float("depth_threshold", cfg.reproj_depth_threshold)
        rp.set_uniform_float("normal_threshold", cfg.reproj_normal_threshold)
        rp.set_texture_uniform(GL_TEXTURE_2D, g["velocity"], "gMotion")
        rp.set_texture_uniform(GL_TEXTURE_2D, color, "gColor")
        rp.set_texture_uniform(GL_TEXTURE_2D, albedo, "gAlbedo")
        rp.set_texture_uniform(GL_TEXTURE_2D, emission, "gEmission")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.hist_illum[pb], "gPrevIllum")
        rp.set_texture_uniform(GL_TEXTURE_2D, self.moments[pb], "gPrevMoments_HistoryLength")
        rp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
        rp.set_texture_uniform(GL_TEXTURE_2D, gp["normal_depth"], "gPrevNormalAndLinearZ")
        rp.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
        self._rows(rp, "reproject")
        self._draw(rp, "reproject")
        self._halo("variance", {"illum": self.illum, "moments": self.moments[b], "nd": g["normal_depth"]})
        vp = self.variance_compute_pass
        vp.reset_texture_slot()
        vp.set_uniform_float("gPhiColor", cfg.sigma_l)
        vp.set_uniform_float("gPhiNormal", cfg.sigma_n)
        vp.set_texture_uniform(GL_TEXTURE_2D, self.illum, "gIllumination")
        vp.set_texture_uniform(GL_TEXTURE_2D, self.moments[b], "gMoments_HistoryLength")
        vp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
        vp.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
        self._rows(vp, "variance")
        self._draw(vp, "variance")
        # a-trous chain without copies: i0 var->ping, i1 ping->hist[b] (next frame's history),
        # then alternate through ping/pong
        src = self.var_out
        hist_key = "hist0" if b == 0 else "hist1"
        dests = []
        n = cfg.num_atrous_iterations
        for i in range(n):
            if i == 1:
                dests.append(hist_key)
            else:
                prev_tex = None if not dests else self._atrous_tex(dests[-1])
                dests.append("pong" if prev_tex == self.ping else "ping")
        self._atrous_last = (g, [(dests[i], 1 << i) for i in range(n)], src)
        fused = self.fuse_modulate and n > 0
        for i in range(n):
            self._halo(f"atrous{i}", {"atrous_in": src})
            last = fused and i == n - 1
            ap = (self.atrous_mod_to if last else self.atrous_to)[dests[i]]
            ap.reset_texture_slot()
            if last:
                ap.set_texture_uniform(GL_TEXTURE_2D, albedo, "gAlbedo")
                ap.set_texture_uniform(GL_TEXTURE_2D, emission, "gEmission")
            ap.set_uniform_float("gPhiColor", cfg.sigma_l)
            ap.set_uniform_float("gPhiNormal", cfg.sigma_n)
            ap.set_uniform_int("gStepSize", 1 << i)
            ap.set_uniform_int("exact", int(self.atrous_exact))
            ap.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
            ap.set_texture_uniform(GL_TEXTURE_2D, g["fwidth"], "gNormalDepthFwidth")
            ap.set_texture_uniform(GL_TEXTURE_2D, src, "gIllumination")
            self._rows(ap, "atrous")
            self._draw(ap, "atrous_modulate" if last else "atrous")
            src = self._atrous_tex(dests[i])
            if i == 1 and self._early_history is not None:  # the next frame's history is written
                nxt = self._pending[0] if self._pending and self._pending[0]["f"] == f + 1 else None
                with self._on_back():
                    self._early_history({"prev_illum": self.hist_illum[b], "prev_moments": self.moments[b],
                                         "prev_nd": g["normal_depth"]}, None if nxt is None else (f + 1) % ng)
        self.atrous_final = src
        if not fused:
            mp = self.svgf_modulate_pass
            mp.reset_texture_slot()
            mp.set_texture_uniform(GL_TEXTURE_2D, albedo, "gAlbedo")
            mp.set_texture_uniform(GL_TEXTURE_2D, emission, "gEmission")
            mp.set_texture_uniform(GL_TEXTURE_2D, src, "gIllumination")
            mp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "gNormalAndLinearZ")
            self._rows(mp, "modulate")
            self._draw(mp, "modulate")
        if self.run_taa:
            self._halo("taa", {"modulate": self.modulate_color, "velocity": g["velocity"], "prev_taa": self.taa[pb]})
            tp = self.pass_taa[b]
            tp.reset_texture_slot()
            tp.set_texture_uniform(GL_TEXTURE_2D, self.modulate_color, "currentColor")
            tp.set_texture_uniform(GL_TEXTURE_2D, self.taa[pb], "previousColor")
            tp.set_texture_uniform(GL_TEXTURE_2D, g["velocity"], "velocityTexture")
            tp.set_texture_uniform(GL_TEXTURE_2D, g["normal_depth"], "normal_depth")
            tp.set_uniform_uint("frameCounter", ctx["frame_counter"])
            self._rows(tp, "taa")
            self._draw(tp, "taa")
        self.final = self.taa[b] if self.run_taa else self.modulate_color

    def _rows(self, p: RenderPass, stage: str) -> None:
        if self._stage_rows is not None:
            rows = self._stage_rows(stage)
            if rows is not None:
                p.set_rows(*rows)

    def time_atrous(self, reps: int = 20) -> float:
        """Average duration (ms) of one a-trous launch: the last frame's iterations (same inputs, so the
        replay rewrites the same bits) issued `reps` times back to back between two HIP events on the
        library's stream, kernels alone on the GPU (everything in flight is drained first). Fast driver."""
        import torch

        self.flush()
        g, iters, src0 = self._atrous_last
        stream = self._back if self.K > 1 else self._serial_stream
        torch.cuda.synchronize()
        self._stream_to(stream)
        e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)

        def once():
            src = src0
            for key, step in iters:
                ap = self.atrous_to[key]
                ap.set_uniform_int("gStepSize", step)
                ap.set_texture_uniform(GL_TEXTURE_2D, src, "gIllumination")
                ap.draw()
                src = self._atrous_tex(key)

        once()  # warm
        e0.record(stream)
        for _ in range(reps):
            once()
        e1.record(stream)
        e1.synchronize()
        return e0.elapsed_time(e1) / (reps * len(iters))

    STAT_KEYS = ("primary_rays", "primary_visits", "bounce_rays", "bounce_visits", "shadow_rays", "shadow_visits",
                 "tie_rewalks", "primary_retries", "spills", "primary_slots", "bounce_slots",
                 "shadow_slots", "shadow_point_rays", "shadow_occluded")  # pt_pass_set_trace_stats order (pt_device.h kStat*)

    def trace_stats(self) -> dict:
        """Render one frame with the path tracer's traversal counters on (pt_pass_set_trace_stats): rays traced and
        node + triangle visits per traversal kind. Synchronises; diagnostics, not for timed frames."""
        import torch

        buf = torch.zeros(len(self.STAT_KEYS), dtype=torch.int64, device="cuda")
        self.flush()  # frames already issued are not counted
        torch.cuda.synchronize()
        for p, _ in self.pt_slots:
            p.set_trace_stats(buf.data_ptr(), buf.numel())
        try:
            self.frame()
            self._issue_batch()  # this frame alone
            torch.cuda.synchronize()
        finally:
            for p, _ in self.pt_slots:
                p.set_trace_stats(0)
        return dict(zip(self.STAT_KEYS, (int(v) for v in buf.cpu().tolist())))

    def latency_ms(self) -> float | None:
        """Mean camera-to-modulate latency (ms) of the frames recorded since latency_events was set to a list: from
        the moment a frame's camera went to the GPU to the end of its SVGF chain (flushes and synchronises)."""
        import torch

        self.flush()
        torch.cuda.synchronize()
        ev = self.latency_events or []
        return sum(a.elapsed_time(b) for a, b in ev) / len(ev) if ev else None

    def _stream_to(self, stream) -> None:
        """Issue the following draws on this torch stream."""
        _set_stream(stream)
        self._lib_stream = stream

    def _on_back(self):
        """Context: torch's current stream = the back end's (exchanges issue on the current stream)."""
        import contextlib

        if self.K > 1:
            import torch

            return torch.cuda.stream(self._back)
        return contextlib.nullcontext()

    def _halo(self, stage: str, handles: dict) -> None:
        if self._halo_cb is None:
            return
        stages = getattr(self._halo_cb, "stages", None)  # the stages the callback acts on (None: all)
        if stages is not None and stage not in stages:
            return  # (a stream context per stage costs host time on every frame)
        with self._on_back():
            self._halo_cb(stage, handles)

    def _draw(self, p: RenderPass, name: str) -> None:
        p.draw()
        if self._profile:
            self._times.setdefault(name, []).append(p.last_ms())

    def profile(self, on: bool) -> None:
        """Time every draw with HIP events (synchronises after each draw: diagnostics only)."""
        gl.set_profiling(on)
        self._profile = on
        self._times = {}

    def pass_times(self) -> dict:
        """Per-pass ms of the profiled frames (sum per frame) + the a-trous per-launch average."""
        out = {k: float(np.sum(v)) for k, v in self._times.items()}
        if self._times.get("atrous"):
            out["atrous_avg_ms"] = float(np.mean(self._times["atrous"]))
        out["frame_sum_ms"] = float(sum(np.sum(v) for k, v in self._times.items()))
        return out

    def _atrous_tex(self, key: str) -> int:
        return {"ping": self.ping, "pong": self.pong, "hist0": self.hist_illum[0], "hist1": self.hist_illum[1]}[key]

    def frame(self) -> None:
        """One iteration of main.cpp's while-loop body (436-602), headless (with back_lag D: this frame's front
        end and frame f - D's back end)."""
        if self.host_pace and self._slot_free[self.frame_index % self.K] is not None:
            t0 = time.perf_counter()
            self._slot_free[self.frame_index % self.K].synchronize()  # before the camera is read (host_pace)
            self.pace_wait_s += time.perf_counter() - t0
        self.camera.update()
        if self._serial_stream is not None:
            self._stream_to(self._serial_stream)
        if self.mode == "reference":
            self._frame_reference()
            self._finish(None)
        else:
            self._pending.append(self._front_fast())
            while len(self._pending) > self.lag:
                self._finish(self._pending.pop(0))
        # main.cpp:599-600: pre_viewproj = projection * inverse(cameraRotate) = projection * view
        self.pre_viewproj = mat_mul(self.camera.cam_proj_mat, self.camera.cam_view_mat)
        self.camera.frameCounter += 1
        self.frame_index += 1

    def flush(self) -> None:
        """Issue the open path-tracing batch and the back ends still pending (back_lag)."""
        self._issue_batch()
        if self._pt_flush is not None:
            self._pt_flush()
        while self._pending:
            self._finish(self._pending.pop(0))

    def _finish(self, ctx) -> None:
        """Back end (fast driver) + output pass of one frame; then its frame slot is free for frame f + K."""
        f = self.frame_index if ctx is None else ctx["f"]
        if ctx is not None:
            self._back_fast(ctx)
        if self.run_output:                                    # main.cpp:556-590 (final view)
            op = self.output_pass
            op.reset_texture_slot()
            op.set_uniform_bool("accumulate", self.cfg.accumulate_color)
            op.set_texture_uniform(GL_TEXTURE_2D, self._view_plane(f), "texPass0")
            self._draw(op, "output")
        if self.K > 1:  # the slot's buffers are free again once this frame's back end has run
            import torch

            ev = torch.cuda.Event()
            ev.record(self._back)
            if self.back_events is not None and ctx is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(self._back)
                self.back_events[-1][1] = e1
            if self.latency_events is not None and ctx is not None and ctx.get("t_cam") is not None:
                e1 = torch.cuda.Event(enable_timing=True)
                e1.record(self._back)
                self.latency_events.append((ctx["t_cam"], e1))
            self._slot_free[f % self.K] = ev

    # --------------------------------------------------------- accessors ---
    def rebuild_bvh(self, tri_enc=None, raster=None, leaf_n: int = 3, ploc_radius: int = 32):
        """Dynamic scenes: rebuild the path tracer's BVH on the GPU (pt_bvh_build) into the scene
        buffers the passes are bound to. `tri_enc` (Triangle_encoded rows, any order; default: the scene's
        triangles) carries moved vertices; `raster` (the pre-BVH vertex list, obj_loader.h:143-160) moves the
        G-buffer's triangles with them; ploc_radius > 0 rebuilds the tree above the LBVH leaves by PLOC (0: the plain
        LBVH). Defaults: the fastest 4K walk measured (tools/dyn_sweep.py: leaves of <= 3, radius 32: 160 fps, against
        146 for 8 / 16 and 126 for the plain LBVH). Frames already issued finish first. Returns (nodes, device ms)."""
        if self._streams is not None:
            import torch

            self.flush()
            torch.cuda.synchronize()
        src = gl.texture_buffer(self.scene.tri_enc if tri_enc is None else np.asarray(tri_enc, np.float32))
        try:
            nodes, ms = gl.bvh_build(src, self.trianglesTextureBuffer, self.nodesTextureBuffer, leaf_n, ploc_radius)
        finally:
            gl.destroy_texture(src)
        for p, _ in self.pt_slots:
            p.set_uniform_int("nNodes", nodes)
        if raster is not None:
            # the G-buffer passes: trees built on the GPU from one device copy; a plain LBVH, since the tile-binned
            # rasteriser walks it only when a tile list overflows
            import torch

            v = torch.from_numpy(np.ascontiguousarray(raster, np.float32).reshape(-1)).cuda()
            torch.cuda.synchronize()
            self.init_pass[0].rebind_vertices_device(v.data_ptr(), v.numel(), 0)
            for p in self.init_pass[1:]:  # the other G-buffer sets draw the same triangles: one tree
                p.share_vertices(self.init_pass[0])
        return nodes, ms

    def close(self) -> None:
        """Release every pass and texture this renderer created (the GL objects main.cpp never frees)."""
        if self._streams is not None:
            import torch

            torch.cuda.synchronize()  # frames may still be in flight on the renderer's streams
            for st in self._streams + [self._back] + ([self._clock] if self._clock is not None else []):
                release_stream(st)
            self._streams = []
            self._back = None
            self._clock = None
        for v in list(vars(self).values()):
            if isinstance(v, PassGroup):
                continue  # its passes are the pt_slots' (destroyed below)
            for q in (v if isinstance(v, list) else list(v.values()) if isinstance(v, dict) else [v]):
                if isinstance(q, tuple):
                    q = q[0]  # pt_slots entries: (pass, outputs)
                if isinstance(q, RenderPass):
                    q.destroy()
        for t in self._owned:
            gl.destroy_texture(t)
        self._owned = []

    def planes(self) -> dict:
        """Handles of the last frame's per-pass outputs (for readback / tests); issues pending back ends first."""
        self.flush()
        return self._planes_of(self.frame_index - 1)

    def _planes_of(self, f: int) -> dict:
        if self.mode == "reference":
            g = self.gbuf[0]
            return dict(world=g["world"], normal_depth=g["normal_depth"], velocity=g["velocity"], fwidth=g["fwidth"],
                        color=self.curColor, emission=self.Emission, albedo=self.Albedo,
                        reproj_illum=self.curIllumination, reproj_moments=self.curMomentHistory,
                        variance=self.variance_compute_illumination, atrous=self.atrous_output,
                        history_illum=self.lastIllumination, modulate=self.modulate_color, final=self.final,
                        output=self.output_tex)
        b = f & 1
        g = self.gbuf[f % len(self.gbuf)]
        _, (color, emission, albedo) = self.pt_slots[f % len(self.pt_slots)]
        return dict(world=g["world"], normal_depth=g["normal_depth"], velocity=g["velocity"], fwidth=g["fwidth"],
                    color=color, emission=emission, albedo=albedo, reproj_illum=self.illum,
                    reproj_moments=self.moments[b], variance=self.var_out, atrous=self.atrous_final,
                    history_illum=self.hist_illum[b], modulate=self.modulate_color, final=self.final,
                    output=self.output_tex)
