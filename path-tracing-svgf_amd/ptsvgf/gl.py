"""Python mirror of the reference's GPU plumbing API (layer L2), over the C ABI.

Same names, argument meaning and call order as the reference's C++ classes, so
a port of ``main.cpp`` reads line for line:

==========================================  ===================================
reference (file:line)                       here
==========================================  ===================================
``getShaderProgram`` Utils/shader.h:21-67   :func:`getShaderProgram`
``getTextureRGB32F`` Utils/help_func.h:22   :func:`getTextureRGB32F`
``glTexBuffer(RGB32F)`` main.cpp:136-168    :func:`texture_buffer`
``glTexImage2D(RGB32F)`` main.cpp:173-180   :func:`upload_rgb32f`
``RenderPass`` Utils/render_pass.h:82-182   :class:`RenderPass`
``Rasterize_RenderPass`` render_pass.h:5-80 :class:`Rasterize_RenderPass`
==========================================  ===================================

Errors: where the reference ``exit(-1)``s (missing shader, shader.h:8-12) or
prints (incomplete FBO, render_pass.h:58-59) this raises :class:`PtError`.
Unknown uniform names are ignored, as GL ignores location -1.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from ._lib import (PT_RGB32F, PT_RGBA32F, PT_TEXTURE_2D, PT_TEXTURE_2D_ARRAY, PT_TEXTURE_BUFFER, check, fptr,
                   pt)

GL_TEXTURE_2D = PT_TEXTURE_2D
GL_TEXTURE_BUFFER = PT_TEXTURE_BUFFER
GL_TEXTURE_2D_ARRAY = PT_TEXTURE_2D_ARRAY
GL_RGB32F = PT_RGB32F
GL_RGBA32F = PT_RGBA32F

SCR_WIDTH = 800   # Utils/camera.h:5-6
SCR_HEIGHT = 800


def init(device: int = 0) -> None:
    check(pt().pt_init(device))


def shutdown() -> None:
    check(pt().pt_shutdown())


def sync() -> None:
    check(pt().pt_sync())


def set_band(frame_w: int, frame_h: int, y0: int, y1: int, row0: int, rows: int) -> None:
    check(pt().pt_set_band(frame_w, frame_h, y0, y1, row0, rows))


def set_profiling(on: bool) -> None:
    check(pt().pt_set_profiling(1 if on else 0))


def getShaderProgram(fshader: str, vshader: str) -> int:
    h = C.c_uint32()
    check(pt().pt_program_create(fshader.encode(), vshader.encode(), C.byref(h)))
    return h.value


def getTextureRGB32F(width: int, height: int) -> int:
    h = C.c_uint32()
    check(pt().pt_texture2d_create(width, height, C.byref(h)))
    return h.value


def wrap_device_texture(ptr: int, width: int, height: int) -> int:
    h = C.c_uint32()
    check(pt().pt_texture2d_wrap(C.c_void_p(ptr), width, height, C.byref(h)))
    return h.value


def upload_rgb32f(tex: int, data: np.ndarray) -> None:
    """glTexImage2D(GL_TEXTURE_2D, 0, GL_RGB32F|GL_RGBA32F, w, h, ...) of a full image (h, w, 3|4)."""
    a = np.ascontiguousarray(data, dtype=np.float32)
    h, w, ch = a.shape
    check(pt().pt_texture2d_upload(tex, w, h, PT_RGB32F if ch == 3 else PT_RGBA32F, fptr(a)))


def texture_buffer(data: np.ndarray) -> int:
    """glGenBuffers + glBufferData + glTexBuffer(GL_TEXTURE_BUFFER, GL_RGB32F, ...)."""
    a = np.ascontiguousarray(data, dtype=np.float32)
    h = C.c_uint32()
    check(pt().pt_texbuffer_create(a.ctypes.data_as(C.c_void_p), a.nbytes, PT_RGB32F, C.byref(h)))
    return h.value


def buffer_readback(tex: int) -> np.ndarray:
    """Device contents of a texture buffer as flat float32 (3 floats per RGB32F texel)."""
    w, _, _ = texture_info(tex)
    out = np.empty(w * 3, np.float32)
    check(pt().pt_texture_readback(tex, fptr(out), out.nbytes))
    return out


def bvh_build(tri_in: int, tri_out: int, node_out: int, leaf_n: int = 8, ploc_radius: int = 0):
    """pt_bvh_build: GPU LBVH over the device triangles of tri_in (Triangle_encoded texels) into tri_out (leaf
    order) and node_out (BVHNode_encoded, dummy node 0, root 1) — the reference's buffer formats (main.cpp:88-151);
    ploc_radius > 0 rebuilds the tree above the LBVH leaves by PLOC. Returns (node count, device build ms)."""
    n, ms = C.c_int(), C.c_float()
    check(pt().pt_bvh_build(tri_in, leaf_n, ploc_radius, tri_out, node_out, C.byref(n), C.byref(ms)))
    return n.value, ms.value


class PtTileSeg(C.Structure):
    _fields_ = [("y_begin", C.c_int), ("y_end", C.c_int), ("offset", C.c_int), ("packed", C.c_void_p)]


def tiles_count(frame_w: int, stride: int, offset: int, y0: int, y1: int, tile_y0: int = 0) -> int:
    """Pixels per texture of the tile subset k * stride + offset in rows [y0, y1) (pt_tiles_count)."""
    n = C.c_int64()
    check(pt().pt_tiles_count(frame_w, tile_y0, stride, offset, y0, y1, C.byref(n)))
    return n.value


def tiles_copy(textures, stride: int, segs, unpack: bool, tile_y0: int = 0) -> None:
    """pt_tiles_copy: segs = [(y0, y1, offset, packed device pointer)]; one launch on the library stream."""
    tex = (C.c_uint32 * len(textures))(*textures)
    arr = (PtTileSeg * max(1, len(segs)))(*[PtTileSeg(a, b, o, C.c_void_p(p)) for a, b, o, p in segs])
    check(pt().pt_tiles_copy(tex, len(textures), tile_y0, stride, C.cast(arr, C.c_void_p), len(segs), int(bool(unpack))))


def texture_array(layers: np.ndarray) -> int:
    """main.cpp:184-205: glTexStorage3D(GL_TEXTURE_2D_ARRAY, 1, GL_RGBA8, w, h, n) + one glTexSubImage3D per layer
    (help_func.h:4-20). `layers` is (n, h, w, 3|4) uint8, rows already in GL order (stbi flipped on load)."""
    a = np.ascontiguousarray(layers, dtype=np.uint8)
    n, hh, ww, ch = a.shape
    h = C.c_uint32()
    check(pt().pt_texarray_create(ww, hh, n, C.byref(h)))
    for i in range(n):
        check(pt().pt_texarray_upload_layer(h.value, i, ww, hh, ch, a[i].ctypes.data_as(C.POINTER(C.c_uint8))))
    return h.value


def texture_info(tex: int):
    w, h, r0 = C.c_int(), C.c_int(), C.c_int()
    check(pt().pt_texture_info(tex, C.byref(w), C.byref(h), C.byref(r0)))
    return w.value, h.value, r0.value


def draw_batch(passes) -> None:
    """pt_pass_draw_batch: the frames of up to 8 path-tracing passes in one run, their traversals batched."""
    hs = (C.c_uint32 * len(passes))(*[p._handle() for p in passes])
    check(pt().pt_pass_draw_batch(hs, len(passes)))


def readback(tex: int) -> np.ndarray:
    """Stored rows of an RGBA32F texture as (rows, W, 4) float32."""
    w, rows, _ = texture_info(tex)
    out = np.empty((rows, w, 4), np.float32)
    check(pt().pt_texture_readback(tex, fptr(out), out.nbytes))
    return out


def upload_rgba(tex: int, data: np.ndarray) -> None:
    a = np.ascontiguousarray(data, dtype=np.float32)
    check(pt().pt_texture_upload_rgba(tex, fptr(a), a.nbytes))


def device_ptr(tex: int) -> int:
    p = C.c_void_p()
    check(pt().pt_texture_device_ptr(tex, C.byref(p)))
    return p.value or 0


def destroy_texture(tex: int) -> None:
    check(pt().pt_texture_destroy(tex))


class RenderPass:
    """Utils/render_pass.h:82-182 — a full-screen pass drawing into MRT attachments."""

    def __init__(self, program: int = 0, width: int = SCR_WIDTH, height: int = SCR_HEIGHT):
        self.program = program
        self.colorAttachments: list[int] = []
        self.width = width
        self.height = height
        self.texture_slot = 0
        self._h = None

    def _handle(self) -> int:
        if self._h is None:
            h = C.c_uint32()
            check(pt().pt_pass_create(self.program, self.width, self.height, C.byref(h)))
            self._h = h.value
        return self._h

    def bindData(self, finalPass: bool = False) -> None:
        h = self._handle()
        for t in self.colorAttachments:
            check(pt().pt_pass_add_color_attachment(h, t))
        check(pt().pt_pass_bind(h, 1 if finalPass else 0))

    def draw(self, texPassArray=()) -> None:
        h = self._handle()
        for i, t in enumerate(texPassArray):
            check(pt().pt_pass_set_texture(h, GL_TEXTURE_2D, t, f"texPass{i}".encode()))
        check(pt().pt_pass_draw(h))

    def reset_texture_slot(self) -> None:
        self.texture_slot = 0
        check(pt().pt_pass_reset_texture_slot(self._handle()))

    def set_texture_uniform(self, target: int, texture: int, uniform_name: str) -> None:
        check(pt().pt_pass_set_texture(self._handle(), target, texture, uniform_name.encode()))
        self.texture_slot += 1

    def set_uniform_mat4(self, name: str, value) -> None:
        m = np.ascontiguousarray(value, dtype=np.float32).reshape(16)
        check(pt().pt_pass_set_uniform_mat4(self._handle(), name.encode(), fptr(m)))

    def set_uniform_float(self, name: str, value: float) -> None:
        check(pt().pt_pass_set_uniform_float(self._handle(), name.encode(), float(np.float32(value))))

    def set_uniform_int(self, name: str, value: int) -> None:
        check(pt().pt_pass_set_uniform_int(self._handle(), name.encode(), int(value)))

    def set_uniform_uint(self, name: str, value: int) -> None:
        check(pt().pt_pass_set_uniform_uint(self._handle(), name.encode(), int(value) & 0xFFFFFFFF))

    def set_uniform_bool(self, name: str, value: bool) -> None:
        check(pt().pt_pass_set_uniform_bool(self._handle(), name.encode(), 1 if value else 0))

    def set_uniform_vec3(self, name: str, value) -> None:
        v = np.ascontiguousarray(value, dtype=np.float32).reshape(3)
        check(pt().pt_pass_set_uniform_vec3(self._handle(), name.encode(), fptr(v)))

    # MI355X extensions
    def set_rows(self, y0: int, y1: int) -> None:
        check(pt().pt_pass_set_rows(self._handle(), y0, y1))

    def set_row_cost(self, device_ptr: int) -> None:
        """Accumulate per-row BVH visits into a device uint32 array (path tracer; 0 disables)."""
        check(pt().pt_pass_set_row_cost(self._handle(), C.c_void_p(device_ptr or None)))

    def set_trace_stats(self, device_ptr: int, count: int = 14) -> None:
        """Path-tracing pass: add traversal counters (`count` x uint64, pt_pass_set_trace_stats_n; the library writes
        pt_trace_stats_count() = 14, and none past `count`) on every draw (0 disables)."""
        check(pt().pt_pass_set_trace_stats_n(self._handle(), C.c_void_p(device_ptr or None), count))

    def set_motion_bound(self, device_ptr: int) -> None:
        """G-buffer pass: store the largest |motion.y| of every draw into a device uint32 (float bits; 0 disables)."""
        check(pt().pt_pass_set_motion_bound(self._handle(), C.c_void_p(device_ptr or None)))

    def destroy(self) -> None:
        if self._h is not None:
            check(pt().pt_pass_destroy(self._h))
            self._h = None

    def last_ms(self) -> float:
        v = C.c_float()
        check(pt().pt_pass_last_ms(self._handle(), C.byref(v)))
        return v.value


class Rasterize_RenderPass(RenderPass):
    """Utils/render_pass.h:5-80 — the G-buffer pass over the model's vertex list."""

    def bindData(self, vertices) -> None:  # type: ignore[override]
        h = self._handle()
        for t in self.colorAttachments:
            check(pt().pt_pass_add_color_attachment(h, t))
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1)
        check(pt().pt_raster_pass_bind(h, fptr(v), v.size))

    def rebind_vertices(self, vertices) -> None:
        """A new vertex list for the bound pass (moved geometry): pt_raster_pass_bind again, attachments kept."""
        v = np.ascontiguousarray(vertices, dtype=np.float32).reshape(-1)
        check(pt().pt_raster_pass_bind(self._handle(), fptr(v), v.size))

    def rebind_vertices_device(self, device_ptr: int, n_floats: int, ploc_radius: int = 16) -> None:
        """pt_raster_pass_bind_device: the vertex list already in device memory, its tree built on the GPU."""
        check(pt().pt_raster_pass_bind_device(self._handle(), C.c_void_p(device_ptr), n_floats, ploc_radius))

    def adopt(self, y0: int, y1: int) -> None:
        """pt_raster_pass_adopt: the attachments' rows [y0, y1) were written elsewhere (another rank's draw of the same
        frame); derive the a-trous side data a draw makes, on the current library stream."""
        check(pt().pt_raster_pass_adopt(self._handle(), y0, y1))

    def share_vertices(self, src: "Rasterize_RenderPass") -> None:
        """pt_raster_pass_share: draw src's triangles and tree (src bound on its own)."""
        check(pt().pt_raster_pass_share(self._handle(), src._handle()))
