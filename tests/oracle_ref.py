"""ctypes wrapper over the CPU oracle (oracle/_build/liboracle.so).

TEST INFRASTRUCTURE ONLY — imported by tests/, __graft_entry__.smoke() and
bench.py's cpu_baseline leg as the checker, never by the product.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
ORACLE_DIR = os.path.join(REPO, "oracle")
ORACLE_SO = os.path.join(ORACLE_DIR, "_build", "liboracle.so")

_fp = C.POINTER(C.c_float)
_lib = None


class PTParams(C.Structure):
    _fields_ = [("frameCounter", C.c_uint32), ("width", C.c_int), ("height", C.c_int), ("eye", C.c_float * 3),
                ("cameraRotate", C.c_float * 16), ("accumulate", C.c_int), ("clamp_threshold", C.c_float),
                ("max_tracing_depth", C.c_int), ("aspect_corrected", C.c_int), ("y_begin", C.c_int),
                ("y_end", C.c_int), ("use_normal_map", C.c_int)]


def lib() -> C.CDLL:
    global _lib
    if _lib is None:
        if not os.path.exists(ORACLE_SO):
            subprocess.run(["make", "-C", ORACLE_DIR], check=True, capture_output=True)
        L = C.CDLL(ORACLE_SO)
        L.orc_scene_create.restype = C.c_void_p
        L.orc_scene_create.argtypes = [_fp, C.c_int, _fp, C.c_int, _fp, C.c_int, _fp, _fp, C.c_int, C.c_int]
        L.orc_scene_destroy.argtypes = [C.c_void_p]
        L.orc_scene_set_material_array.argtypes = [C.c_void_p, C.c_void_p, C.c_int, C.c_int, C.c_int]
        L.orc_path_trace.argtypes = [C.c_void_p, C.POINTER(PTParams), _fp, _fp, _fp, _fp, C.c_int]
        L.orc_gbuffer.argtypes = [_fp, C.c_int, C.c_int, C.c_int, _fp, _fp, _fp, _fp, _fp, _fp, _fp, C.c_int]
        L.orc_reproject.argtypes = [C.c_int, C.c_int] + [_fp] * 9 + [C.c_float] * 4 + [_fp, _fp, C.c_int]
        L.orc_variance.argtypes = [C.c_int, C.c_int, _fp, _fp, _fp, _fp, C.c_float, C.c_float, C.c_float, C.c_float,
                                   _fp, C.c_int]
        L.orc_atrous.argtypes = [C.c_int, C.c_int, _fp, _fp, _fp, C.c_int, C.c_float, C.c_float, C.c_float,
                                 C.c_float, _fp, C.c_int]
        L.orc_modulate.argtypes = [C.c_int, C.c_int, _fp, _fp, _fp, _fp, _fp, C.c_int]
        L.orc_output.argtypes = [C.c_int, C.c_int, _fp, _fp, C.c_int]
        L.orc_taa.argtypes = [C.c_int, C.c_int, _fp, _fp, _fp, _fp, C.c_uint32, _fp, C.c_int]
        L.orc_wang_hash.restype = C.c_uint32
        L.orc_wang_hash.argtypes = [C.c_uint32]
        L.orc_sobol.restype = C.c_float
        L.orc_sobol.argtypes = [C.c_uint32, C.c_uint32]
        L.orc_brdf_eval.argtypes = [_fp, _fp, _fp, _fp, _fp]
        L.orc_brdf_pdf.restype = C.c_float
        L.orc_brdf_pdf.argtypes = [_fp, _fp, _fp, _fp]
        L.orc_hit_aabb.restype = C.c_float
        L.orc_hit_aabb.argtypes = [_fp, _fp, _fp, _fp]
        L.orc_hit_triangle.argtypes = [_fp, _fp, _fp, _fp, _fp]
        L.orc_math.argtypes = [C.c_int, _fp, C.c_int, _fp]
        _lib = L
    return _lib


def fp(a: np.ndarray):
    assert a.dtype == np.float32 and a.flags["C_CONTIGUOUS"]
    return a.ctypes.data_as(_fp)


def f32(a) -> np.ndarray:
    return np.ascontiguousarray(a, dtype=np.float32)


def frame(H: int, W: int) -> np.ndarray:
    return np.zeros((H, W, 4), np.float32)


THREADS = min(8, os.cpu_count() or 1)


class OracleScene:
    def __init__(self, scene):
        self.s = scene
        self._keep = [f32(scene.tri_enc), f32(scene.node_enc), f32(scene.lights), f32(scene.hdr), f32(scene.cache)]
        t, n, l, h, c = self._keep
        self.h = lib().orc_scene_create(fp(t), t.shape[0], fp(n), n.shape[0], fp(l), l.shape[0], fp(h), fp(c),
                                        h.shape[1], h.shape[0])
        tex = getattr(scene, "textures", None)
        if tex is not None:  # (layers, h, w, 4) uint8 material_array
            tex = np.ascontiguousarray(tex, np.uint8)
            self._keep.append(tex)
            assert lib().orc_scene_set_material_array(self.h, tex.ctypes.data, tex.shape[2], tex.shape[1],
                                                      tex.shape[0]) == 0

    def __del__(self):
        if getattr(self, "h", None):
            lib().orc_scene_destroy(self.h)
            self.h = None

    def path_trace(self, W, H, frameCounter, eye, cameraRotate, clamp_threshold=10.0, max_depth=2,
                   aspect_corrected=False, accumulate=False, last_frame=None, rows=None, threads=THREADS,
                   use_normal_map=False):
        p = PTParams()
        p.frameCounter = frameCounter & 0xFFFFFFFF
        p.width, p.height = W, H
        p.eye[:] = [float(v) for v in np.asarray(eye, np.float32)]
        p.cameraRotate[:] = [float(v) for v in np.asarray(cameraRotate, np.float32).reshape(16)]
        p.accumulate = int(accumulate)
        p.clamp_threshold = float(np.float32(clamp_threshold))
        p.max_tracing_depth = max_depth
        p.aspect_corrected = int(aspect_corrected)
        p.y_begin, p.y_end = rows if rows else (0, H)
        p.use_normal_map = int(use_normal_map)
        col, em, al = frame(H, W), frame(H, W), frame(H, W)
        lf = f32(last_frame) if last_frame is not None else None
        rc = lib().orc_path_trace(self.h, C.byref(p), fp(lf) if lf is not None else None, fp(col), fp(em), fp(al),
                                  threads)
        assert rc == 0
        return col, em, al


def gbuffer(raster, W, H, view, proj, pre_viewproj, threads=THREADS):
    r = f32(raster)
    v, p, pv = f32(view).reshape(16), f32(proj).reshape(16), f32(pre_viewproj).reshape(16)
    outs = [frame(H, W) for _ in range(4)]
    lib().orc_gbuffer(fp(r), r.size // 18, W, H, fp(v), fp(p), fp(pv), *[fp(o) for o in outs], threads)
    return dict(world=outs[0], normal_depth=outs[1], velocity=outs[2], fwidth=outs[3])


def reproject(motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fwidth, inv_w, inv_h,
              depth_thr=10.0, normal_thr=16.0, threads=THREADS):
    H, W, _ = color.shape
    ins = [f32(a) for a in (motion, color, albedo, emission, prev_illum, prev_moments, nd, prev_nd, fwidth)]
    oi, om = frame(H, W), frame(H, W)
    lib().orc_reproject(W, H, *[fp(a) for a in ins], np.float32(inv_w), np.float32(inv_h), np.float32(depth_thr),
                        np.float32(normal_thr), fp(oi), fp(om), threads)
    return oi, om


def variance(illum, moments, nd, fwidth, phi_color=4.0, phi_normal=128.0, threads=THREADS):
    H, W, _ = illum.shape
    ins = [f32(a) for a in (illum, moments, nd, fwidth)]
    o = frame(H, W)
    lib().orc_variance(W, H, *[fp(a) for a in ins], phi_color, phi_normal, 1.0 / W, 1.0 / H, fp(o), threads)
    return o


def atrous(illum, nd, fwidth, step, phi_color=4.0, phi_normal=128.0, threads=THREADS):
    H, W, _ = illum.shape
    ins = [f32(a) for a in (illum, nd, fwidth)]
    o = frame(H, W)
    lib().orc_atrous(W, H, *[fp(a) for a in ins], step, phi_color, phi_normal, 1.0 / W, 1.0 / H, fp(o), threads)
    return o


def modulate(albedo, emission, illum, nd, threads=THREADS):
    H, W, _ = illum.shape
    ins = [f32(a) for a in (albedo, emission, illum, nd)]
    o = frame(H, W)
    lib().orc_modulate(W, H, *[fp(a) for a in ins], fp(o), threads)
    return o


def taa(cur, prev, velocity, nd, frame_counter, threads=THREADS):
    H, W, _ = cur.shape
    ins = [f32(a) for a in (cur, prev, velocity, nd)]
    o = frame(H, W)
    lib().orc_taa(W, H, *[fp(a) for a in ins], int(frame_counter), fp(o), threads)
    return o


def output(color, threads=THREADS):
    H, W, _ = color.shape
    c = f32(color)
    o = frame(H, W)
    lib().orc_output(W, H, fp(c), fp(o), threads)
    return o


class OracleFrameLoop:
    """main.cpp:436-553 on the oracle: G-buffer -> PT -> reproject -> variance -> a-trous x N -> modulate,
    with the reference's history plumbing (iteration-1 a-trous output becomes next frame's gPrevIllum).

    Accumulate mode (cfg.accumulate_color, path_tracing.frag:1116-1119): lastFrame is last_acc_color, which
    save_frame_data (main.cpp:546-553, save_frame_data.frag accColor) refreshes from this frame's curColor."""

    def __init__(self, scene, W, H, cfg=None, aspect_corrected=None, threads=THREADS, run_taa=True,
                 run_output=False):
        from ptsvgf.camera import Camera, mat_mul, parameter_config
        self.scene = scene
        self.os = OracleScene(scene)
        self.W, self.H = W, H
        self.cfg = cfg or parameter_config()
        self.camera = Camera(W, H)
        self.aspect_corrected = (W != H) if aspect_corrected is None else aspect_corrected
        self.threads = threads
        self.run_taa, self.run_output = run_taa, run_output
        self.pre_viewproj = mat_mul(self.camera.cam_proj_mat, self.camera.cam_view_mat)
        z = lambda: frame(H, W)  # noqa: E731
        self.prev_illum, self.prev_moments, self.prev_nd, self.prev_taa = z(), z(), z(), z()
        self.prev_acc = z()  # last_acc_color (zero-filled like every build texture)
        self._mat_mul = mat_mul

    def frame(self):
        from ptsvgf.camera import rigid_inverse
        cam, cfg, W, H = self.camera, self.cfg, self.W, self.H
        cam.update()
        view, proj = cam.cam_view_mat, cam.cam_proj_mat
        g = gbuffer(self.scene.raster, W, H, view, proj, self.pre_viewproj, self.threads)
        col, em, al = self.os.path_trace(W, H, cam.frameCounter, cam.cam_position, rigid_inverse(view),
                                         cfg.clamp_threshold, cfg.max_tracing_depth, self.aspect_corrected,
                                         accumulate=cfg.accumulate_color,
                                         last_frame=self.prev_acc if cfg.accumulate_color else None,
                                         threads=self.threads, use_normal_map=cfg.use_normal_texture)
        ri, rm = reproject(g["velocity"], col, al, em, self.prev_illum, self.prev_moments, g["normal_depth"],
                           self.prev_nd, g["fwidth"], np.float32(1.0 / W), np.float32(1.0 / H),
                           cfg.reproj_depth_threshold, cfg.reproj_normal_threshold, self.threads)
        v = variance(ri, rm, g["normal_depth"], g["fwidth"], cfg.sigma_l, cfg.sigma_n, self.threads)
        a = v
        hist = self.prev_illum
        for i in range(cfg.num_atrous_iterations):
            a = atrous(a, g["normal_depth"], g["fwidth"], 1 << i, cfg.sigma_l, cfg.sigma_n, self.threads)
            if i == 1:
                hist = a
        m = modulate(al, em, a, g["normal_depth"], self.threads)
        out = dict(g, color=col, emission=em, albedo=al, reproj_illum=ri, reproj_moments=rm, variance=v, atrous=a,
                   history_illum=hist, modulate=m)
        if self.run_taa:                                                  # main.cpp:537-544
            out["final"] = self.prev_taa = taa(m, self.prev_taa, g["velocity"], g["normal_depth"], cam.frameCounter,
                                               self.threads)
            if self.run_output:                                           # main.cpp:555-591
                out["output"] = output(out["final"], self.threads)
        self.prev_illum, self.prev_moments, self.prev_nd = hist, rm, g["normal_depth"]
        self.prev_acc = col
        self.pre_viewproj = self._mat_mul(proj, view)
        cam.frameCounter += 1
        return out
