"""Scene assembly (reference layer L1) on the native host library.

Produces exactly the buffers ``main.cpp`` uploads (main.cpp:65-181): encoded
triangles (Triangle_encoded, 45 floats), BVH nodes (BVHNode_encoded, 12 floats,
dummy node 0), point lights (6 floats each), the raster vertex list, the HDR
environment and its importance cache.

Assets: ``assets/models/{clock,table}.obj`` are the reference's own meshes.
``plant.obj``, ``teapot.obj``, ``room.hdr`` and every texture are absent from
the reference (.MISSING_LARGE_BLOBS), so the scenes use deterministic
synthetic stand-ins generated natively (pts_gen_*) and constant materials.
"""
from __future__ import annotations

import ctypes as C
import os
import time
from dataclasses import dataclass, field

import numpy as np

from ._lib import REPO_ROOT, check_host, fptr, pts

ASSETS = os.path.join(REPO_ROOT, "assets", "models")

# main.cpp:157-160
POINT_LIGHTS = np.array([[0.5, 0.5, 0.5, 10, 10, 10],
                         [-0.5, 0.75, 0.5, 8, 4, 4],
                         [-0.5, 0.75, 0.75, 0, 3, 4],
                         [0.75, 0.75, 0.75, 12, 3, 4]], np.float32)


def material(baseColor=(1.0, 1.0, 1.0), emissive=(0.0, 0.0, 0.0), subsurface=0.0, metallic=0.0, specular=0.5,
             specularTint=0.0, roughness=0.5, anisotropic=0.0, sheen=0.0, sheenTint=0.5, clearcoat=0.0,
             clearcoatGloss=1.0, IOR=1.0, transmission=0.0) -> np.ndarray:
    """Utils/Material.h:8-22 defaults, packed as the 18 floats of ptsvgf_scene.h."""
    return np.array([*emissive, *baseColor, subsurface, metallic, specular, specularTint, roughness, anisotropic,
                     sheen, sheenTint, clearcoat, clearcoatGloss, IOR, transmission], np.float32)


def transform(rot=(0.0, 0.0, 0.0), trans=(0.0, 0.0, 0.0), scale=(1.0, 1.0, 1.0)) -> np.ndarray:
    """getTransformMatrix (obj_loader.h:166-182)."""
    out = np.zeros(16, np.float32)
    r, t, s = (np.asarray(v, np.float32) for v in (rot, trans, scale))
    pts().pts_transform_matrix(fptr(r), fptr(t), fptr(s), fptr(out))
    return out


@dataclass
class Scene:
    name: str
    tri_enc: np.ndarray        # (N, 45)
    node_enc: np.ndarray       # (M, 12)
    raster: np.ndarray         # (N*18,) raster vertex list (pre-BVH order)
    lights: np.ndarray         # (L, 6)
    hdr: np.ndarray            # (h, w, 3)
    cache: np.ndarray          # (h, w, 3)
    counts: dict = field(default_factory=dict)
    textures: np.ndarray | None = None  # material_array (layers, h, w, 4) uint8, or None (no texture path)

    @property
    def ntris(self) -> int:
        return int(self.tri_enc.shape[0])

    @property
    def hdr_resolution(self) -> int:
        return int(self.hdr.shape[1])


class SceneBuilder:
    def __init__(self):
        self._s = pts().pts_scene_create()
        if not self._s:
            raise RuntimeError("pts_scene_create failed")

    def __del__(self):
        if getattr(self, "_s", None):
            pts().pts_scene_destroy(self._s)
            self._s = None

    def add_obj(self, path: str, mat: np.ndarray, trans: np.ndarray, smooth: bool = True, obj_index: int = 0):
        check_host(pts().pts_scene_add_obj(self._s, path.encode(), fptr(mat), fptr(trans), int(smooth), obj_index))

    def add_mesh(self, positions: np.ndarray, indices: np.ndarray, mat: np.ndarray, trans: np.ndarray,
                 smooth: bool = True, obj_index: int = 0, uvs: np.ndarray | None = None):
        p = np.ascontiguousarray(positions, np.float32).reshape(-1)
        i = np.ascontiguousarray(indices, np.int32).reshape(-1)
        u = None if uvs is None else np.ascontiguousarray(uvs, np.float32).reshape(-1)
        check_host(pts().pts_scene_add_mesh(self._s, fptr(p), None if u is None else fptr(u), p.size // 3,
                                            i.ctypes.data_as(C.POINTER(C.c_int)), i.size // 3, fptr(mat), fptr(trans),
                                            int(smooth), obj_index))

    def build(self, leaf_n: int = 8):
        check_host(pts().pts_scene_build_bvh(self._s, leaf_n))

    def counts(self) -> dict:
        c = (C.c_int64 * 6)()
        check_host(pts().pts_scene_counts(self._s, c))
        return dict(triangles=c[0], nodes=c[1], leaves=c[2], max_depth=c[3], max_leaf=c[4], raster_floats=c[5])

    def root_aabb(self) -> np.ndarray:
        o = np.zeros(6, np.float32)
        check_host(pts().pts_scene_root_aabb(self._s, fptr(o)))
        return o

    def encode(self):
        c = self.counts()
        tri = np.zeros((c["triangles"], 45), np.float32)
        node = np.zeros((c["nodes"], 12), np.float32)
        raster = np.zeros(c["raster_floats"], np.float32)
        check_host(pts().pts_scene_encode(self._s, fptr(tri), fptr(node), fptr(raster)))
        return tri, node, raster


def _gen(fn, *args):
    nv, nt = C.c_int(), C.c_int()
    check_host(fn(*args, C.byref(nv), C.byref(nt), None, None))
    pos = np.zeros(nv.value * 3, np.float32)
    idx = np.zeros(nt.value * 3, np.int32)
    check_host(fn(*args, C.byref(nv), C.byref(nt), fptr(pos), idx.ctypes.data_as(C.POINTER(C.c_int))))
    return pos.reshape(-1, 3), idx.reshape(-1, 3)


def gen_plant(seed: int = 0, leaves: int = 150):
    return _gen(pts().pts_gen_plant, seed, leaves)


def gen_teapot(segments: int = 48):
    return _gen(pts().pts_gen_teapot, segments)


def gen_cornell():
    return _gen(pts().pts_gen_cornell)


def env_map(width: int = 2048, height: int = 1024) -> np.ndarray:
    out = np.zeros((height, width, 3), np.float32)
    check_host(pts().pts_gen_env_map(width, height, fptr(out)))
    return out


def load_hdr(path: str) -> np.ndarray:
    """HDRLoader::load (lib/hdrloader.cpp): Radiance RGBE -> (h, w, 3) float32, file scanline order."""
    w, h = C.c_int(), C.c_int()
    check_host(pts().pts_load_hdr(path.encode(), C.byref(w), C.byref(h), None))
    out = np.zeros((h.value, w.value, 3), np.float32)
    check_host(pts().pts_load_hdr(path.encode(), C.byref(w), C.byref(h), fptr(out)))
    return out


def hdr_cache(hdr: np.ndarray) -> np.ndarray:
    h, w, _ = hdr.shape
    a = np.ascontiguousarray(hdr, np.float32)
    out = np.zeros_like(a)
    check_host(pts().pts_hdr_cache(fptr(a), w, h, fptr(out)))
    return out


def material_layers(size: int = 256, image: int = 192, objects: int = 3, seed: int = 0) -> np.ndarray:
    """Synthetic stand-in for the reference's Textures/*.bmp (all absent): per object index o, layers 4o..4o+3 =
    albedo, metallic, normal, roughness (main.cpp:196-205 order), each an `image`-texel square uploaded at the
    origin of a `size`-texel layer — the reference's sub-rectangle upload into its 4096^2 array, so uv in [0, 1]
    also samples the unwritten (zero) texels beyond the image (help_func.h:12). Seeded, deterministic."""
    rng = np.random.default_rng(seed)
    out = np.zeros((4 * objects, size, size, 4), np.uint8)
    yy, xx = np.mgrid[0:image, 0:image].astype(np.float32) / image
    for o in range(objects):
        f = 4.0 + 3.0 * o
        check = ((np.floor(xx * f) + np.floor(yy * f)) % 2).astype(np.float32)
        base = rng.uniform(0.2, 0.9, 3).astype(np.float32)
        alb = np.stack([base[c] * (0.55 + 0.45 * check) for c in range(3)], -1)
        out[4 * o, :image, :image, :3] = np.round(alb * 255)
        out[4 * o + 1, :image, :image, 0] = np.round((0.5 + 0.5 * np.sin(6.28 * xx * (o + 1))) * 255)
        nx, ny = 0.35 * np.sin(6.28 * xx * f), 0.35 * np.cos(6.28 * yy * f)
        nz = np.sqrt(np.maximum(0.0, 1.0 - nx * nx - ny * ny))
        out[4 * o + 2, :image, :image, :3] = np.round((np.stack([nx, ny, nz], -1) * 0.5 + 0.5) * 255)
        out[4 * o + 3, :image, :image, 0] = np.round((0.2 + 0.6 * yy) * 255)
        out[4 * o:4 * o + 4, :image, :image, 3] = 255
    return out


def build_scene(name: str = "table_clock_plant", hdr_size=(2048, 1024), plant_leaves: int = 150,
                timings: dict | None = None) -> Scene:
    """Named scenes of BASELINE.json's configs.

    ``clock``               main.cpp:72-80 (textures absent -> constant brass material)
    ``table_clock_plant``   configs[1..4]: table + clock + synthetic plant (+ synthetic room.hdr)
    ``cornell_teapot``      configs[0]: Cornell-style box + synthetic teapot stand-in
    ``textured``            table + clock with the texture path: negative baseColor / metallic / roughness
                            select material_array layers objIndex*4 + {0, 1, 3} (path_tracing.frag:331-364)
    """
    b = SceneBuilder()
    clock = os.path.join(ASSETS, "clock.obj")
    table = os.path.join(ASSETS, "table.obj")
    brass = material(baseColor=(0.80, 0.62, 0.35), metallic=0.6, specular=0.0, roughness=0.35, clearcoat=0.0,
                     clearcoatGloss=0.0)
    if name == "clock":
        b.add_obj(clock, brass, transform(), True, 0)
    elif name == "table_clock_plant":
        wood = material(baseColor=(0.45, 0.28, 0.14), roughness=0.6, clearcoat=0.5, clearcoatGloss=0.8)
        leaf = material(baseColor=(0.16, 0.42, 0.12), roughness=0.7, sheen=0.3)
        # table top at y = -0.25, clock and plant standing on it, filling the default orbit view
        b.add_obj(table, wood, transform(trans=(0.176, -0.73, -0.16), scale=(3.84, 3.84, 3.84)), True, 0)
        b.add_obj(clock, brass, transform(trans=(-0.914, -0.155, -1.03), scale=(1.12, 1.12, 1.12)), True, 1)
        ppos, pidx = gen_plant(0, plant_leaves)
        b.add_mesh(ppos, pidx, leaf, transform(trans=(0.8, -0.4, -0.24), scale=(1.28, 1.28, 1.28)), True, 2)
    elif name == "cornell_teapot":
        white = material(baseColor=(0.73, 0.73, 0.73), roughness=0.8)
        china = material(baseColor=(0.85, 0.85, 0.80), roughness=0.25, clearcoat=1.0, clearcoatGloss=0.9)
        cpos, cidx = gen_cornell()
        b.add_mesh(cpos, cidx, white, transform(), False, 0)
        tpos, tidx = gen_teapot(48)
        b.add_mesh(tpos, tidx, china, transform(trans=(0.0, -1.0, 0.0), scale=(0.9, 0.9, 0.9)), True, 1)
    elif name == "textured":
        textured = material(baseColor=(-1.0, -1.0, -1.0), metallic=-1.0, roughness=-1.0, specular=0.5)
        half = material(baseColor=(0.6, 0.6, 0.6), metallic=-1.0, roughness=0.4)  # texture on one param only
        b.add_obj(table, half, transform(trans=(0.176, -0.73, -0.16), scale=(3.84, 3.84, 3.84)), True, 0)
        b.add_obj(clock, textured, transform(trans=(-0.914, -0.155, -1.03), scale=(1.12, 1.12, 1.12)), True, 1)
    else:
        raise ValueError(f"unknown scene {name!r}")
    t0 = time.perf_counter()
    b.build(8)  # buildBVHwithSAH (BVH.h:42-173) on the host, as main.cpp:96
    if timings is not None:
        timings["host_sah_build_ms"] = (time.perf_counter() - t0) * 1e3
    tri, node, raster = b.encode()
    hdr = env_map(*hdr_size)
    tex = material_layers() if name == "textured" else None
    return Scene(name, tri, node, raster, POINT_LIGHTS.copy(), hdr, hdr_cache(hdr), b.counts(), tex)
