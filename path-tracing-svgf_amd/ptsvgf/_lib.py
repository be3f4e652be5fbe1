"""ctypes bindings for the in-tree native libraries.

``lib/libptsvgf.so``      HIP kernels + the C ABI of include/ptsvgf.h
``lib/libptsvgf_host.so`` host scene preparation (include/ptsvgf_scene.h)

There is no fallback: if a library is missing the import fails loudly with the
command that builds it. Every ``pt_*`` call is checked; a negative status raises
:class:`PtError` carrying ``pt_last_error()``.
"""
from __future__ import annotations

import ctypes as C
import os

_HERE = os.path.dirname(os.path.abspath(__file__))
PKG_ROOT = os.path.dirname(_HERE)
LIB_DIR = os.path.join(PKG_ROOT, "lib")
REPO_ROOT = os.path.dirname(PKG_ROOT)
INCLUDE_DIR = os.path.join(REPO_ROOT, "include")

PT_TEXTURE_2D = 0x0DE1
PT_TEXTURE_BUFFER = 0x8C2A
PT_TEXTURE_2D_ARRAY = 0x8C1A
PT_RGB32F = 0x8815
PT_RGBA32F = 0x8814

ERRORS = {
    -1: "PT_ERR_INVALID_HANDLE",
    -2: "PT_ERR_UNKNOWN_PROGRAM",
    -3: "PT_ERR_FILE",
    -4: "PT_ERR_MISSING_TEXTURE",
    -5: "PT_ERR_HIP",
    -6: "PT_ERR_ARG",
    -7: "PT_ERR_FORMAT",
    -8: "PT_ERR_NO_DEVICE",
    -9: "PT_ERR_STATE",
}


class PtError(RuntimeError):
    def __init__(self, code: int, msg: str):
        super().__init__(f"{ERRORS.get(code, code)}: {msg}")
        self.code = code


def _load(name: str) -> C.CDLL:
    # One HIP runtime per process: PyTorch-ROCm ships its own libamdhip64.so.7 and the dynamic loader
    # binds every later request for that soname to whichever copy came first. Load torch's first, so the
    # streams and buffers torch hands to the C ABI (renderer frames in flight, bench, dist) live in the
    # same runtime as the kernels; loading /opt/rocm's first leaves torch without a device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    # PTSVGF_LIB_DIR: an alternative in-tree build (A/B experiments, tools/exp_*.sh)
    path = os.path.join(os.environ.get("PTSVGF_LIB_DIR", LIB_DIR), name)
    if not os.path.exists(path):
        raise ImportError(
            f"{path} is missing: build it with `make -C {PKG_ROOT}` "
            "(or __graft_entry__.build()); there is no CPU fallback"
        )
    return C.CDLL(path)


_u32 = C.c_uint32
_u32p = C.POINTER(C.c_uint32)
_fp = C.POINTER(C.c_float)
_vp = C.c_void_p

# (name, restype, argtypes)
_PT_SIGS = [
    ("pt_init", C.c_int, [C.c_int]),
    ("pt_shutdown", C.c_int, []),
    ("pt_set_stream", C.c_int, [_vp]),
    ("pt_use_own_stream", C.c_int, []),
    ("pt_stream_release", C.c_int, [_vp]),
    ("pt_stream_create_cu_masked", C.c_int, [C.c_uint32, C.POINTER(C.c_uint32), C.POINTER(C.c_void_p)]),
    ("pt_stream_create_priority", C.c_int, [C.c_int, C.POINTER(C.c_void_p)]),
    ("pt_stream_priority_range", C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pt_stream_destroy", C.c_int, [_vp]),
    ("pt_tree_check", C.c_int, [C.POINTER(C.c_float), C.c_int, C.POINTER(C.c_float), C.c_int, C.c_int, C.c_int,
                                C.POINTER(C.c_double), C.c_int]),
    ("pt_device_cus", C.c_int, [C.POINTER(C.c_int)]),
    ("pt_sync", C.c_int, []),
    ("pt_last_error", C.c_char_p, []),
    ("pt_version", C.c_int, []),
    ("pt_set_band", C.c_int, [C.c_int] * 6),
    ("pt_set_profiling", C.c_int, [C.c_int]),
    ("pt_program_create", C.c_int, [C.c_char_p, C.c_char_p, _u32p]),
    ("pt_texture2d_create", C.c_int, [C.c_int, C.c_int, _u32p]),
    ("pt_texture2d_upload", C.c_int, [_u32, C.c_int, C.c_int, _u32, _fp]),
    ("pt_texture2d_wrap", C.c_int, [_vp, C.c_int, C.c_int, _u32p]),
    ("pt_texbuffer_create", C.c_int, [_vp, C.c_size_t, _u32, _u32p]),
    ("pt_bvh_build", C.c_int, [_u32, C.c_int, C.c_int, _u32, _u32, C.POINTER(C.c_int), _fp]),
    ("pt_texarray_create", C.c_int, [C.c_int, C.c_int, C.c_int, _u32p]),
    ("pt_texarray_upload_layer", C.c_int, [_u32, C.c_int, C.c_int, C.c_int, C.c_int, C.POINTER(C.c_uint8)]),
    ("pt_texture_readback", C.c_int, [_u32, _fp, C.c_size_t]),
    ("pt_texture_upload_rgba", C.c_int, [_u32, _fp, C.c_size_t]),
    ("pt_texture_device_ptr", C.c_int, [_u32, C.POINTER(_vp)]),
    ("pt_texture_info", C.c_int, [_u32, C.POINTER(C.c_int), C.POINTER(C.c_int), C.POINTER(C.c_int)]),
    ("pt_texture_destroy", C.c_int, [_u32]),
    ("pt_pass_create", C.c_int, [_u32, C.c_int, C.c_int, _u32p]),
    ("pt_pass_add_color_attachment", C.c_int, [_u32, _u32]),
    ("pt_pass_bind", C.c_int, [_u32, C.c_int]),
    ("pt_raster_pass_bind", C.c_int, [_u32, _fp, C.c_size_t]),
    ("pt_raster_pass_bind_device", C.c_int, [_u32, _vp, C.c_size_t, C.c_int]),
    ("pt_raster_pass_share", C.c_int, [_u32, _u32]),
    ("pt_raster_pass_adopt", C.c_int, [_u32, C.c_int, C.c_int]),
    ("pt_tiles_count", C.c_int, [C.c_int] * 6 + [C.POINTER(C.c_int64)]),
    ("pt_tiles_copy", C.c_int, [_u32p, C.c_int, C.c_int, C.c_int, _vp, C.c_int, C.c_int]),
    ("pt_pass_reset_texture_slot", C.c_int, [_u32]),
    ("pt_pass_set_texture", C.c_int, [_u32, _u32, _u32, C.c_char_p]),
    ("pt_pass_set_uniform_mat4", C.c_int, [_u32, C.c_char_p, _fp]),
    ("pt_pass_set_uniform_float", C.c_int, [_u32, C.c_char_p, C.c_float]),
    ("pt_pass_set_uniform_int", C.c_int, [_u32, C.c_char_p, C.c_int]),
    ("pt_pass_set_uniform_uint", C.c_int, [_u32, C.c_char_p, C.c_uint32]),
    ("pt_pass_set_uniform_bool", C.c_int, [_u32, C.c_char_p, C.c_int]),
    ("pt_pass_set_uniform_vec3", C.c_int, [_u32, C.c_char_p, _fp]),
    ("pt_pass_set_rows", C.c_int, [_u32, C.c_int, C.c_int]),
    ("pt_pass_set_row_cost", C.c_int, [_u32, C.c_void_p]),
    ("pt_pass_set_motion_bound", C.c_int, [_u32, C.c_void_p]),
    ("pt_pass_set_trace_stats", C.c_int, [_u32, C.c_void_p]),
    ("pt_pass_set_trace_stats_n", C.c_int, [_u32, C.c_void_p, C.c_int]),
    ("pt_trace_stats_count", C.c_int, []),
    ("pt_pass_draw", C.c_int, [_u32]),
    ("pt_pass_draw_batch", C.c_int, [C.POINTER(_u32), C.c_int]),
    ("pt_pass_last_ms", C.c_int, [_u32, _fp]),
    ("pt_pass_destroy", C.c_int, [_u32]),
]

_PTS_SIGS = [
    ("pts_scene_create", _vp, []),
    ("pts_scene_destroy", None, [_vp]),
    ("pts_scene_add_obj", C.c_int, [_vp, C.c_char_p, _fp, _fp, C.c_int, C.c_int]),
    ("pts_scene_add_mesh", C.c_int, [_vp, _fp, _fp, C.c_int, C.POINTER(C.c_int), C.c_int, _fp, _fp, C.c_int, C.c_int]),
    ("pts_scene_add_raw", C.c_int, [_vp, _fp, C.c_int, _fp, C.c_int]),
    ("pts_scene_build_bvh", C.c_int, [_vp, C.c_int]),
    ("pts_scene_counts", C.c_int, [_vp, C.POINTER(C.c_int64)]),
    ("pts_scene_root_aabb", C.c_int, [_vp, _fp]),
    ("pts_scene_encode", C.c_int, [_vp, _fp, _fp, _fp]),
    ("pts_transform_matrix", None, [_fp, _fp, _fp, _fp]),
    ("pts_hdr_cache", C.c_int, [_fp, C.c_int, C.c_int, _fp]),
    ("pts_gen_plant", C.c_int, [C.c_uint32, C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), _fp, C.POINTER(C.c_int)]),
    ("pts_gen_teapot", C.c_int, [C.c_int, C.POINTER(C.c_int), C.POINTER(C.c_int), _fp, C.POINTER(C.c_int)]),
    ("pts_gen_cornell", C.c_int, [C.POINTER(C.c_int), C.POINTER(C.c_int), _fp, C.POINTER(C.c_int)]),
    ("pts_gen_env_map", C.c_int, [C.c_int, C.c_int, _fp]),
    ("pts_load_hdr", C.c_int, [C.c_char_p, C.POINTER(C.c_int), C.POINTER(C.c_int), _fp]),
    ("pts_last_error", C.c_char_p, []),
]

_pt = None
_pts = None


def _bind(lib: C.CDLL, sigs) -> C.CDLL:
    for name, res, args in sigs:
        fn = getattr(lib, name)
        fn.restype = res
        fn.argtypes = args
    return lib


def pt() -> C.CDLL:
    """The HIP library (kernels + C ABI)."""
    global _pt
    if _pt is None:
        _pt = _bind(_load("libptsvgf.so"), _PT_SIGS)
    return _pt


def pts() -> C.CDLL:
    """Host scene preparation library (no GPU needed)."""
    global _pts
    if _pts is None:
        _pts = _bind(_load("libptsvgf_host.so"), _PTS_SIGS)
    return _pts


def check(rc: int) -> int:
    if rc < 0:
        raise PtError(rc, (pt().pt_last_error() or b"").decode())
    return rc


def check_host(rc: int) -> int:
    if rc < 0:
        raise RuntimeError((pts().pts_last_error() or b"").decode())
    return rc


def fptr(a):
    """float32 numpy array -> POINTER(c_float) (array must stay alive)."""
    return a.ctypes.data_as(_fp)


def exported_symbols():
    return [n for n, _, _ in _PT_SIGS], [n for n, _, _ in _PTS_SIGS]
