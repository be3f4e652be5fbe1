"""The drop-in boundary: the C-ABI libraries load on a CPU-only host, export
every entry point include/*.h declares, and refuse compute without a device."""
import ctypes as C
import os
import re

import pytest

from ptsvgf import _lib

INC = _lib.INCLUDE_DIR


def _declared(header: str, prefix: str):
    txt = open(os.path.join(INC, header)).read()
    txt = re.sub(r"/\*.*?\*/", "", txt, flags=re.S)
    return sorted(set(re.findall(r"\b(" + prefix + r"_\w+)\s*\(", txt)))


def test_headers_declare_the_boundary():
    pt = _declared("ptsvgf.h", "pt")
    for name in ("pt_program_create", "pt_texture2d_create", "pt_texbuffer_create", "pt_pass_create",
                 "pt_pass_add_color_attachment", "pt_pass_bind", "pt_pass_draw", "pt_pass_reset_texture_slot",
                 "pt_pass_set_texture", "pt_pass_set_uniform_mat4", "pt_raster_pass_bind", "pt_texture_readback",
                 "pt_sync", "pt_init", "pt_set_band"):
        assert name in pt


def test_gpu_library_exports_every_declared_symbol():
    lib = C.CDLL(os.path.join(_lib.LIB_DIR, "libptsvgf.so"))
    missing = [n for n in _declared("ptsvgf.h", "pt") + _declared("ptsvgf_scene.h", "pts") if not hasattr(lib, n)]
    assert not missing, missing


def test_host_library_exports_scene_symbols():
    lib = C.CDLL(os.path.join(_lib.LIB_DIR, "libptsvgf_host.so"))
    missing = [n for n in _declared("ptsvgf_scene.h", "pts") if not hasattr(lib, n)]
    assert not missing, missing


def test_python_bindings_cover_the_headers():
    pt_names, pts_names = _lib.exported_symbols()
    assert set(_declared("ptsvgf.h", "pt")) <= set(pt_names)
    assert set(_declared("ptsvgf_scene.h", "pts")) <= set(pts_names)


def test_calls_before_init_fail_loudly():
    L = _lib.pt()
    h = C.c_uint32()
    rc = L.pt_texture2d_create(4, 4, C.byref(h))
    if rc == 0:
        pytest.skip("library already initialised in this process")
    assert rc == -9  # PT_ERR_STATE
    assert b"pt_init" in L.pt_last_error()


def test_init_without_device_reports_no_device():
    try:
        import torch
        if torch.cuda.is_available():
            pytest.skip("a GPU is visible")
    except ImportError:
        pass
    L = _lib.pt()
    assert L.pt_init(0) == -8  # PT_ERR_NO_DEVICE
    assert b"device" in L.pt_last_error()
