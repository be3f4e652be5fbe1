"""HDRLoader::load (lib/hdrloader.cpp) restated as pts_load_hdr: Radiance RGBE files written here in the three
encodings the loader reads — flat pixels (scanlines shorter than 8), the new per-component run-length format,
and the old (1,1,1,n) repeat run — decode to (v / 256) * 2^(E - 128) per component in file scanline order
(hdrloader.cpp:101-117), compared with an independent numpy decode. The asset room.hdr is absent (SURVEY.md
§8(d)); these synthetic files are the fixtures."""
import os
import tempfile

import numpy as np
import pytest

from ptsvgf.scene import load_hdr


def _decode(px):
    px = px.astype(np.float64)
    return (px[..., :3] / 256.0 * np.exp2(px[..., 3:4] - 128.0)).astype(np.float32)


def _header(w, h):
    return b"#?RADIANCE\nFORMAT=32-bit_rle_rgbe\nEXPOSURE=1.0\n\n" + f"-Y {h} +X {w}\n".encode()


def _rle_scanline(line):
    """New-format scanline: 2, 2, hi(w), lo(w), then each component as runs (>128) and literals."""
    w = line.shape[0]
    out = bytearray([2, 2, w >> 8, w & 255])
    for c in range(4):
        v = line[:, c]
        j = 0
        while j < w:
            r = 1
            while j + r < w and r < 127 and v[j + r] == v[j]:
                r += 1
            if r >= 3:
                out += bytes([128 + r, int(v[j])])
                j += r
            else:
                k = j
                while k < w and k - j < 128 and not (k + 2 < w and v[k] == v[k + 1] == v[k + 2]):
                    k += 1
                out += bytes([k - j]) + bytes(int(x) for x in v[j:k])
                j = k
    return bytes(out)


def _write(path, data: bytes):
    with open(path, "wb") as f:
        f.write(data)


def _pixels(rng, h, w, runs=False):
    px = rng.integers(0, 256, (h, w, 4), dtype=np.uint8)
    px[..., 3] = rng.integers(120, 140, (h, w))
    if runs:
        px[:, 3:20, :] = px[:, 3:4, :]
    return px


def test_flat_scanlines_short_width():
    rng = np.random.default_rng(1)
    px = _pixels(rng, 5, 6)  # w < 8: oldDecrunch reads flat RGBE quadruples
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "flat.hdr")
        _write(p, _header(6, 5) + px.tobytes())
        got = load_hdr(p)
    assert got.shape == (5, 6, 3)
    assert np.array_equal(got, _decode(px))


def test_new_rle_scanlines_with_runs():
    rng = np.random.default_rng(2)
    h, w = 7, 40
    px = _pixels(rng, h, w, runs=True)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "rle.hdr")
        _write(p, _header(w, h) + b"".join(_rle_scanline(px[y]) for y in range(h)))
        got = load_hdr(p)
    assert np.array_equal(got, _decode(px))  # row 0 = the first scanline in the file, as the reference stores


def test_old_rle_repeat_run():
    px = np.array([[[10, 20, 30, 130], [1, 1, 1, 3], [40, 50, 60, 129]]], np.uint8)  # pixel, repeat x3, pixel
    want = np.array([[[10, 20, 30, 130]] * 4 + [[40, 50, 60, 129]]], np.uint8)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "old.hdr")
        _write(p, _header(5, 1) + px.tobytes())
        got = load_hdr(p)
    assert np.array_equal(got, _decode(want))


def test_malformed_files_are_errors():
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "bad.hdr")
        _write(p, b"P6\n")
        with pytest.raises(RuntimeError):
            load_hdr(p)
        _write(p, _header(16, 4) + b"\x02\x02\x00\x10" + b"\x85")  # truncated run
        with pytest.raises(RuntimeError):
            load_hdr(p)
        with pytest.raises(RuntimeError):
            load_hdr(os.path.join(d, "missing.hdr"))
