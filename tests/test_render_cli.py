"""Image writers of the headless render CLI (ptsvgf.render_cli): the PNG decodes back (zlib + filter 0) to the
8-bit image top-down, the PFM holds the floats in GL row order."""
import os
import struct
import tempfile
import zlib

import numpy as np

from ptsvgf.render_cli import write_pfm, write_png


def test_png_roundtrip():
    rng = np.random.default_rng(0)
    img = rng.uniform(-0.2, 1.2, (5, 7, 4)).astype(np.float32)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.png")
        write_png(p, img)
        data = open(p, "rb").read()
    assert data[:8] == b"\x89PNG\r\n\x1a\n"
    pos, chunks = 8, {}
    while pos < len(data):
        n = struct.unpack(">I", data[pos:pos + 4])[0]
        tag = data[pos + 4:pos + 8]
        body = data[pos + 8:pos + 8 + n]
        assert struct.unpack(">I", data[pos + 8 + n:pos + 12 + n])[0] == zlib.crc32(tag + body) & 0xFFFFFFFF
        chunks[tag] = chunks.get(tag, b"") + body
        pos += 12 + n
    w, h = struct.unpack(">II", chunks[b"IHDR"][:8])
    assert (w, h) == (7, 5)
    raw = zlib.decompress(chunks[b"IDAT"])
    rows = [np.frombuffer(raw[y * (1 + 3 * w) + 1:(y + 1) * (1 + 3 * w)], np.uint8).reshape(w, 3) for y in range(h)]
    got = np.stack(rows)
    want = np.clip(np.round(img[::-1, :, :3] * 255), 0, 255).astype(np.uint8)
    assert np.array_equal(got, want)


def test_pfm_roundtrip():
    img = np.arange(2 * 3 * 4, dtype=np.float32).reshape(2, 3, 4)
    with tempfile.TemporaryDirectory() as d:
        p = os.path.join(d, "a.pfm")
        write_pfm(p, img)
        data = open(p, "rb").read()
    head = b"PF\n3 2\n-1.0\n"
    assert data.startswith(head)
    assert np.array_equal(np.frombuffer(data[len(head):], "<f4").reshape(2, 3, 3), img[..., :3])
