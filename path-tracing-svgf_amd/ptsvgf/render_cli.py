"""Headless render to image files: the reference's window loop (main.cpp:436-602) for N frames with the
debug-view switch of its GUI (main.cpp:398-415, gui_config.h:7-45) as a flag, the output pass's display image
written as PNG and, optionally, the selected plane's raw floats as PFM.

    python -m ptsvgf.render_cli --width 800 --height 800 --frames 8 --view final_pic --png out.png
"""
from __future__ import annotations

import argparse
import struct
import zlib

import numpy as np


def write_png(path: str, rgb01: np.ndarray) -> None:
    """8-bit RGB PNG of an (H, W, 3) image in [0, 1], GL row 0 (bottom) written last (images are top-down)."""
    img = np.clip(np.round(np.nan_to_num(rgb01[::-1, :, :3]) * 255.0), 0, 255).astype(np.uint8)
    h, w, _ = img.shape
    raw = b"".join(b"\x00" + img[y].tobytes() for y in range(h))

    def chunk(tag, data):
        return struct.pack(">I", len(data)) + tag + data + struct.pack(">I", zlib.crc32(tag + data) & 0xFFFFFFFF)

    with open(path, "wb") as f:
        f.write(b"\x89PNG\r\n\x1a\n" + chunk(b"IHDR", struct.pack(">IIBBBBB", w, h, 8, 2, 0, 0, 0)) +
                chunk(b"IDAT", zlib.compress(raw, 6)) + chunk(b"IEND", b""))


def write_pfm(path: str, rgb: np.ndarray) -> None:
    """Portable float map (little endian), rows bottom-up as PFM stores them = GL row order."""
    h, w, _ = rgb.shape
    with open(path, "wb") as f:
        f.write(f"PF\n{w} {h}\n-1.0\n".encode())
        f.write(np.ascontiguousarray(rgb[..., :3], "<f4").tobytes())


def main(argv=None) -> int:
    from . import gl
    from .camera import parameter_config
    from .renderer import Renderer
    from .scene import build_scene, load_hdr

    ap = argparse.ArgumentParser(description=__doc__.splitlines()[0])
    ap.add_argument("--width", type=int, default=800)
    ap.add_argument("--height", type=int, default=800)
    ap.add_argument("--frames", type=int, default=8)
    ap.add_argument("--scene", default="table_clock_plant")
    ap.add_argument("--hdr", default=None, help="Radiance .hdr environment (default: the synthetic room.hdr)")
    ap.add_argument("--view", default="final_pic", choices=Renderer.VIEWS)
    ap.add_argument("--orbit", type=float, default=0.0, help="degrees per frame (moving camera)")
    ap.add_argument("--mode", default="fast", choices=("fast", "reference"))
    ap.add_argument("--png", default="render.png")
    ap.add_argument("--pfm", default=None, help="also write the selected plane's floats")
    ap.add_argument("--device", type=int, default=0)
    a = ap.parse_args(argv)

    scene = build_scene(a.scene)
    if a.hdr:
        from .scene import hdr_cache
        scene.hdr = load_hdr(a.hdr)
        scene.cache = hdr_cache(scene.hdr)
    gl.init(a.device)
    try:
        r = Renderer(scene, a.width, a.height, parameter_config(), mode=a.mode, run_taa=True, run_output=True)
        r.set_view(a.view)
        for _ in range(a.frames):
            if a.orbit:
                r.camera.orbit(a.orbit, 0.0)
            r.frame()
        gl.sync()
        write_png(a.png, gl.readback(r.planes()["output"]))
        if a.pfm:
            write_pfm(a.pfm, gl.readback(r._view_plane(r.frame_index - 1)))
        r.close()
    finally:
        gl.shutdown()
    print(f"wrote {a.png}" + (f" and {a.pfm}" if a.pfm else ""))
    return 0


if __name__ == "__main__":
    raise SystemExit(main())
