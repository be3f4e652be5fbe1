"""Identity of a kernel's machine code inside a HIP library, for tying a committed PMC profile to the library bench.py
times.

A rebuild of the same sources does not give the same .so bytes (the offload bundles differ run to run), so the whole
file's hash cannot say whether two builds carry the same kernel. This reads the gfx950 code objects out of the
library's .hip_fatbin clang offload bundles (uncompressed: hipcc's default here), and hashes the instruction bytes of
every function symbol whose name contains the pattern, in name order: equal for rebuilds, different as soon as the
kernel's code changes.

usage: python tools/kernel_hash.py LIB [PATTERN]   (default pattern: atrous_tile_kernel)
"""
from __future__ import annotations

import hashlib
import struct
import sys

BUNDLE_MAGIC = b"__CLANG_OFFLOAD_BUNDLE__"


def _sections(elf: bytes):
    """{name: (offset, size, addr)} of an ELF64 little-endian image."""
    if elf[:4] != b"\x7fELF" or elf[4] != 2:
        raise ValueError("not an ELF64 image")
    shoff, = struct.unpack_from("<Q", elf, 0x28)
    shentsize, shnum, shstrndx = struct.unpack_from("<HHH", elf, 0x3A)
    hdrs = []
    for i in range(shnum):
        name, typ, flags, addr, off, size = struct.unpack_from("<IIQQQQ", elf, shoff + i * shentsize)
        link, = struct.unpack_from("<I", elf, shoff + i * shentsize + 0x28)
        hdrs.append((name, typ, addr, off, size, link))
    stroff = hdrs[shstrndx][3]

    def cstr(base, o):
        e = elf.index(b"\0", base + o)
        return elf[base + o:e].decode()

    return {cstr(stroff, h[0]): h for h in hdrs}, hdrs, cstr


def _functions(elf: bytes):
    """(name, code bytes) of every FUNC symbol of a code object."""
    secs, hdrs, cstr = _sections(elf)
    if ".symtab" not in secs:
        return []
    _, _, _, off, size, link = secs[".symtab"]
    stroff = hdrs[link][3]
    out = []
    for k in range(size // 24):
        st_name, st_info, _, st_shndx, st_value, st_size = struct.unpack_from("<IBBHQQ", elf, off + k * 24)
        if st_info & 0xF != 2 or st_size == 0 or st_shndx == 0 or st_shndx >= len(hdrs):
            continue
        _, _, saddr, soff, _, _ = hdrs[st_shndx]
        start = soff + (st_value - saddr)
        out.append((cstr(stroff, st_name), elf[start:start + st_size]))
    return out


def code_objects(lib: bytes, arch: str = "gfx950"):
    """The device code objects for `arch` in every offload bundle of the library's .hip_fatbin section."""
    secs, _, _ = _sections(lib)
    if ".hip_fatbin" not in secs:
        return []
    _, _, _, off, size, _ = secs[".hip_fatbin"]
    fat = lib[off:off + size]
    objs, pos = [], 0
    while True:
        pos = fat.find(BUNDLE_MAGIC, pos)
        if pos < 0:
            break
        n, = struct.unpack_from("<Q", fat, pos + 24)
        p = pos + 32
        for _ in range(n):
            eoff, esize, tlen = struct.unpack_from("<QQQ", fat, p)
            triple = fat[p + 24:p + 24 + tlen].decode(errors="replace")
            p += 24 + tlen
            if arch in triple:
                objs.append(fat[pos + eoff:pos + eoff + esize])
        pos += 32
    return objs


def kernel_code_hash(path: str, pattern: str = "atrous_tile_kernel") -> str | None:
    """sha256 over (name, instruction bytes) of the matching functions in name order; None if none matches."""
    with open(path, "rb") as f:
        lib = f.read()
    funcs = sorted((n, c) for co in code_objects(lib) for n, c in _functions(co) if pattern in n)
    if not funcs:
        return None
    h = hashlib.sha256()
    for n, c in funcs:
        h.update(n.encode() + b"\0" + c)
    return h.hexdigest()


if __name__ == "__main__":
    print(kernel_code_hash(sys.argv[1], sys.argv[2] if len(sys.argv) > 2 else "atrous_tile_kernel"))
