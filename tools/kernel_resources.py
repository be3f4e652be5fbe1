"""Register / LDS / scratch use of the kernels in a HIP library (the code object's AMDGPU metadata notes), for the
occupancy arguments in DESIGN.md: python tools/kernel_resources.py LIB [PATTERN ...]"""
import os
import re
import subprocess
import sys
import tempfile

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from kernel_hash import code_objects  # noqa: E402

READOBJ = "/opt/rocm/lib/llvm/bin/llvm-readobj"


def resources(lib_path):
    with open(lib_path, "rb") as f:
        lib = f.read()
    out = {}
    for co in code_objects(lib):
        with tempfile.NamedTemporaryFile(suffix=".co") as t:
            t.write(co)
            t.flush()
            txt = subprocess.run([READOBJ, "--notes", t.name], capture_output=True, text=True).stdout
        for blk in re.split(r"\n\s*- \.agpr_count", txt)[1:]:
            name = re.search(r"\.name:\s+(\S+)", blk)
            if not name:
                continue
            g = lambda k: (re.search(rf"\.{k}:\s+(\d+)", blk) or [None, None])[1]  # noqa: E731
            out[name.group(1)] = dict(vgpr=g("vgpr_count"), sgpr=g("sgpr_count"), lds=g("group_segment_fixed_size"),
                                      scratch=g("private_segment_fixed_size"), spill_v=g("vgpr_spill_count"))
    return out


if __name__ == "__main__":
    res = resources(sys.argv[1])
    pats = sys.argv[2:] or [""]
    for n, r in sorted(res.items()):
        if any(p in n for p in pats):
            print(f"{r['vgpr']:>4} vgpr {r['sgpr']:>4} sgpr {r['lds']:>6} lds {r['scratch']:>5} scratch  {n[:110]}")
