"""Reference citations (``file:line`` / ``file:a-b``) in the product, oracle, tests and docs point inside the cited
reference file, and the anchors the oracle's fidelity rests on name the function they claim.

Runs where the reference tree is present (this container); skipped on the GPU box, which has no /root/reference.
The reference is read as text only."""
import os
import re
from collections import defaultdict

import pytest

REF = "/root/reference"
REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
SCAN = ["path-tracing-svgf_amd", "oracle", "include", "tests", "tools", "bench.py", "__graft_entry__.py", "DESIGN.md",
        "INTEGRATION.md", "README.md"]
CITE = re.compile(r"([A-Za-z_][\w.\-/]*\.(?:frag|vert|h|cpp|hpp|c))(:\d+(?:-\d+)?(?:,\s*:?\d+(?:-\d+)?)*)")
# (file, line, text that line must contain): the functions SURVEY.md §8(a) maps the hot path onto
ANCHORS = [
    ("path_tracing.frag", 215, "hitTriangle"), ("path_tracing.frag", 275, "hitAABB"),
    ("path_tracing.frag", 298, "hitArray"), ("path_tracing.frag", 372, "hitBVH"),
    ("path_tracing.frag", 438, "wang_hash"), ("path_tracing.frag", 620, "BRDF_Evaluate"),
    ("path_tracing.frag", 787, "SampleHdr"), ("path_tracing.frag", 948, "shade"),
    ("path_tracing.frag", 1056, "main"), ("path_tracing.frag", 1117, "lastFrame"),
    ("svgf_reproject.frag", 162, "main"), ("svgf_variance.frag", 23, "computeWeight"),
    ("svgf_variance.frag", 39, "main"), ("svgf_Atrous.frag", 20, "computeVarianceCenter"),
    ("svgf_Atrous.frag", 43, "computeWeight"), ("svgf_Atrous.frag", 61, "main"),
    ("svgf_modulate.frag", 18, "main"), ("hdr_compute.h", 5, "calculateHdrCache"),
    ("hdrloader.cpp", 118, "decrunch"), ("hdrloader.cpp", 161, "oldDecrunch"),
]

pytestmark = pytest.mark.skipif(not os.path.isdir(REF), reason="reference tree not present (GPU box)")


def _ref_files():
    files = defaultdict(list)
    for dp, _, fn in os.walk(REF):
        if "/.git" in dp:
            continue
        for f in fn:
            files[f].append(os.path.join(dp, f))
    return files


def _lines(path):
    """Lines as editors number them (split on LF only: the reference's GBK comments hold bytes str.splitlines
    would also break on)."""
    with open(path, "rb") as fh:
        data = fh.read()
    lines = data.split(b"\n")
    if lines and lines[-1] == b"":
        lines.pop()
    return [ln.decode("latin-1") for ln in lines]


def test_citations_lie_inside_the_cited_files():
    files = _ref_files()
    nlines = {name: max(len(_lines(p)) for p in paths) for name, paths in files.items()}
    bad, seen = [], 0
    for root in SCAN:
        top = os.path.join(REPO, root)
        paths = [top] if os.path.isfile(top) else [os.path.join(dp, f) for dp, _, fn in os.walk(top) for f in fn]
        for p in paths:
            if "__pycache__" in p or not re.search(r"\.(py|hip|h|cpp|md|inc|sh)$", p):
                continue
            with open(p, errors="ignore") as fh:
                for ln, line in enumerate(fh, 1):
                    for m in CITE.finditer(line):
                        name = os.path.basename(m.group(1))
                        if name not in nlines:
                            continue
                        for a, b in re.findall(r"(\d+)(?:-(\d+))?", m.group(2)):
                            a, b = int(a), int(b or a)
                            seen += 1
                            if not (1 <= a <= b <= nlines[name]):
                                bad.append(f"{os.path.relpath(p, REPO)}:{ln}: {m.group(0)} ({name} has {nlines[name]})")
    assert seen > 200, seen  # the scan really finds the citations
    assert not bad, "\n".join(bad)


@pytest.mark.parametrize("name,line,text", ANCHORS)
def test_anchor_lines_name_their_function(name, line, text):
    paths = _ref_files()[name]
    assert paths, name
    assert any(text in _lines(p)[line - 1] for p in paths), (name, line, text)
