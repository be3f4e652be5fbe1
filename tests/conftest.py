import os
import sys

import pytest

REPO = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(REPO, "path-tracing-svgf_amd")
for p in (PKG, os.path.join(REPO, "tests")):
    if p not in sys.path:
        sys.path.insert(0, p)


def pytest_configure(config):
    config.addinivalue_line("markers", "gpu: needs a real MI355X (runs through the HIP kernels)")


@pytest.fixture(scope="session")
def gpu():
    """Initialise the HIP library once per session (device 0)."""
    from ptsvgf import gl

    gl.init(0)
    yield gl
    gl.shutdown()


@pytest.fixture(scope="session")
def scene_small():
    from ptsvgf.scene import build_scene

    return build_scene("table_clock_plant", hdr_size=(256, 128), plant_leaves=40)


@pytest.fixture(scope="session")
def scene_cornell():
    from ptsvgf.scene import build_scene

    return build_scene("cornell_teapot", hdr_size=(128, 64))
