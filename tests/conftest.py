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
def scene_nan():
    """Clock + a quad fan holding one zero-area face: readObj's normal accumulation turns it into
    NaN vertex normals on the neighbouring faces (obj_loader.h:101-110), exercising NaN paths."""
    import numpy as np

    from ptsvgf.scene import POINT_LIGHTS, Scene, SceneBuilder, env_map, hdr_cache, material, transform
    b = SceneBuilder()
    b.add_obj(os.path.join(REPO, "assets", "models", "clock.obj"), material(baseColor=(0.8, 0.6, 0.3)),
              transform(), True, 0)
    pos = np.array([[-0.6, -0.6, 0.2], [0.6, -0.6, 0.2], [0.6, 0.1, 0.2], [-0.6, 0.1, 0.2]], np.float32)
    idx = np.array([[0, 1, 2], [0, 2, 3], [0, 0, 2]], np.int32)  # last face has zero area
    b.add_mesh(pos, idx, material(baseColor=(0.3, 0.6, 0.8)), transform(), True, 1)
    b.build(8)
    tri, node, raster = b.encode()
    hdr = env_map(128, 64)
    return Scene("nan_probe", tri, node, raster, POINT_LIGHTS.copy(), hdr, hdr_cache(hdr), b.counts())


@pytest.fixture(scope="session")
def scene_cornell():
    from ptsvgf.scene import build_scene

    return build_scene("cornell_teapot", hdr_size=(128, 64))


@pytest.fixture(scope="session")
def scene_bench():
    """The bench scene at full size (150 leaves, 2048x1024 HDR)."""
    from ptsvgf.scene import build_scene

    return build_scene("table_clock_plant")
