"""ptsvgf — MI355X-native path tracing + SVGF behind the reference's GL plumbing API.

Layout:
  gl        Python mirror of RenderPass / Rasterize_RenderPass / getShaderProgram /
            getTextureRGB32F (Utils/render_pass.h, shader.h, help_func.h) over the C ABI
  scene     reference layer L1 (readObj, buildBVHwithSAH, encodings, HDR cache) on
            the native host library, plus synthetic stand-ins for missing assets
  camera    Camera / parameter_config / glm helpers (Utils/camera.h, gui_config.h)
  renderer  headless main.cpp (startup + frame loop), reference and fast drivers
  dist      screen-band sharding across GPUs with halo exchange (torch.distributed)
"""
from ._lib import PtError  # noqa: F401

__all__ = ["PtError"]
