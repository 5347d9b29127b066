"""lighthouse2_amd - MI355X-native wavefront path-tracing render core for Lighthouse 2.

The product is the shared library libRenderCore_MI355X.so (C++ host + gfx950 HIP kernels) that
exports the reference RenderCore C-ABI (CreateCore / DestroyCore / CoreAPI_Base vtable) plus a flat
extern "C" mirror (include/lh2_rendercore.h).  This package holds its Python binding (core.py),
the ABI mirror (abi.py), synthetic scenes for the benchmark configurations (scene.py) and the
multi-GPU tile partition (parallel.py).
"""
from . import abi  # noqa: F401
from .core import RenderCore, CoreError, load_library  # noqa: F401

__all__ = ["abi", "RenderCore", "CoreError", "load_library"]
