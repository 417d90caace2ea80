"""rtamd — MI355X-native trace path for 3169651074/real-time-gpu-ray-tracer.

The product is librtamd.so (C ABI in include/rt.h; hand-written HIP kernels for gfx950).
This package is the Python host mirror used by tests and benchmarks.
"""
from . import abi, scenes  # noqa: F401
from .renderer import Renderer  # noqa: F401

__all__ = ["abi", "scenes", "Renderer"]
