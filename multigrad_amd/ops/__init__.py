"""Device ops: hand-written gfx950 HIP kernels (``csrc/``) behind thin Python wrappers."""
from ._ext import available, ext

__all__ = ["available", "ext"]
