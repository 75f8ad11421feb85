"""Optimizers: fixed-step GD (utils.util), Adam (fused HIP update), L-BFGS-B (host scipy)
and device L-BFGS with all-reduced dot products."""
from . import adam, bfgs, transforms  # noqa: F401
from .adam import Adam, run_adam, run_adam_unbounded
from .bfgs import run_bfgs

__all__ = ["adam", "bfgs", "transforms", "Adam", "run_adam", "run_adam_unbounded", "run_bfgs"]
