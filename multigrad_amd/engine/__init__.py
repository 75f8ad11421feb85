"""Execution engines: the fused device-resident optimizer loop (HIP graphs, streams)."""
from .fused import FusedAdamEngine

__all__ = ["FusedAdamEngine"]
