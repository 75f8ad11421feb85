"""Model layer: the one-point model contract and the SMF model families."""
from .onepoint import OnePointModel, OnePointGroup

__all__ = ["OnePointModel", "OnePointGroup"]
