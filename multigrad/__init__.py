"""Drop-in import name for code written against AlanPearl/multigrad.

``import multigrad`` gives the MI355X-native implementation in :mod:`multigrad_amd`
(same public names: ``OnePointModel``, ``OnePointGroup``, ``reduce_sum``,
``split_subcomms``, ``split_subcomms_by_node``, ``util``, ``__version__``; submodules
``multigrad.util``, ``multigrad.adam``, ``multigrad.bfgs``, ``multigrad.mpi4jax``).
User models are written with PyTorch ops instead of jax.numpy.
"""
from multigrad_amd import (OnePointModel, OnePointGroup, reduce_sum, split_subcomms,  # noqa: F401
                           split_subcomms_by_node, __version__)
from . import util, adam, bfgs, mpi4jax, multigrad  # noqa: F401

__all__ = ["OnePointModel", "OnePointGroup", "reduce_sum", "split_subcomms",
           "split_subcomms_by_node", "util"]


def __getattr__(name):
    import multigrad_amd
    return getattr(multigrad_amd, name)
