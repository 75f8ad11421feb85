"""multigrad_amd -- an MI355X-native distributed-gradient fitting engine.

Same public API as AlanPearl/multigrad (reference ``multigrad/__init__.py:1-9``):
``OnePointModel``, ``OnePointGroup``, ``reduce_sum``, ``split_subcomms``,
``split_subcomms_by_node``, ``util`` and ``__version__``; plus ``adam``/``bfgs`` optimizer
modules, the communicator layer and the fused device engine.
"""
from ._version import __version__  # noqa: F401
from .models.onepoint import OnePointModel, OnePointGroup
from .parallel.subcomm import reduce_sum, split_subcomms, split_subcomms_by_node
from .parallel.comm import get_world_comm, init_distributed
from .utils import util
from . import parallel
from .optim import adam, bfgs

__all__ = ["OnePointModel", "OnePointGroup", "reduce_sum", "split_subcomms",
           "split_subcomms_by_node", "util", "adam", "bfgs", "get_world_comm",
           "init_distributed", "__version__"]


def __getattr__(name):
    # COMM / RANK / N_RANKS module globals of the reference, resolved lazily so that
    # importing the package never touches the launcher or the GPU.
    if name == "COMM":
        return get_world_comm()
    if name == "RANK":
        return get_world_comm().rank
    if name == "N_RANKS":
        return get_world_comm().size
    raise AttributeError(name)
