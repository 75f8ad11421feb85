"""``multigrad.multigrad`` -> the model and communicator layers."""
from multigrad_amd.models.onepoint import OnePointModel, OnePointGroup  # noqa: F401
from multigrad_amd.parallel.subcomm import (reduce_sum, split_subcomms,  # noqa: F401
                                            split_subcomms_by_node)
from multigrad_amd.utils import util  # noqa: F401
from multigrad_amd.optim.adam import run_adam  # noqa: F401
from multigrad_amd.optim.bfgs import run_bfgs  # noqa: F401


def __getattr__(name):
    if name in ("COMM", "RANK", "N_RANKS"):
        import multigrad_amd
        return getattr(multigrad_amd, name)
    raise AttributeError(name)

from multigrad_amd.utils.progress import (trange_no_tqdm, make_trange_with_tqdm,  # noqa: E402,F401
                                          make_module_trange)

trange_with_tqdm = make_trange_with_tqdm(None)
trange = make_module_trange(None)
