"""``multigrad.util`` -> :mod:`multigrad_amd.utils.util`."""
from multigrad_amd.utils.util import *  # noqa: F401,F403
from multigrad_amd.utils.util import (GradDescentResult, latin_hypercube_sampler,  # noqa: F401
                                      scatter_nd, simple_grad_descent)

from multigrad_amd.utils.progress import (trange_no_tqdm, make_trange_with_tqdm,  # noqa: E402,F401
                                          make_module_trange)

trange_with_tqdm = make_trange_with_tqdm(None)
trange = make_module_trange(None)


def __getattr__(name):
    # the reference's import-time MPI globals (COMM, RANK, N_RANKS in every module)
    if name in ("COMM", "RANK", "N_RANKS"):
        import multigrad_amd
        return getattr(multigrad_amd, name)
    raise AttributeError(name)
