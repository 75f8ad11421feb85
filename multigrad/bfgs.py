"""``multigrad.bfgs`` -> :mod:`multigrad_amd.optim.bfgs`."""
from multigrad_amd.optim.bfgs import run_bfgs  # noqa: F401
from multigrad_amd.optim.adam import init_randkey  # noqa: F401

from multigrad_amd.utils.progress import (trange_no_tqdm, make_trange_with_tqdm,  # noqa: E402,F401
                                          make_module_trange)

trange_with_tqdm = make_trange_with_tqdm('BFGS Gradient Descent Progress')
bfgs_trange = make_module_trange('BFGS Gradient Descent Progress')


def __getattr__(name):
    # the reference's import-time MPI globals (COMM, RANK, N_RANKS in every module)
    if name in ("COMM", "RANK", "N_RANKS"):
        import multigrad_amd
        return getattr(multigrad_amd, name)
    raise AttributeError(name)
