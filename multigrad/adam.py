"""``multigrad.adam`` -> :mod:`multigrad_amd.optim.adam`."""
from multigrad_amd.optim.adam import (run_adam, run_adam_unbounded, apply_transforms,  # noqa: F401
                                      apply_inverse_transforms, transform, inverse_transform,
                                      init_randkey, gen_new_key, Adam)

from multigrad_amd.utils.progress import (trange_no_tqdm, make_trange_with_tqdm,  # noqa: E402,F401
                                          make_module_trange)

trange_with_tqdm = make_trange_with_tqdm('Adam Gradient Descent Progress')
adam_trange = make_module_trange('Adam Gradient Descent Progress')


def __getattr__(name):
    # the reference's import-time MPI globals (COMM, RANK, N_RANKS in every module)
    if name in ("COMM", "RANK", "N_RANKS"):
        import multigrad_amd
        return getattr(multigrad_amd, name)
    raise AttributeError(name)
