"""``multigrad.util`` -> :mod:`multigrad_amd.utils.util`."""
from multigrad_amd.utils.util import *  # noqa: F401,F403
from multigrad_amd.utils.util import (GradDescentResult, latin_hypercube_sampler,  # noqa: F401
                                      scatter_nd, simple_grad_descent)

from multigrad_amd.utils.progress import (trange_no_tqdm, make_trange_with_tqdm,  # noqa: E402,F401
                                          make_module_trange)

trange_with_tqdm = make_trange_with_tqdm(None)
trange = make_module_trange(None)
