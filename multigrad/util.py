"""``multigrad.util`` -> :mod:`multigrad_amd.utils.util`."""
from multigrad_amd.utils.util import *  # noqa: F401,F403
from multigrad_amd.utils.util import (GradDescentResult, latin_hypercube_sampler,  # noqa: F401
                                      scatter_nd, simple_grad_descent)
