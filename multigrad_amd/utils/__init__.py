"""Utilities: gradient-descent helpers, PRNG keys, checkpoints, metrics, profiling."""
from . import util  # noqa: F401
from .util import GradDescentResult, latin_hypercube_sampler, scatter_nd, simple_grad_descent
from .random import PRNGKey, init_randkey, gen_new_key

__all__ = ["util", "GradDescentResult", "latin_hypercube_sampler", "scatter_nd",
           "simple_grad_descent", "PRNGKey", "init_randkey", "gen_new_key"]
