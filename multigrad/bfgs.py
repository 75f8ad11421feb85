"""``multigrad.bfgs`` -> :mod:`multigrad_amd.optim.bfgs`."""
from multigrad_amd.optim.bfgs import run_bfgs  # noqa: F401
from multigrad_amd.optim.adam import init_randkey  # noqa: F401
