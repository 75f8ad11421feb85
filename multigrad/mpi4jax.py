"""``multigrad.mpi4jax`` -> :mod:`multigrad_amd.ingraph` (device-resident, HIP-graph GD)."""
from multigrad_amd.ingraph import distribute_data, reduce_sum, simple_grad_descent  # noqa: F401
