"""``multigrad.adam`` -> :mod:`multigrad_amd.optim.adam`."""
from multigrad_amd.optim.adam import (run_adam, run_adam_unbounded, apply_transforms,  # noqa: F401
                                      apply_inverse_transforms, transform, inverse_transform,
                                      init_randkey, gen_new_key, Adam)
