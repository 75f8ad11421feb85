"""Counter-based, splittable PRNG keys (replacement for JAX threefry keys).

The reference threads ``jax.random`` keys through ``randkey`` kwargs
(``multigrad/adam.py:60-62,242-257``).  Here a key is an immutable 64-bit value; splits
are derived with SplitMix64 finalisers so that the *same* key sequence is produced on
every rank without communication (fixes SURVEY Q3, where master and workers derived
different per-step keys).  User models turn a key into a ``torch.Generator`` (Philox on
the GPU) with :meth:`PRNGKey.generator`.
"""
from __future__ import annotations

from dataclasses import dataclass

import numpy as np
import torch

__all__ = ["PRNGKey", "key", "split", "init_randkey", "gen_new_key", "is_key"]

_M64 = (1 << 64) - 1


def _mix64(z: int) -> int:
    z = (z + 0x9E3779B97F4A7C15) & _M64
    z = ((z ^ (z >> 30)) * 0xBF58476D1CE4E5B9) & _M64
    z = ((z ^ (z >> 27)) * 0x94D049BB133111EB) & _M64
    return z ^ (z >> 31)


@dataclass(frozen=True)
class PRNGKey:
    """An immutable 64-bit PRNG key."""

    value: int

    dtype = "prng_key"  # mirrors jax's typed-key dtype check in init_randkey

    def split(self, num: int = 2):
        """``num`` independent child keys (deterministic function of this key)."""
        return tuple(PRNGKey(_mix64(self.value ^ _mix64(i + 1))) for i in range(int(num)))

    def fold_in(self, data: int) -> "PRNGKey":
        return PRNGKey(_mix64(self.value ^ _mix64((int(data) & _M64) + 0x632BE59BD9B4E019)))

    @property
    def seed(self) -> int:
        """A non-negative 63-bit integer seed (for ``torch.Generator.manual_seed``)."""
        return self.value & ((1 << 63) - 1)

    def generator(self, device="cpu") -> torch.Generator:
        g = torch.Generator(device=device)
        g.manual_seed(self.seed)
        return g

    def numpy_rng(self) -> np.random.Generator:
        return np.random.default_rng(self.seed)

    def __int__(self) -> int:
        return self.value


def key(seed: int) -> PRNGKey:
    return PRNGKey(_mix64(int(seed) & _M64))


def split(k: PRNGKey, num: int = 2):
    return k.split(num)


def is_key(x) -> bool:
    return isinstance(x, PRNGKey)


def init_randkey(randkey) -> PRNGKey:
    """Check that ``randkey`` is a key or create one from an int (reference
    ``multigrad/adam.py:242-251``)."""
    if isinstance(randkey, (int, np.integer)) and not isinstance(randkey, bool):
        return key(int(randkey))
    msg = f"Invalid {type(randkey)=}: Must be int or PRNG Key"
    assert isinstance(randkey, PRNGKey), msg
    return randkey


def gen_new_key(randkey: PRNGKey) -> PRNGKey:
    """Split a key to generate a new one (reference ``multigrad/adam.py:254-257``)."""
    return randkey.split(1)[0]
