"""Rank-0 progress bars (reference ``multigrad/multigrad.py:29-45``, ``util.py:27-47``).

Bars are shown only on world rank 0 and only when tqdm is importable; set
``MULTIGRAD_PROGRESS=0`` to silence them (benchmarks do).
"""
from __future__ import annotations

import os

__all__ = ["trange", "progress_enabled", "trange_no_tqdm", "make_trange_with_tqdm", "make_module_trange"]


def progress_enabled() -> bool:
    if os.environ.get("MULTIGRAD_PROGRESS", "1").lower() in ("0", "false", "off", "no"):
        return False
    from ..parallel.comm import launcher_env
    if launcher_env()["rank"] != 0:
        return False
    try:
        import tqdm  # noqa: F401
    except ImportError:
        return False
    return True


def trange(n, desc=None, leave=None):
    if progress_enabled():
        from tqdm import auto as tqdm
        kw = {} if leave is None else {"leave": leave}
        return tqdm.trange(n, desc=desc, **kw)
    return range(n)


# Module-level helpers the reference defines in each of its modules (multigrad/adam.py:28-36,
# bfgs.py:21-29, multigrad.py:37-45, util.py:39-47): a plain range, a tqdm bar with the
# module's default title, and the module's pick between them.  Here the pick also honours
# the rank-0 / MULTIGRAD_PROGRESS policy of :func:`trange`.
def trange_no_tqdm(n, desc=None):
    return range(n)


def make_trange_with_tqdm(default_desc=None):
    def trange_with_tqdm(n, desc=default_desc):
        from tqdm import auto as tqdm
        return tqdm.trange(n, desc=desc)
    return trange_with_tqdm


def make_module_trange(default_desc=None):
    def module_trange(n, desc=default_desc):
        return trange(n, desc=desc)
    return module_trange
