"""Rank-0 progress bars (reference ``multigrad/multigrad.py:29-45``, ``util.py:27-47``).

Bars are shown only on world rank 0 and only when tqdm is importable; set
``MULTIGRAD_PROGRESS=0`` to silence them (benchmarks do).
"""
from __future__ import annotations

import os

__all__ = ["trange", "progress_enabled"]


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
