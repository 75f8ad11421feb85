"""Set-up tracing to stderr (``MULTIGRAD_TRACE=1``): one time-stamped line per phase of the
collective set-up paths (re-partition, engine setup, peer-memory connects, autotune), so a
multi-rank run that stalls shows where each rank is.  Off by default (no cost)."""
from __future__ import annotations

import os
import sys
import time

__all__ = ["trace", "tracing"]

_T0 = time.perf_counter()


def tracing() -> bool:
    return os.environ.get("MULTIGRAD_TRACE", "0").lower() not in ("", "0", "false", "off", "no")


def trace(msg: str) -> None:
    if not tracing():
        return
    r = os.environ.get("RANK", "0")
    sys.stderr.write(f"[multigrad t={time.perf_counter() - _T0:9.3f}s rank={r}] {msg}\n")
    sys.stderr.flush()
