"""Loader for the native extension.

Device (HIP) tensors always go through ``_C``; if the extension cannot be imported while
a GPU op is requested we raise instead of silently falling back to eager PyTorch, so a
GPU run can never "pass" on a fallback path.  Set ``MULTIGRAD_AUTOBUILD=1`` to compile
on first use.
"""
from __future__ import annotations

import importlib
import os

_EXT = None
_ERR = None


def ext():
    """The ``multigrad_amd._C`` module (raises with a build hint if unavailable)."""
    global _EXT, _ERR
    if _EXT is not None:
        return _EXT
    try:
        import torch  # noqa: F401  (loads libamdhip64/libtorch before _C)
        so = os.environ.get("MULTIGRAD_EXT_SO")
        if so:  # an A/B build variant (tools/build_variant.sh) in place of the in-tree _C.so
            import sys
            from importlib import util as ilu
            spec = ilu.spec_from_file_location("multigrad_amd._C", so)
            mod = ilu.module_from_spec(spec)
            spec.loader.exec_module(mod)
            sys.modules["multigrad_amd._C"] = mod
            _EXT = mod
            return _EXT
        _EXT = importlib.import_module("multigrad_amd._C")
        return _EXT
    except ImportError as e:  # pragma: no cover - depends on build state
        _ERR = e
        if os.environ.get("MULTIGRAD_AUTOBUILD", "0") == "1":
            from . import build
            build.build()
            _EXT = importlib.import_module("multigrad_amd._C")
            return _EXT
        raise ImportError(
            "multigrad_amd native extension (_C.so) is not built; run "
            "`python -m multigrad_amd.ops.build` (gfx950) -- original error: " + repr(e)) from e


def available() -> bool:
    try:
        ext()
        return True
    except ImportError:
        return False
