"""Loader for the in-tree native extensions.

``nfdp()`` returns the HIP data-plane module, ``agent()`` the C++ control-mailbox/agent module.
Both are built in-tree by :mod:`dpu_operator_amd.native.build` (``__graft_entry__.build()``).
There is deliberately NO Python fallback for the GPU path: when a GPU is present and the
extension is missing or stale, importing it raises, so a run can never silently measure an
eager/PyTorch stand-in.  The CPU oracle lives inside the same extension.
"""
from __future__ import annotations

import importlib
import os
import sys
from pathlib import Path

_HERE = Path(__file__).resolve().parent
_cache: dict[str, object] = {}


def _load(name: str, autobuild: bool = True):
    if name in _cache:
        return _cache[name]
    if str(_HERE) not in sys.path:
        sys.path.insert(0, str(_HERE))
    variant = os.environ.get("NFDP_EXT_DIR")  # build-flag experiments (native/build.py NFDP_BUILD_OUT)
    if variant and sys.path[0] != variant:
        sys.path.insert(0, variant)
    # torch first: it loads its ROCm runtime libraries into the global symbol scope, and the
    # extension's HIP runtime must bind to that same HSA runtime.  Loaded the other way round the
    # process ends up with two HSA runtimes and the extension's sees no device.
    try:
        import torch  # noqa: F401
    except ImportError:
        pass
    try:
        mod = importlib.import_module(name)
    except ImportError:
        if not autobuild or os.environ.get("NFDP_NO_AUTOBUILD"):
            raise
        from . import build

        build.build_module(name)
        mod = importlib.import_module(name)
    _cache[name] = mod
    return mod


def nfdp():
    """The `_nfdp` HIP extension (raises if it cannot be built/loaded)."""
    return _load("_nfdp")


def agent():
    """The `_agent` C++ extension (control mailbox + control-plane agent)."""
    return _load("_agent")
