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
    if not variant:
        _check_provenance(name, autobuild and not os.environ.get("NFDP_NO_AUTOBUILD"))
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


class StaleExtensionError(ImportError):
    """The built module's embedded source digest is not the digest of the sources in the tree."""


def _check_provenance(name: str, autobuild: bool) -> None:
    """Refuse (or, when building is allowed, rebuild) a module not built from the sources at hand.

    The digest compiled into the ``.so`` (native/build.py ``source_digest``) must equal the digest
    of csrc/ as it is now.  Without csrc/ (an installed package) there is nothing to compare."""
    from . import build

    spec = build.MODULES[name]
    if not all((spec["dir"] / s).exists() for s in spec["sources"]):
        return
    so = _HERE / f"{name}{build.EXT}"
    if not so.exists():
        return                       # the import below builds it (or fails loudly)
    want = build.source_digest(name)
    have = build.embedded_digest(so)
    if have == want:
        return
    if autobuild:
        build.build_module(name)
        if build.embedded_digest(so) == want:
            return
    raise StaleExtensionError(
        f"{so.name} was built from other sources (embedded digest {have or 'none'}, csrc/ digest {want[:16]}...): "
        f"rebuild with `python -m dpu_operator_amd.native.build`")


def provenance() -> dict:
    """{module: {"built": embedded digest, "sources": digest of csrc/ now}} (bench / reports)."""
    from . import build

    out = {}
    for name in build.MODULES:
        so = _HERE / f"{name}{build.EXT}"
        out[name] = {"built": build.embedded_digest(so), "sources": build.source_digest(name)}
    return out


def nfdp():
    """The `_nfdp` HIP extension (raises if it cannot be built/loaded)."""
    return _load("_nfdp")


def agent():
    """The `_agent` C++ extension (control mailbox + control-plane agent)."""
    return _load("_agent")
