"""Native byte ops.

* ``_native``  (host C++, pybind11): OpenSSL-EVP hashing on a GIL-free thread pool and the
  zero-copy HTTP transport (splice / sendfile).
* ``_gpuhash`` (HIP, gfx950): batched SHA-1 piece verification on the MI355X.

Both are built in-tree by ``downloader_amd.ops.build`` (``__graft_entry__.build()``). A
missing extension is an error, not a silent fallback: ``native()`` / ``gpuhash()`` raise
with the build command in the message.
"""
from __future__ import annotations

import importlib
import os
from types import ModuleType
from typing import Optional

_native: Optional[ModuleType] = None
_gpu: Optional[ModuleType] = None


class NativeBuildMissing(ImportError):
    pass


def _load(name: str) -> ModuleType:
    try:
        return importlib.import_module(f"downloader_amd.ops.{name}")
    except ImportError as e:  # pragma: no cover - exercised only on a broken checkout
        raise NativeBuildMissing(
            f"native extension {name} is not built ({e}); run "
            f"`python -m downloader_amd.ops.build`") from e


def native() -> ModuleType:
    global _native
    if _native is None:
        try:
            _native = _load("_native")
        except NativeBuildMissing:
            if os.environ.get("STAGER_AUTOBUILD", "1") != "1":
                raise
            from . import build
            build.build_native(verbose=False)
            _native = _load("_native")
    return _native


def gpuhash() -> ModuleType:
    global _gpu
    if _gpu is None:
        _gpu = _load("_gpuhash")
    return _gpu


def gpu_available() -> bool:
    """True when the HIP module loads and sees at least one device."""
    if os.environ.get("STAGER_DISABLE_GPU") == "1":
        return False
    try:
        return gpuhash().device_count() > 0
    except Exception:
        return False
