"""Loaders of the in-tree native extensions.

``host()`` returns the C++ host runtime (``_twtml_host``), building it on first
use if it is missing or stale (a few seconds of g++).  ``hip()`` returns the
MI355X engine (``_twtml_hip``).  It imports torch first so the HIP runtime and
RCCL that torch ships are the ones resolved for the extension (one runtime
per process), and it FAILS LOUDLY if the extension cannot be loaded — there is
no silent PyTorch fallback for the device path.
"""
from __future__ import annotations

import importlib
import os
import threading
from types import ModuleType
from typing import Optional

__all__ = ["host", "hip", "hip_available", "NativeUnavailable"]

_lock = threading.Lock()
_host: Optional[ModuleType] = None
_hip: Optional[ModuleType] = None


class NativeUnavailable(RuntimeError):
    pass


def host() -> ModuleType:
    global _host
    if _host is not None:
        return _host
    with _lock:
        if _host is None:
            from .. import _build
            # build only when missing (or forced): snapshots copied to another
            # machine may not preserve mtimes, so staleness is not trusted
            if os.environ.get("TWTML_REBUILD") == "1" or not os.path.exists(_build.HOST_SO):
                _build.build_host()
            try:
                _host = importlib.import_module("twitter_stream_ml_amd._twtml_host")
            except ImportError as e:  # pragma: no cover
                raise NativeUnavailable(f"_twtml_host not importable: {e}") from e
    return _host


def hip() -> ModuleType:
    global _hip
    if _hip is not None:
        return _hip
    with _lock:
        if _hip is None:
            import torch  # noqa: F401  (binds the HIP runtime/RCCL SONAMEs first)
            from .. import _build
            if os.environ.get("TWTML_REBUILD") == "1" or not os.path.exists(_build.HIP_SO):
                try:
                    _build.build_hip()
                except Exception as e:
                    if not os.path.exists(_build.HIP_SO):
                        raise NativeUnavailable(f"cannot build _twtml_hip: {e}") from e
            try:
                _hip = importlib.import_module("twitter_stream_ml_amd._twtml_hip")
            except ImportError as e:
                raise NativeUnavailable(
                    f"_twtml_hip (MI355X engine) not importable: {e}. "
                    "Run `python -m twitter_stream_ml_amd._build` first.") from e
    return _hip


def hip_available() -> bool:
    """True when a GPU is visible AND the HIP extension loads."""
    try:
        import torch
        if not torch.cuda.is_available():
            return False
        hip()
        return True
    except Exception:
        return False
