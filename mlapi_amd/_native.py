"""Loader for the native extension ``mlapi_amd._C``.

torch is imported FIRST: torch bundles its own libamdhip64 (same SONAME ``libamdhip64.so.7`` as
the system ROCm). Importing torch first makes our extension bind to the HIP runtime torch already
loaded, so kernels, streams and pointers are shared with torch tensors.

On a machine with a GPU the extension is mandatory: :func:`C` raises instead of silently falling
back to Python. Set ``MLAPI_AUTOBUILD=1`` to compile on first import when the ``.so`` is missing.
"""
from __future__ import annotations

import importlib
import os
import threading

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            import torch  # noqa: F401  (must precede _C: shared HIP runtime)
        except Exception:  # pragma: no cover - torch is part of the stack
            pass
        try:
            _mod = importlib.import_module("mlapi_amd._C")
        except ImportError as e:
            if os.environ.get("MLAPI_AUTOBUILD") == "1":
                from mlapi_amd import _build

                _build.build()
                _mod = importlib.import_module("mlapi_amd._C")
            else:
                _err = e


def available() -> bool:
    _load()
    return _mod is not None


def C():
    """Return the extension module or raise a clear error (never a silent fallback)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "mlapi_amd native extension is not built (run `python -m mlapi_amd._build`): " + repr(_err))
    return _mod


def gpu_count() -> int:
    if not available():
        return 0
    try:
        import torch

        return torch.cuda.device_count() if torch.cuda.is_available() else 0
    except Exception:  # pragma: no cover
        return 0
