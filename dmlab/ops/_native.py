"""Loader for the in-tree HIP extension ``dmlab/_C*.so``.

Policy: on a machine with a GPU the native extension is REQUIRED — every op that
runs on a HIP device calls :func:`lib` and fails loudly if the extension is not
built, so a test can never pass on a silent eager-PyTorch fallback.  CPU tensors
take the explicit PyTorch reference path (the numerics oracle), never this
module.
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must be imported before _C: it owns the HIP runtime)

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            _mod = importlib.import_module("dmlab._C")
        except Exception as e:  # pragma: no cover - depends on build state
            if os.environ.get("DMLAB_AUTOBUILD", "0") == "1":
                from dmlab import _build

                _build.build()
                _mod = importlib.import_module("dmlab._C")
            else:
                _err = e


def available() -> bool:
    _load()
    return _mod is not None


class _SyncDebug:
    """DMLAB_SYNC_DEBUG=1: synchronise after every native launch so a faulting kernel
    is reported at its own call site (stream-ordering / race debugging aid)."""

    def __init__(self, mod):
        self._mod = mod

    def __getattr__(self, name):
        f = getattr(self._mod, name)
        if not callable(f):
            return f

        def wrapped(*a, **kw):
            out = f(*a, **kw)
            try:
                torch.cuda.synchronize()
            except Exception as e:  # pragma: no cover - only on a faulting kernel
                raise RuntimeError(f"dmlab native op {name} failed: {e}") from e
            return out

        return wrapped


def lib():
    """Return the native module or raise (never silently fall back)."""
    _load()
    if _mod is None:
        raise RuntimeError(
            "dmlab native extension (dmlab/_C*.so) is not built: run "
            "`python -m dmlab._build` (hipcc --offload-arch=gfx950). "
            f"Import error: {_err!r}")
    if os.environ.get("DMLAB_SYNC_DEBUG", "0") == "1":
        return _SyncDebug(_mod)
    return _mod
