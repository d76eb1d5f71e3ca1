"""Loader for the in-tree HIP extension ``dmlab/_C*.so``.

Policy: on a machine with a GPU the native extension is REQUIRED — every op that
runs on a HIP device calls :func:`lib` and fails loudly if the extension is not
built, so a test can never pass on a silent eager-PyTorch fallback.  CPU tensors
take the explicit PyTorch reference path (the numerics oracle), never this
module.

Identity: the library carries the sha256 of the ``csrc/`` tree it was built from
(:func:`dmlab._build.source_hash`).  Before importing it the loader compares that stamp
with the current tree and refuses a stale or unstamped ``.so`` -- a prebuilt binary pushed
with newer sources would otherwise validate old kernels -- or, under
``DMLAB_AUTOBUILD=1``, rebuilds it first.  ``DMLAB_SKIP_HASH_CHECK=1`` disables the check
(a tree without ``csrc/``).
"""
from __future__ import annotations

import importlib
import os
import threading

import torch  # noqa: F401  (must be imported before _C: it owns the HIP runtime)

_lock = threading.Lock()
_mod = None
_err: Exception | None = None


class StaleExtensionError(RuntimeError):
    pass


def check_stamp(so_path, tree_hash=None):
    """Raise :class:`StaleExtensionError` unless the library at ``so_path`` carries the
    source hash of the current ``csrc/`` tree (``tree_hash``, default: computed now)."""
    from dmlab import _build

    tree = tree_hash or _build.source_hash()
    emb = _build.embedded_hash(so_path)
    if emb != tree:
        raise StaleExtensionError(
            f"dmlab native extension {so_path} was built from other sources "
            f"(stamp {emb or 'missing'}, csrc/ tree {tree}): rebuild it with "
            "`python -m dmlab._build` or set DMLAB_AUTOBUILD=1")
    return tree


def _verify_or_build():
    from dmlab import _build

    if os.environ.get("DMLAB_SKIP_HASH_CHECK", "0") == "1" or not _build.CSRC.is_dir():
        return
    try:
        check_stamp(_build.ext_path())
    except StaleExtensionError:
        if os.environ.get("DMLAB_AUTOBUILD", "0") != "1":
            raise
        _build.build()
        check_stamp(_build.ext_path())


def _load():
    global _mod, _err
    with _lock:
        if _mod is not None or _err is not None:
            return
        try:
            _verify_or_build()
            _mod = importlib.import_module("dmlab._C")
        except StaleExtensionError as e:
            _err = e
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
    if isinstance(_err, StaleExtensionError):
        raise _err
    if _mod is None:
        raise RuntimeError(
            "dmlab native extension (dmlab/_C*.so) is not built: run "
            "`python -m dmlab._build` (hipcc --offload-arch=gfx950). "
            f"Import error: {_err!r}")
    if os.environ.get("DMLAB_SYNC_DEBUG", "0") == "1":
        return _SyncDebug(_mod)
    return _mod
