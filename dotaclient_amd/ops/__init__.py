"""Native gfx950 HIP kernels (``_C``) and their python-facing wrappers.

``available()`` tells whether the compiled extension can be used (it is built in-tree by
``python -m dotaclient_amd.ops.build`` / ``__graft_entry__.build()``). On a GPU host the framework refuses to fall
back silently: :func:`require` raises if the extension is missing or fails to load, so a GPU run can never pass on an
eager-PyTorch path by accident.
"""
from __future__ import annotations

import importlib
import os

_C = None
_ERR = None


def _load():
    global _C, _ERR
    if _C is not None or _ERR is not None:
        return _C
    try:
        _C = importlib.import_module('dotaclient_amd.ops._C')
    except Exception as e:  # pragma: no cover - depends on build state
        _ERR = e
    return _C


def available() -> bool:
    import torch
    return torch.cuda.is_available() and _load() is not None


def require():
    """Return the extension module or raise loudly (never silently fall back on a GPU host)."""
    m = _load()
    if m is None:
        raise RuntimeError(
            'dotaclient_amd HIP extension not available '
            f'({_ERR!r}); build it with `python -m dotaclient_amd.ops.build`')
    return m


def extension_path():
    m = _load()
    return getattr(m, '__file__', None) if m is not None else None
