"""Checkpoint / resume.

Reference format (optimizer.py:211, 691-715, 244-272, 294-315): a weights-only ``torch.save(state_dict)`` per
iteration named ``model_%09d.pt`` under ``log_dir``; resume = lexicographically latest ``*.pt`` with the iteration
parsed by ``(\\d+)(?=.pt)``. We keep that file unchanged (so a dotaclient agent can load our models with
``strict=True``) and add a sidecar ``trainer_state_%09d.pt`` holding what the reference loses on restart: Adam moments
and per-parameter step counts, running reward statistics, RNG states and the iteration counter. Writes are atomic
(temp file + rename) so a crash never leaves a truncated checkpoint. Fixes the reference's broken local resume
(§2.10-5) and worker/master iteration skew (§2.10-7: every rank resumes from the same iteration, broadcast by rank 0).
"""
from __future__ import annotations

import os
import re
from typing import Optional, Tuple

import torch

MODEL_FILENAME_FMT = 'model_%09d.pt'
STATE_FILENAME_FMT = 'trainer_state_%09d.pt'
_ITER_RE = re.compile(r'(\d+)(?=\.pt)')


def iteration_from_model_filename(filename: str) -> int:
    return int(_ITER_RE.search(os.path.basename(filename)).group(0))


def _atomic_save(obj, path: str):
    tmp = path + '.tmp'
    torch.save(obj, tmp)
    os.replace(tmp, path)


def save_model(state_dict, log_dir: str, version: int) -> Tuple[str, bytes]:
    """Write ``model_%09d.pt``; returns (path, serialized bytes) so the caller can also publish the bytes."""
    import io
    buf = io.BytesIO()
    torch.save({k: v.detach().cpu() for k, v in state_dict.items()}, buf)
    data = buf.getvalue()
    return write_model_bytes(data, log_dir, version), data


def write_model_bytes(data: bytes, log_dir: str, version: int) -> str:
    """Atomically write already-serialised ``model_%09d.pt`` bytes (tmp file + rename)."""
    os.makedirs(log_dir, exist_ok=True)
    path = os.path.join(log_dir, MODEL_FILENAME_FMT % version)
    tmp = path + '.tmp'
    with open(tmp, 'wb') as f:
        f.write(data)
    os.replace(tmp, path)
    return path


def save_trainer_state(state, log_dir: str, version: int) -> str:
    path = os.path.join(log_dir, STATE_FILENAME_FMT % version)
    _atomic_save(state, path)
    return path


def latest_model(log_dir: str) -> Optional[str]:
    if not log_dir or not os.path.isdir(log_dir):
        return None
    fns = sorted(f for f in os.listdir(log_dir) if f.startswith('model_') and f.endswith('.pt'))
    return os.path.join(log_dir, fns[-1]) if fns else None


def load_model_file(path: str):
    """Load a reference-format (weights-only) checkpoint safely."""
    return torch.load(path, map_location='cpu', weights_only=True)


def load_trainer_state(log_dir: str, version: int):
    path = os.path.join(log_dir, STATE_FILENAME_FMT % version)
    if not os.path.exists(path):
        return None
    return torch.load(path, map_location='cpu', weights_only=True)


def prune(log_dir: str, keep: int):
    """Keep the newest ``keep`` checkpoints (0 = keep everything, the reference's behaviour)."""
    if keep <= 0:
        return
    for prefix in ('model_', 'trainer_state_'):
        fns = sorted(f for f in os.listdir(log_dir) if f.startswith(prefix) and f.endswith('.pt'))
        for f in fns[:-keep]:
            os.remove(os.path.join(log_dir, f))
