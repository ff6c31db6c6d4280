"""Process-group helpers (reference optimizer.py:41-49, 203-206, 718-726).

One process per GPU. On ROCm the ``nccl`` backend *is* RCCL (collectives over xGMI inside a node); ``gloo`` is used
for CPU runs and multi-process CPU tests. Rendezvous is env:// (RANK / WORLD_SIZE / MASTER_ADDR / MASTER_PORT, as
set by ``torch.distributed.run`` or the Kubeflow PyTorch operator).
"""
from __future__ import annotations

import logging
import os
from datetime import timedelta

import torch
import torch.distributed as dist

logger = logging.getLogger(__name__)


def is_distributed() -> bool:
    return dist.is_available() and dist.is_initialized()


def get_rank() -> int:
    return dist.get_rank() if is_distributed() else 0


def get_world_size() -> int:
    return dist.get_world_size() if is_distributed() else 1


def is_master() -> bool:
    return get_rank() == 0


def local_rank() -> int:
    return int(os.environ.get('LOCAL_RANK', 0))


def default_backend(device: torch.device | str | None = None) -> str:
    dev = torch.device(device) if device is not None else None
    if dev is not None and dev.type == 'cuda':
        return 'nccl'   # RCCL on ROCm
    return 'gloo'


def init_distribution(backend: str | None = None, device=None, timeout_s: float = 600.0) -> bool:
    """Initialise the default process group from env vars; no-op when WORLD_SIZE < 2 (optimizer.py:718-726)."""
    world_size = int(os.environ.get('WORLD_SIZE', '1'))
    if world_size < 2:
        logger.info('skipping distribution: world size %d', world_size)
        return False
    if is_distributed():
        return True
    backend = backend or default_backend(device)
    kwargs = {}
    if backend == 'nccl' and device is not None:
        kwargs['device_id'] = torch.device(device)
    dist.init_process_group(backend=backend, timeout=timedelta(seconds=timeout_s), **kwargs)
    logger.info('distribution initialised: backend=%s rank=%d/%d', backend, get_rank(), world_size)
    return True


def all_gather_cat(t: torch.Tensor) -> torch.Tensor:
    """Gather a tensor from every rank and concatenate (reference optimizer.py:203-206, unused there)."""
    if not is_distributed():
        return t
    out = [torch.empty_like(t) for _ in range(get_world_size())]
    dist.all_gather(out, t)
    return torch.cat(out)


def barrier():
    if is_distributed():
        dist.barrier()


def destroy():
    if is_distributed():
        dist.destroy_process_group()
