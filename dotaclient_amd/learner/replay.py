"""On-HBM experience replay: a preallocated device ring buffer of training sequences.

BASELINE.json config 5 asks for a replay buffer sized for the MI355X's 288 GB of HBM3E. The reference has no
replay at all — every iteration trains on exactly the ``seq_per_epoch`` freshly consumed sequences, on the CPU
(optimizer.py:433-483). :class:`HbmReplay` keeps every field the learner step reads as one preallocated tensor
per field on the GPU (``(capacity, seq_len, …)``), so

* ingest is one pinned host→device copy per field per iteration (``add``), written at the ring cursor;
* a minibatch is an on-device ``index_select`` of ``B`` rows (``sample``) — no host round trip, no allocation;
* capacity is chosen from a byte budget (``capacity_for_bytes``): one LSTM-512 1v1 sequence of 1400 steps is
  ≈2.4 MB, so 200 GB holds ≈80k sequences (≈115 M timesteps).

Sampling is uniform over the filled part, optionally restricted to the ``recent`` newest sequences. Off-policy
correction: the PPO ratio against the stored behaviour ``logp_old``, and — with the in-step V-trace (``vtrace``,
learner/optimizer.py advantages='vtrace-step') — every sampled sequence's advantages and value targets recomputed
at the weights being trained, with truncated importance weights against that behaviour log-prob.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np
import torch

from ..constants import UnitLayout

_F32 = torch.float32


def field_specs(S: int, layout: UnitLayout, hidden: Optional[int], reset: bool = False, vtrace: bool = False):
    U = layout.max_units
    A = 21 + U
    spec = {
        'env': ((S, 3), _F32), 'units': ((S, U, 10), _F32), 'actions': ((S, A), torch.uint8),
        'masks': ((S, A), torch.uint8), 'ret': ((S,), _F32), 'norm_ret': ((S,), _F32), 'adv': ((S,), _F32),
        'logp_old': ((S,), _F32), 'valid': ((S,), _F32),
    }
    if reset:                       # sequence packing: episode-start flags (learner/ingest.py SequencePacker)
        spec['reset'] = ((S,), torch.uint8)
    if vtrace:                      # in-step V-trace rows {reward, bootstrap, valid, last}: replayed sequences get
        spec['vt'] = ((S, 4), _F32)  # their advantages recomputed at every sampling, from the weights being trained
    if hidden:
        spec['h0'] = ((hidden,), _F32)
        spec['c0'] = ((hidden,), _F32)
    return spec


def bytes_per_sequence(S: int, layout: UnitLayout, hidden: Optional[int], reset: bool = False,
                       vtrace: bool = False) -> int:
    n = 0
    for shape, dt in field_specs(S, layout, hidden, reset, vtrace).values():
        k = 1
        for d in shape:
            k *= d
        n += k * torch.tensor([], dtype=dt).element_size()
    return n + 8     # version


class HbmReplay:
    def __init__(self, capacity: int, S: int, layout: UnitLayout, hidden: Optional[int], device, seed: int = 0,
                 reset: bool = False, vtrace: bool = False):
        if capacity < 1:
            raise ValueError('replay capacity must be >= 1')
        self.capacity = int(capacity)
        self.S = S
        self.device = torch.device(device)
        self.specs = field_specs(S, layout, hidden, reset, vtrace)
        self.data = {k: torch.zeros((self.capacity,) + shape, dtype=dt, device=self.device)
                     for k, (shape, dt) in self.specs.items()}
        self.version = torch.full((self.capacity,), -1, dtype=torch.long, device=self.device)
        self.cursor = 0
        self.size = 0
        self.inserted = 0
        self._g = torch.Generator(device=self.device).manual_seed(seed)
        # captured learner steps sample this pool through sample_into (host generator, one copy) instead of
        # sample_indices (the device generator); off by default so sample_indices' stream of indices stays the one
        # the learner uses (tests replay it)
        self.host_sampling = False

    @staticmethod
    def capacity_for_bytes(budget: float, S: int, layout: UnitLayout, hidden: Optional[int], reset: bool = False,
                           vtrace: bool = False) -> int:
        return max(1, int(budget // bytes_per_sequence(S, layout, hidden, reset, vtrace)))

    @property
    def nbytes(self) -> int:
        return sum(t.numel() * t.element_size() for t in self.data.values()) + self.version.numel() * 8

    def __len__(self):
        return self.size

    # ------------------------------------------------------------------------------------------------
    def add(self, batch: Dict[str, torch.Tensor], version: int = 0):
        """Append ``n`` sequences (host or device tensors, leading dim n) at the ring cursor (wrapping)."""
        n = int(next(iter(batch.values())).shape[0])
        if n > self.capacity:
            batch = {k: v[-self.capacity:] for k, v in batch.items()}
            n = self.capacity
        first = min(n, self.capacity - self.cursor)
        spans = [(self.cursor, 0, first)]
        if first < n:
            spans.append((0, first, n - first))
        for k, dst in self.data.items():
            src = batch.get(k)
            if src is None and k == 'reset':        # unpacked sequences: no episode starts inside
                for d0, _, cnt in spans:
                    dst[d0:d0 + cnt].zero_()
                continue
            src = batch[k]
            if src.device.type == 'cpu' and self.device.type == 'cuda' and not src.is_pinned():
                src = src.pin_memory()
            for d0, s0, cnt in spans:
                dst[d0:d0 + cnt].copy_(src[s0:s0 + cnt], non_blocking=True)
        for d0, _, cnt in spans:
            self.version[d0:d0 + cnt] = int(version)
        self.cursor = (self.cursor + n) % self.capacity
        self.size = min(self.capacity, self.size + n)
        self.inserted += n
        return n

    def prefill(self) -> int:
        """Fill the rest of the ring with copies of the sequences it already holds (device-to-device, doubling
        spans: ≈2 bytes moved per byte filled, so 100 GB takes tens of ms at HBM rate) and mark the copies as
        version -1. Benchmarks use it so a minibatch gathers from the whole ``capacity``-sized pool — the TLB and
        HBM-page spread of a full 100-200 GB replay — from the first timed step, not from a few GB of fresh data.
        New sequences keep landing at the cursor and overwrite the copies oldest-first. Returns the rows written."""
        if self.size == 0:
            raise RuntimeError('prefill needs at least one added sequence')
        if self.size >= self.capacity:
            return 0
        # the held sequences are the ring's first `size` rows (the cursor has not wrapped yet)
        have, wrote = self.size, 0
        while have < self.capacity:
            n = min(have, self.capacity - have)
            for v in self.data.values():
                v[have:have + n].copy_(v[:n])
            self.version[have:have + n] = -1
            have += n
            wrote += n
        self.size = self.capacity
        return wrote

    @property
    def fill_fraction(self) -> float:
        return self.size / self.capacity

    def _window(self, recent: Optional[int]):
        m = self.size if not recent else min(self.size, int(recent))
        return m

    def sample_indices(self, B: int, recent: Optional[int] = None) -> torch.Tensor:
        if self.size == 0:
            raise RuntimeError('replay is empty')
        m = self._window(recent)
        r = torch.randint(0, m, (B,), device=self.device, generator=self._g)
        # newest-first window ending at the cursor: position (cursor - 1 - r) mod capacity
        return (self.cursor - 1 - r) % self.capacity

    def sample_into(self, out: torch.Tensor, recent: Optional[int] = None) -> torch.Tensor:
        """Sample ``out.numel()`` pool positions (same window as :meth:`sample_indices`) with a host generator and
        write them into the device tensor ``out`` with ONE pinned host→device copy on the current stream — instead
        of the device RNG + two index-arithmetic kernels + a copy (≈26 µs of launches per learner step). The pinned
        slots form a ring; a slot is refilled only after its previous copy has run."""
        if self.size == 0:
            raise RuntimeError('replay is empty')
        B = out.numel()
        if out.device.type != 'cuda':
            out.copy_(self.sample_indices(B, recent))
            return out
        ring = self.__dict__.get('_pin_ring')
        if ring is None or ring[0][0].numel() != B:
            ring = self._pin_ring = [[torch.empty(B, dtype=torch.long, pin_memory=True), None] for _ in range(4)]
            self._pin_pos = 0
            self._host_rng = np.random.default_rng(int(torch.randint(0, 2 ** 31 - 1, (1,)).item()))
        slot = ring[self._pin_pos]
        self._pin_pos = (self._pin_pos + 1) % len(ring)
        if slot[1] is not None:
            slot[1].synchronize()
        r = self._host_rng.integers(0, self._window(recent), B)
        slot[0].numpy()[:] = (self.cursor - 1 - r) % self.capacity
        out.copy_(slot[0], non_blocking=True)
        ev = slot[1] = slot[1] or torch.cuda.Event()
        ev.record()
        return out

    def gather(self, idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {k: v.index_select(0, idx) for k, v in self.data.items()}

    def sample(self, B: int, recent: Optional[int] = None) -> Dict[str, torch.Tensor]:
        return self.gather(self.sample_indices(B, recent))
