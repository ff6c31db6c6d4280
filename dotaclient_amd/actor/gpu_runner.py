"""GPU policy runner for the :class:`~dotaclient_amd.actor.game.Actor` game loop.

The reference actor steps one player per process on the CPU: ``policy.single`` → ``select_actions`` every observation
(agent.py:641-660) and carries the LSTM state in Python (agent.py:655-657). :class:`GpuRunner` serves all players
of one policy object from a graph-captured :class:`~dotaclient_amd.actor.batched.GpuActorPolicy`:

* every player owns a device slot (keyed by an opaque player key) — its LSTM h / c never leave the GPU; a freshly
  assigned slot is zeroed inside the captured step (keep mask), a finished player's slot is recycled (``release``);
* a call steps only the slots of the players passed in (the Actor steps one team at a time): the LSTM-cell kernel
  leaves the state of every other slot untouched (``active`` mask), so both teams' players share one graph;
* the recurrent state crosses PCIe only when the experience record needs it (``need_hidden``: every
  ``hidden_stride`` steps, reference-free R2D2-style stored state), otherwise only the featurized inputs go in and
  the sampled indices / masks / log-probs / values come out;
* weight updates are picked up by version (``policy.weight_version``, set by the WeightStore) and loaded in place,
  so the captured graph stays valid; capacity doubles on demand (re-capture, state carried over).

``step(env, units, handles, hidden)`` keeps the stateless :class:`~dotaclient_amd.actor.runner.PolicyRunner` API
(host hidden in, new hidden out) for callers that manage the state themselves.
"""
from __future__ import annotations

from typing import Dict, Hashable, List, Optional, Sequence, Tuple

import numpy as np
import torch

from ..models.policy import Policy
from .batched import GpuActorPolicy
from .runner import StepOutput


def gpu_runner_supported(policy: Policy) -> bool:
    """Policies the batched GPU actor path covers: 128-wide embeddings; entity attention over 64 slots × 4 heads."""
    cfg = policy.config
    if cfg.entity_attention and (cfg.layout.max_units != 64 or cfg.attention_heads != 4):
        return False
    return cfg.unit_dim == 128 and cfg.env_dim == 128


class GpuRunner:
    stateful = True

    def __init__(self, policy: Policy, device='cuda', seed: int = 0, capacity: int = 64,
                 use_graph: bool = True):
        if not gpu_runner_supported(policy):
            raise ValueError('GpuRunner: policy not covered by the batched GPU actor (see gpu_runner_supported)')
        self.policy = policy
        self.device = torch.device(device)
        self.seed = int(seed)
        self.use_graph = use_graph
        self.recurrent = policy.config.rnn == 'lstm'
        self.H = policy.config.hidden
        self.slots: Dict[Hashable, int] = {}
        self.free: List[int] = []
        self.gp: Optional[GpuActorPolicy] = None
        self._version = None
        self._grow(max(1, int(capacity)))

    # ------------------------------------------------------------------------------------------------
    @property
    def capacity(self) -> int:
        return self.gp.n

    def __len__(self):
        return len(self.slots)

    def _grow(self, cap: int):
        old = self.gp
        gp = GpuActorPolicy(self.policy, cap, device=self.device, seed=self.seed, use_graph=self.use_graph,
                            record=True)
        if self.use_graph:
            gp.capture()                 # capture zeroes the slot state: do it before carrying the old state over
        if old is not None:
            torch.cuda.synchronize(self.device)
            gp.h[:old.n].copy_(old.h)
            gp.c[:old.n].copy_(old.c)
            gp.ctr.copy_(old.ctr)
            self.free = list(range(cap - 1, old.n - 1, -1)) + self.free
        else:
            self.free = list(range(cap - 1, -1, -1))
        self.gp = gp
        self._version = getattr(self.policy, 'weight_version', None)

    def _assign(self, keys: Sequence[Hashable]) -> Tuple[np.ndarray, np.ndarray]:
        fresh = np.zeros(len(keys), bool)
        need = sum(1 for k in keys if k not in self.slots)
        if need > len(self.free):
            cap = self.gp.n
            while cap - len(self.slots) < need:
                cap *= 2
            self._grow(cap)
        rows = np.empty(len(keys), np.int64)
        for j, k in enumerate(keys):
            s = self.slots.get(k)
            if s is None:
                s = self.slots[k] = self.free.pop()
                fresh[j] = True
            rows[j] = s
        return rows, fresh

    def release(self, key: Hashable):
        """Return a finished player's slot; its state is zeroed when the slot is next assigned."""
        s = self.slots.pop(key, None)
        if s is not None:
            self.free.append(s)

    def _sync_weights(self):
        v = getattr(self.policy, 'weight_version', None)
        if v != self._version:
            self.gp.load_weights(self.policy)
            self._version = v

    # ------------------------------------------------------------------------------------------------
    def _run(self, rows: np.ndarray, fresh: np.ndarray, env, units, handles) -> StepOutput:
        gp = self.gp
        self._sync_weights()
        gp.h_env.numpy()[rows] = env
        gp.h_units.numpy()[rows] = units
        gp.h_handles.numpy()[rows] = handles
        keep = gp.h_keep.numpy()
        keep[:, 0] = 1.0
        keep[rows[fresh], 0] = 0.0
        act = gp.h_active.numpy()
        act[:] = 0.0
        act[rows] = 1.0
        gp.step_async()
        o = gp.wait()
        idx = o['idx'][rows].astype(np.int64)
        return StepOutput(enum=idx[:, 0], x=idx[:, 1], y=idx[:, 2], target=idx[:, 3],
                          actions=o['actions'][rows], masks=o['masks'][rows], logp=o['logp'][rows].copy(),
                          value=o['value'][rows].copy())

    def _read_hidden(self, rows: np.ndarray):
        r = torch.as_tensor(rows, device=self.device)
        return self.gp.h.index_select(0, r).cpu().numpy(), self.gp.c.index_select(0, r).cpu().numpy()

    def step_players(self, env: np.ndarray, units: np.ndarray, handles: np.ndarray, keys: Sequence[Hashable],
                     need_hidden: Optional[Sequence[bool]] = None):
        """One policy step for the players ``keys`` (rows of env/units/handles). Returns the StepOutput and, for
        recurrent policies, ``{row: (h, c)}`` of the state each ``need_hidden`` row had BEFORE this step."""
        rows, fresh = self._assign(keys)
        prev = None
        if self.recurrent and need_hidden is not None and any(need_hidden):
            sel = np.flatnonzero(np.asarray(need_hidden, bool))
            h, c = self._read_hidden(rows[sel])
            prev = {}
            for i, j in enumerate(sel):
                if fresh[j]:
                    prev[int(j)] = (np.zeros(self.H, np.float32), np.zeros(self.H, np.float32))
                else:
                    prev[int(j)] = (h[i], c[i])
        return self._run(rows, fresh, env, units, handles), prev

    @torch.no_grad()
    def step(self, env: np.ndarray, units: np.ndarray, handles: np.ndarray, hidden=None):
        """Stateless PolicyRunner-compatible step: host (h, c) (n,H) in → (StepOutput, new (h, c) or None)."""
        n = env.shape[0]
        keys = [('__tmp__', j) for j in range(n)]
        rows, fresh = self._assign(keys)
        try:
            if self.recurrent:
                r = torch.as_tensor(rows, device=self.device)
                if hidden is None:
                    fresh[:] = True
                else:
                    self.gp.h.index_copy_(0, r, torch.as_tensor(hidden[0], device=self.device, dtype=torch.float32))
                    self.gp.c.index_copy_(0, r, torch.as_tensor(hidden[1], device=self.device, dtype=torch.float32))
                    fresh[:] = False
                torch.cuda.current_stream(self.device).synchronize()
            out = self._run(rows, fresh, env, units, handles)
            new_hidden = self._read_hidden(rows) if self.recurrent else None
        finally:
            for k in keys:
                self.release(k)
        return out, new_hidden
