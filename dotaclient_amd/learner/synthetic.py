"""Synthetic experience batches of the exact learner schema, generated on the target device.

The learner benchmark (bench.py) and tests need experience without a running game. Shapes, dtypes and the
structure of masks/actions follow the experience contract (reference agent.py:340-409):

* per step a random number of live units per block (zero rows for padding, −1 handles), features in the
  featurizer's value ranges;
* valid-action masks derived from the handles exactly like ``Policy.action_masks`` (self never targetable,
  attack disabled without targets), the enum sampled among valid options, then only the heads the enum needs
  (hierarchical sampling, policy.py:245-262); the selected-heads mask = head mask ∧ valid mask (agent.py:660);
* rewards/values/behaviour log-probs drawn from plausible ranges, GAE / discounted returns computed per sequence;
* a tail of padded steps (no selection) in some sequences, like the learner's rollout padding (optimizer.py:363-378).
"""
from __future__ import annotations

from typing import Dict, Optional

import torch

from ..constants import ENUM_ATTACK, ENUM_MOVE, N_MOVE_ENUMS, UnitLayout


def _gae_torch(rew, val, gamma, lam, valid):
    B, S = rew.shape
    adv = torch.zeros_like(rew)
    acc = torch.zeros(B, device=rew.device)
    next_v = torch.zeros(B, device=rew.device)
    for t in range(S - 1, -1, -1):
        delta = rew[:, t] + gamma * next_v - val[:, t]
        acc = (delta + gamma * lam * acc) * valid[:, t]
        adv[:, t] = acc
        next_v = val[:, t] * valid[:, t]
    return adv, adv + val


def make_batch(B: int, S: int, layout: UnitLayout, hidden: Optional[int], device='cpu', seed: int = 0,
               pad_frac: float = 0.1, gamma: float = 0.98, lam: float = 0.95) -> Dict[str, torch.Tensor]:
    g = torch.Generator(device='cpu').manual_seed(seed)
    U = layout.max_units
    A = 3 + 2 * N_MOVE_ENUMS + U

    def rnd(*shape):
        return torch.rand(*shape, generator=g)

    # live units per block
    live = torch.zeros(B, S, U, dtype=torch.bool)
    for off, cnt in zip(layout.offsets, layout.counts):
        n = (rnd(B, S, 1) * (cnt + 1)).floor().clamp(max=cnt)
        idx = torch.arange(cnt).view(1, 1, cnt)
        live[..., off:off + cnt] = idx < n
    live[..., 0] = True   # self hero
    units = torch.zeros(B, S, U, 10)
    units[..., 0] = rnd(B, S, U)                       # 1 - hp/hp_max
    units[..., 1:3] = rnd(B, S, U, 2) * 2 - 1          # loc x/y
    units[..., 3] = -0.25
    units[..., 4] = rnd(B, S, U) - 0.5                 # distance
    ang = rnd(B, S, U) * 6.2831853
    units[..., 5], units[..., 6] = torch.sin(ang), torch.cos(ang)
    units[..., 7:10] = (rnd(B, S, U, 3) > 0.5).float() - 0.5
    units = units * live.unsqueeze(-1)
    env = torch.stack([rnd(B, S) * 0.5, torch.sin(rnd(B, S) * 6.28), torch.where(rnd(B, S) > 0.5, 0.2, -0.2)], -1)

    targetable = live & (rnd(B, S, U) > 0.3)
    targetable[..., 0] = False
    enum_valid = torch.ones(B, S, 3, dtype=torch.bool)
    enum_valid[..., ENUM_ATTACK] = targetable.any(-1)
    valid = torch.cat([enum_valid, torch.ones(B, S, 2 * N_MOVE_ENUMS, dtype=torch.bool), targetable], -1)

    enum = torch.multinomial(enum_valid.reshape(-1, 3).float(), 1, generator=g).view(B, S)
    xs = (rnd(B, S) * N_MOVE_ENUMS).long().clamp(max=N_MOVE_ENUMS - 1)
    ys = (rnd(B, S) * N_MOVE_ENUMS).long().clamp(max=N_MOVE_ENUMS - 1)
    tprob = targetable.reshape(-1, U).float()
    tprob[tprob.sum(-1) == 0, 0] = 1.0
    tgt = torch.multinomial(tprob, 1, generator=g).view(B, S)
    actions = torch.zeros(B, S, A, dtype=torch.uint8)
    head = torch.zeros(B, S, A, dtype=torch.bool)
    ar = torch.arange
    bi, si = torch.meshgrid(ar(B), ar(S), indexing='ij')
    actions[bi, si, enum] = 1
    head[..., :3] = True
    move = enum == ENUM_MOVE
    att = enum == ENUM_ATTACK
    actions[bi[move], si[move], 3 + xs[move]] = 1
    actions[bi[move], si[move], 3 + N_MOVE_ENUMS + ys[move]] = 1
    head[..., 3:3 + 2 * N_MOVE_ENUMS] |= move.unsqueeze(-1)
    actions[bi[att], si[att], 3 + 2 * N_MOVE_ENUMS + tgt[att]] = 1
    head[..., 3 + 2 * N_MOVE_ENUMS:] |= att.unsqueeze(-1)
    masks = (head & valid).to(torch.uint8)

    # padded tail (no selections, zero states) in some sequences
    step_valid = torch.ones(B, S)
    for b in range(B):
        if rnd(1).item() < pad_frac * 4:
            n_pad = int(rnd(1).item() * pad_frac * S)
            if n_pad:
                step_valid[b, S - n_pad:] = 0
    pv = step_valid.bool()
    actions *= pv.unsqueeze(-1).to(torch.uint8)
    masks *= pv.unsqueeze(-1).to(torch.uint8)
    units *= step_valid.view(B, S, 1, 1)
    env *= step_valid.unsqueeze(-1)

    rew = (torch.randn(B, S, generator=g) * 0.05) * step_valid
    val = torch.randn(B, S, generator=g) * 0.3
    adv, ret = _gae_torch(rew, val, gamma, lam, step_valid)
    adv = (adv - adv[pv].mean()) / (adv[pv].std() + 1e-8) * step_valid
    n_sel = actions.sum(-1).float()
    logp_old = -(rnd(B, S) * 2.0 + 0.5) * (n_sel > 0)
    # in-step V-trace rows {reward, bootstrap, valid, last}: each sequence one episode ending at its last valid row
    # (a terminal: bootstrap 0)
    last = torch.zeros(B, S)
    n_valid = step_valid.sum(1).long()
    last[torch.arange(B), (n_valid - 1).clamp(min=0)] = 1.0
    vt = torch.stack([rew, torch.zeros(B, S), step_valid, last], -1)
    out = {'env': env, 'units': units, 'actions': actions, 'masks': masks, 'adv': adv, 'ret': ret,
           'logp_old': logp_old, 'norm_ret': adv.clone(), 'valid': step_valid, 'vt': vt}
    if hidden:
        out['h0'] = torch.randn(B, hidden, generator=g) * 0.1
        out['c0'] = torch.randn(B, hidden, generator=g) * 0.1
    return {k: v.to(device).contiguous() for k, v in out.items()}


class DeviceReplay:
    """A pool of synthetic sequences resident in device memory (an :class:`~.replay.HbmReplay` filled with
    :func:`make_batch` data); :meth:`sample` gathers a minibatch on-device — the bench's on-HBM replay source."""

    def __init__(self, n_seq: int, S: int, layout: UnitLayout, hidden: Optional[int], device, seed: int = 0,
                 chunk: int = 16, vtrace: bool = False):
        from .replay import HbmReplay
        self.buf = HbmReplay(n_seq, S, layout, hidden, device, seed=seed, vtrace=vtrace)
        self.buf.host_sampling = True
        for i in range(0, n_seq, chunk):
            self.buf.add(make_batch(min(chunk, n_seq - i), S, layout, hidden, device=device, seed=seed + i))
        self.data = self.buf.data
        self.n = n_seq
        self.device = torch.device(device)

    def sample(self, B: int) -> Dict[str, torch.Tensor]:
        return self.buf.sample(B)
