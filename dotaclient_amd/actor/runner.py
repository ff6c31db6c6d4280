"""Batched policy step for actors: forward + valid-action masks + hierarchical masked sampling.

Reference per-player path (agent.py:641-660, policy.py:171-283): ``policy.single`` → ``action_masks`` →
``select_actions`` (enum first, then x,y for move or target_unit for attack) → ``head_masks`` ∧ action masks. Here
one call serves a whole batch of players (the reference is strictly batch-1, quirk §2.10-10): all heads are sampled
in one shot and the enum's choice selects which are kept — the same distribution as sampling the needed heads only.
Also returns the joint log-probability of the sampled action and V(s) (behaviour-policy data for PPO) and carries
the LSTM state.

On GPU with the HIP extension, :class:`PolicyRunner` uses ``ops.actor`` (fused LSTM cell + masked Gumbel sampling
kernels) and captures the step in a hipGraph; on CPU it runs the torch reference.
"""
from __future__ import annotations

from collections import OrderedDict
from dataclasses import dataclass
from typing import Callable, Optional

import numpy as np
import torch

from ..constants import ENUM_ATTACK, ENUM_MOVE, N_MOVE_ENUMS
from ..models.policy import Policy, batched_action_masks, masked_log_softmax


@dataclass
class StepOutput:
    enum: np.ndarray          # (n,) int
    x: np.ndarray             # (n,) int
    y: np.ndarray             # (n,) int
    target: np.ndarray        # (n,) int
    actions: np.ndarray       # (n, A) u8 one-hot of sampled heads
    masks: np.ndarray         # (n, A) u8 selected-heads mask (head mask ∧ valid mask)
    logp: np.ndarray          # (n,) f32 joint log-prob
    value: np.ndarray         # (n,) f32

    def action_dict(self, i: int):
        d = {'enum': int(self.enum[i])}
        if d['enum'] == ENUM_MOVE:
            d['x'], d['y'] = int(self.x[i]), int(self.y[i])
        elif d['enum'] == ENUM_ATTACK:
            d['target_unit'] = int(self.target[i])
        return d


def sample_heads(logits: dict, valid: torch.Tensor, U: int, generator=None, stable: bool = True):
    """Sample (enum, x, y, target) for every row; returns tensors + flat one-hot actions/selected masks + logp."""
    n = valid.shape[0]
    offs = {'enum': (0, 3), 'x': (3, N_MOVE_ENUMS), 'y': (3 + N_MOVE_ENUMS, N_MOVE_ENUMS),
            'target_unit': (3 + 2 * N_MOVE_ENUMS, U)}
    samples, logps = {}, {}
    for k, (o, w) in offs.items():
        m = valid[:, o:o + w]
        lp = masked_log_softmax(logits[k].reshape(n, w).float(), m, dim=-1, stable=stable)
        p = torch.exp(lp) * m
        # rows with no valid entry (target when nothing is attackable): sample index 0, never selected
        p = torch.where(m.any(-1, keepdim=True), p, torch.nn.functional.one_hot(torch.zeros(n, dtype=torch.long,
                                                                                            device=p.device), w).float())
        s = torch.multinomial(p, 1, generator=generator).squeeze(1)
        samples[k] = s
        logps[k] = lp.gather(1, s[:, None]).squeeze(1)
    enum = samples['enum']
    move = enum == ENUM_MOVE
    att = enum == ENUM_ATTACK
    A = valid.shape[1]
    head = torch.zeros(n, A, dtype=torch.bool, device=valid.device)
    head[:, :3] = True
    head[:, 3:3 + 2 * N_MOVE_ENUMS] = move[:, None]
    head[:, 3 + 2 * N_MOVE_ENUMS:] = att[:, None]
    actions = torch.zeros(n, A, dtype=torch.uint8, device=valid.device)
    r = torch.arange(n, device=valid.device)
    actions[r, enum] = 1
    actions[r[move], 3 + samples['x'][move]] = 1
    actions[r[move], 3 + N_MOVE_ENUMS + samples['y'][move]] = 1
    actions[r[att], 3 + 2 * N_MOVE_ENUMS + samples['target_unit'][att]] = 1
    logp = logps['enum'] + move * (logps['x'] + logps['y']) + att * logps['target_unit']
    masks = (head & valid).to(torch.uint8)
    return samples, actions, masks, logp


class PolicyRunner:
    """Runs a :class:`Policy` for a batch of players on ``device``; keeps no per-player state itself."""

    def __init__(self, policy: Policy, device='cpu', seed: Optional[int] = None):
        self.policy = policy.to(device).eval()
        self.device = torch.device(device)
        self.generator = torch.Generator(device=self.device)
        if seed is not None:
            self.generator.manual_seed(seed)
        self.U = policy.layout.max_units
        self.stable = not policy.config.compat_bugs

    @torch.no_grad()
    def step(self, env: np.ndarray, units: np.ndarray, handles: np.ndarray, hidden=None):
        """env (n,3), units (n,U,10), handles (n,U) → (StepOutput, new hidden (h,c) each (n,H) or None)."""
        dev = self.device
        e = torch.as_tensor(env, device=dev, dtype=torch.float32)[:, None]
        u = torch.as_tensor(units, device=dev, dtype=torch.float32)[:, None]
        h = None
        if hidden is not None and self.policy.is_recurrent:
            h = (torch.as_tensor(hidden[0], device=dev)[None], torch.as_tensor(hidden[1], device=dev)[None])
        logits, value, hn = self.policy.forward_packed(e, u, h)
        valid = batched_action_masks(torch.as_tensor(handles, device=dev))
        samples, actions, masks, logp = sample_heads({k: v[:, 0] for k, v in logits.items()}, valid, self.U,
                                                     self.generator, self.stable)
        out = StepOutput(enum=samples['enum'].cpu().numpy(), x=samples['x'].cpu().numpy(),
                         y=samples['y'].cpu().numpy(), target=samples['target_unit'].cpu().numpy(),
                         actions=actions.cpu().numpy(), masks=masks.cpu().numpy(),
                         logp=logp.float().cpu().numpy(), value=value[:, 0, 0].float().cpu().numpy())
        new_hidden = None
        if hn is not None:
            new_hidden = (hn[0][0].cpu().numpy(), hn[1][0].cpu().numpy())
        return out, new_hidden


class RunnerCache:
    """``runner_for(policy)`` for the Actor: one runner for the synced latest policy and one per stored weight
    version (LRU of ``max_snapshots``), so games against the same snapshot share a runner — on the GPU, one
    captured graph and one slot table — instead of one per Policy object (the WeightStore builds a fresh object per
    opponent game, actor/weights.py). Players already bound to an evicted stateful runner keep using it."""

    def __init__(self, make: Callable, latest_policy=None, max_snapshots: int = 8):
        self.make = make
        self.latest_policy = latest_policy
        self.max_snapshots = max(1, int(max_snapshots))
        self.latest = None
        self.snapshots: "OrderedDict[int, object]" = OrderedDict()

    def __call__(self, policy):
        if policy is self.latest_policy:
            if self.latest is None:
                self.latest = self.make(policy)
            return self.latest
        key = getattr(policy, 'weight_version', None)
        key = ('obj', id(policy)) if key is None else key
        r = self.snapshots.get(key)
        if r is None:
            r = self.snapshots[key] = self.make(policy)
            while len(self.snapshots) > self.max_snapshots:
                self.snapshots.popitem(last=False)
        else:
            self.snapshots.move_to_end(key)
        return r

    def runners(self):
        return ([self.latest] if self.latest is not None else []) + list(self.snapshots.values())
