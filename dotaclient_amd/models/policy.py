"""Entity-encoder + recurrent policy (torch reference path).

This is the *correctness oracle* for the fused MI355X path (``dotaclient_amd.models.fused``) and the model used on
CPU. Parameter names and shapes are the reference's (reference policy.py:52-78), so ``state_dict``
checkpoints are interchangeable with dotaclient's ``model_%09d.pt`` files in ``compat`` configuration.

Architecture (reference policy.py:92-169):

    env(3) ─ affine_env ─ relu ───────────────────────────────────────────────┐
    units(U,10) ─ affine_unit_basic_stats ─ relu ─ affine_unit_<type> ─ max/type ─┤ cat(896) ─ affine_pre_rnn ─ relu
                                     └──────── unit embeddings (U,128) ──────┐   │
    rnn: 'linear' = fake_rnn Linear (reference, policy.py:145) | 'lstm' = nn.LSTM (north star, policy.py:67)
    heads: enum(3), x(9), y(9), value(1); target_unit = affine_unit_attention(x) · unit_embeddings^T (U)

Extensions over the reference (all opt-in through :class:`PolicyConfig`):

* ``rnn='lstm'`` with any hidden width (BASELINE configs LSTM-128 / LSTM-512); hidden state threaded through
  ``forward`` (the reference passes ``hidden`` but never uses it, agent.py:641);
* ``layout=LAYOUT_5V5`` and ``entity_attention=True`` (BASELINE config 4: per-unit self-attention before pooling);
* ``compat_bugs=True`` reproduces the reference's enemy-tower pooling bug (policy.py:127) and its
  non-max-stabilised masked softmax (policy.py:171-180). Default is the corrected behaviour.
"""
from __future__ import annotations

from dataclasses import dataclass, field, asdict, replace
from typing import Dict, Optional, Tuple

import numpy as np
import torch
import torch.nn as nn
import torch.nn.functional as F

from ..constants import (ACTION_OUTPUT_COUNTS, ENUM_ATTACK, ENUM_MOVE, INPUT_KEYS, LAYOUT_1V1, LAYOUT_5V5,
                         MOVE_ENUMS, N_ENV_FEATURES, N_MOVE_ENUMS, N_UNIT_FEATURES, OBSERVATIONS_PER_SECOND,
                         OUTPUT_KEYS, TICKS_PER_OBSERVATION, UNIT_KEYS, UnitLayout)

TYPE_SUFFIX = ['ah', 'eh', 'anh', 'enh', 'ath', 'eth']


@dataclass
class PolicyConfig:
    rnn: str = 'linear'            # 'linear' (reference fake_rnn) | 'lstm'
    pre_rnn_dim: int = 256
    hidden: int = 256              # rnn output width (heads input)
    unit_dim: int = 128
    env_dim: int = 128
    layout: UnitLayout = field(default_factory=lambda: LAYOUT_1V1)
    compat_bugs: bool = False
    entity_attention: bool = False
    attention_heads: int = 4

    def to_dict(self):
        d = asdict(self)
        d['layout'] = list(self.layout.counts)
        return d

    @classmethod
    def from_dict(cls, d):
        d = dict(d)
        if 'layout' in d and not isinstance(d['layout'], UnitLayout):
            d['layout'] = UnitLayout(*d['layout'])
        return cls(**d)


PRESETS: Dict[str, PolicyConfig] = {
    # exact reference network (policy.py), incl. its quirks
    'compat': PolicyConfig(rnn='linear', hidden=256, compat_bugs=True),
    # BASELINE config 1 (plumbing): LSTM-128
    'lstm128': PolicyConfig(rnn='lstm', hidden=128),
    # BASELINE configs 2/3 (flagship): LSTM-512
    'lstm512': PolicyConfig(rnn='lstm', hidden=512),
    # BASELINE config 4: 5v5 entity attention
    '5v5': PolicyConfig(rnn='lstm', hidden=512, layout=LAYOUT_5V5, entity_attention=True),
}


def get_config(name_or_cfg) -> PolicyConfig:
    if isinstance(name_or_cfg, PolicyConfig):
        return name_or_cfg
    return replace(PRESETS[name_or_cfg])


def masked_log_softmax(logits: torch.Tensor, mask: torch.Tensor, dim: int = -1, stable: bool = True) -> torch.Tensor:
    """``log p = logits − log Σ_{mask} exp(logits)``.

    ``stable=False`` is the reference formula (policy.py:171-180, no max-subtraction). Rows whose mask is all
    false return ``logits`` (finite) instead of the reference's ``+inf``; such rows never contribute to a loss
    (nothing is selected in them), and keeping them finite lets the loss be written densely (no ``masked_select``).
    """
    mask = mask.bool()
    if stable:
        neg = torch.finfo(logits.dtype).min
        m = torch.where(mask, logits, torch.full_like(logits, neg)).amax(dim=dim, keepdim=True)
        m = torch.where(mask.any(dim=dim, keepdim=True), m, torch.zeros_like(m)).detach()
        s = (torch.exp(logits - m) * mask).sum(dim=dim, keepdim=True)
    else:
        m = torch.zeros_like(logits[..., :1])
        s = (torch.exp(logits) * mask).sum(dim=dim, keepdim=True)
    s = torch.where(s > 0, s, torch.ones_like(s))
    return logits - m - torch.log(s)


class EntityAttention(nn.Module):
    """Pre-LN multi-head self-attention over the unit axis (5v5 entity-attention policy, BASELINE config 4)."""

    def __init__(self, dim: int, heads: int):
        super().__init__()
        self.heads = heads
        self.ln = nn.LayerNorm(dim)
        self.qkv = nn.Linear(dim, 3 * dim)
        self.out = nn.Linear(dim, dim)

    def forward(self, x: torch.Tensor, valid: Optional[torch.Tensor] = None) -> torch.Tensor:
        *lead, U, D = x.shape
        h = self.heads
        q, k, v = self.qkv(self.ln(x)).reshape(*lead, U, 3, h, D // h).unbind(-3)
        q, k, v = (t.transpose(-2, -3) for t in (q, k, v))   # (..., h, U, d)
        att = (q @ k.transpose(-1, -2)) / float(np.sqrt(D // h))
        if valid is not None:
            att = att.masked_fill(~valid.unsqueeze(-2).unsqueeze(-3), -1e9)
        o = torch.softmax(att, dim=-1) @ v
        return x + self.out(o.transpose(-2, -3).reshape(*lead, U, D))


class Policy(nn.Module):
    """See module docstring. ``forward`` keeps the reference's keyword signature."""

    TICKS_PER_SECOND = 30
    MAX_MOVE_SPEED = 550
    N_MOVE_ENUMS = N_MOVE_ENUMS
    MOVE_ENUMS = MOVE_ENUMS
    OBSERVATIONS_PER_SECOND = OBSERVATIONS_PER_SECOND
    TICKS_PER_OBSERVATION = TICKS_PER_OBSERVATION
    OUTPUT_KEYS = OUTPUT_KEYS
    INPUT_KEYS = INPUT_KEYS

    def __init__(self, config: PolicyConfig | str = 'compat'):
        super().__init__()
        cfg = get_config(config)
        self.config = cfg
        self.layout = cfg.layout
        self.MAX_UNITS = cfg.layout.max_units
        self.ACTION_OUTPUT_COUNTS = cfg.layout.action_counts()
        U, E = cfg.unit_dim, cfg.env_dim
        self.affine_env = nn.Linear(N_ENV_FEATURES, E)
        self.affine_unit_basic_stats = nn.Linear(N_UNIT_FEATURES, U)
        for s in TYPE_SUFFIX:
            setattr(self, f'affine_unit_{s}', nn.Linear(U, U))
        if cfg.entity_attention:
            self.entity_attn = EntityAttention(U, cfg.attention_heads)
        self.affine_pre_rnn = nn.Linear(E + 6 * U, cfg.pre_rnn_dim)
        if cfg.rnn == 'linear':
            self.fake_rnn = nn.Linear(cfg.pre_rnn_dim, cfg.hidden)
        elif cfg.rnn == 'lstm':
            self.rnn = nn.LSTM(input_size=cfg.pre_rnn_dim, hidden_size=cfg.hidden, num_layers=1, batch_first=True)
        else:
            raise ValueError(cfg.rnn)
        H = cfg.hidden
        self.affine_head_enum = nn.Linear(H, 3)
        self.affine_move_x = nn.Linear(H, N_MOVE_ENUMS)
        self.affine_move_y = nn.Linear(H, N_MOVE_ENUMS)
        self.affine_unit_attention = nn.Linear(H, U)
        self.affine_value = nn.Linear(H, 1)
        self.weight_version = -1

    # ------------------------------------------------------------------------------------------------
    @property
    def is_recurrent(self) -> bool:
        return self.config.rnn == 'lstm'

    def initial_hidden(self, batch: int, device=None, dtype=torch.float32):
        if not self.is_recurrent:
            return None
        H = self.config.hidden
        z = torch.zeros(1, batch, H, device=device, dtype=dtype)
        return (z, z.clone())

    @staticmethod
    def pack_units(inputs: Dict[str, torch.Tensor]) -> torch.Tensor:
        return torch.cat([inputs[k] for k in UNIT_KEYS], dim=-2)

    def single(self, hidden=None, **kwargs):
        """A single element of a sequence (policy.py:80-84)."""
        kwargs = {k: v.unsqueeze(0).unsqueeze(0) for k, v in kwargs.items()}
        return self(**kwargs, hidden=hidden)

    def sequence(self, hidden=None, **kwargs):
        """A single sequence (policy.py:86-90)."""
        kwargs = {k: v.unsqueeze(0) for k, v in kwargs.items()}
        return self(**kwargs, hidden=hidden)

    def forward(self, env, allied_heroes, enemy_heroes, allied_nonheroes, enemy_nonheroes, allied_towers,
                enemy_towers, hidden=None):
        units = torch.cat([allied_heroes, enemy_heroes, allied_nonheroes, enemy_nonheroes, allied_towers,
                           enemy_towers], dim=2)
        return self.forward_packed(env, units, hidden)

    # ------------------------------------------------------------------------------------------------
    def encode(self, env: torch.Tensor, units: torch.Tensor):
        """env (B,S,3), units (B,S,U,10) → x (B,S,pre_rnn_dim), unit_embedding (B,S,U,unit_dim)."""
        cfg = self.config
        env_e = F.relu(self.affine_env(env))
        basic = F.relu(self.affine_unit_basic_stats(units))
        embs = []
        for key, s in zip(UNIT_KEYS, TYPE_SUFFIX):
            sl = self.layout.slices()[key]
            embs.append(getattr(self, f'affine_unit_{s}')(basic[..., sl, :]))
        unit_embedding = torch.cat(embs, dim=2)
        if cfg.entity_attention:
            unit_embedding = self.entity_attn(unit_embedding)
        pools = []
        for i, key in enumerate(UNIT_KEYS):
            sl = self.layout.slices()[key]
            if cfg.compat_bugs and key == 'enemy_towers':
                sl = self.layout.slices()['enemy_nonheroes']   # reference policy.py:127 pools enh_embedding
            pools.append(unit_embedding[..., sl, :].amax(dim=2))
        x = torch.cat([env_e] + pools, dim=2)
        x = F.relu(self.affine_pre_rnn(x))
        return x, unit_embedding

    def recurrent(self, x: torch.Tensor, hidden=None, reset: Optional[torch.Tensor] = None):
        """``reset`` (B, S) bool/u8, sequence packing: an episode starts at step t of row b — its h, c are zero
        before that step (the oracle of the fused recurrence's reset flags, ops/csrc/lstm_team.hip)."""
        if self.config.rnn == 'linear':
            return self.fake_rnn(x), hidden
        if hidden is None:
            hidden = self.initial_hidden(x.shape[0], device=x.device, dtype=x.dtype)
        if reset is not None and bool(reset.any()):
            return self._lstm_with_resets(x, hidden, reset.bool())
        out, hidden = self.rnn(x, hidden)
        return out, hidden

    def _lstm_with_resets(self, x, hidden, reset):
        r = self.rnn
        h, c = hidden[0][0], hidden[1][0]
        xp = F.linear(x, r.weight_ih_l0, r.bias_ih_l0 + r.bias_hh_l0)
        outs = []
        for t in range(x.shape[1]):
            keep = (~reset[:, t]).to(x.dtype).unsqueeze(1)
            h, c = h * keep, c * keep
            i, f, g, o = (xp[:, t] + F.linear(h, r.weight_hh_l0)).chunk(4, 1)
            c = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(g)
            h = torch.sigmoid(o) * torch.tanh(c)
            outs.append(h)
        return torch.stack(outs, 1), (h.unsqueeze(0), c.unsqueeze(0))

    def heads(self, x: torch.Tensor, unit_embedding: torch.Tensor):
        q = self.affine_unit_attention(x)                                        # (B,S,unit_dim)
        target = torch.matmul(q.unsqueeze(2), unit_embedding.transpose(2, 3)).squeeze(2)   # (B,S,U)
        d = {
            'enum': self.affine_head_enum(x),
            'x': self.affine_move_x(x),
            'y': self.affine_move_y(x),
            'target_unit': target,
        }
        return d, self.affine_value(x)

    def forward_packed(self, env: torch.Tensor, units: torch.Tensor, hidden=None, reset=None):
        x, unit_embedding = self.encode(env, units)
        x, hidden = self.recurrent(x, hidden, reset)
        logits, value = self.heads(x, unit_embedding)
        return logits, value, hidden

    # ------------------------------------------------------------------------------------------------
    # Action selection helpers (reference classmethods, policy.py:171-295)
    def masked_softmax(self, logits, mask, dim=2):
        return masked_log_softmax(logits, mask, dim=dim, stable=not self.config.compat_bugs)

    def flatten_selections(self, inputs):
        d = {}
        for key, count in self.ACTION_OUTPUT_COUNTS.items():
            t = torch.zeros(count, dtype=torch.uint8)
            if key in inputs:
                t[inputs[key]] = 1
            d[key] = t
        return d

    @staticmethod
    def flatten_head(inputs, dim=2):
        return torch.cat(list(inputs.values()), dim=dim)

    def unpack_heads(self, inputs):
        out, acc = {}, 0
        for k, n in self.ACTION_OUTPUT_COUNTS.items():
            out[k] = inputs[..., acc:acc + n]
            acc += n
        return out

    def flat_actions_to_headmask(self, inputs):
        parts, acc = [], 0
        for k, n in self.ACTION_OUTPUT_COUNTS.items():
            h = inputs[:, acc:acc + n].any(dim=1, keepdim=True)
            parts.append(h.repeat(1, n))
            acc += n
        return torch.cat(parts, dim=1)

    def sample_action(self, logits, mask, generator=None):
        log_probs = self.masked_softmax(logits=logits, mask=mask)
        probs = torch.exp(log_probs) * mask.bool()
        return torch.multinomial(probs.reshape(-1, probs.shape[-1]), num_samples=1, generator=generator)

    def select_actions(self, heads_logits, masks, generator=None):
        """Hierarchical sampling (policy.py:245-262): enum first, then x,y (move) or target_unit (attack).
        Batch of rows supported (the reference samples only the last row, policy.py:33)."""
        action = {'enum': self.sample_action(heads_logits['enum'], masks['enum'], generator)}
        if action['enum'].numel() == 1:
            e = int(action['enum'])
            if e == ENUM_MOVE:
                action['x'] = self.sample_action(heads_logits['x'], masks['x'], generator)
                action['y'] = self.sample_action(heads_logits['y'], masks['y'], generator)
            elif e == ENUM_ATTACK:
                action['target_unit'] = self.sample_action(heads_logits['target_unit'], masks['target_unit'],
                                                           generator)
        return action

    def head_masks(self, selections):
        return {key: (torch.ones if key in selections else torch.zeros)(1, 1, val).byte()
                for key, val in self.ACTION_OUTPUT_COUNTS.items()}

    def action_masks(self, unit_handles):
        """Valid options from unit handles: self (slot 0) never targetable; no attack without a target."""
        masks = {key: torch.ones(1, 1, val).byte() for key, val in self.ACTION_OUTPUT_COUNTS.items()}
        valid_units = torch.as_tensor(unit_handles) != -1
        valid_units[0] = False
        if not valid_units.any():
            masks['enum'][0, 0, ENUM_ATTACK] = 0
        masks['target_unit'][0, 0] = valid_units
        return masks

    @staticmethod
    def mask_heads(head_prob_dict, unit_handles):
        """Reference's (dead) probability-masking helper (policy.py:285-295)."""
        invalid_units = torch.as_tensor(unit_handles) == -1
        invalid_units[0] = True
        if invalid_units.all():
            head_prob_dict['enum'][0, 0, 2] = 0.
        head_prob_dict['target_unit'][0, 0, invalid_units] = 0.
        return head_prob_dict


def batched_action_masks(handles: torch.Tensor) -> torch.Tensor:
    """(N,U) int handles → (N, 3+9+9+U) bool flat valid-option mask (vectorised ``action_masks``)."""
    N, U = handles.shape
    valid = handles != -1
    valid[:, 0] = False
    enum = torch.ones(N, 3, dtype=torch.bool, device=handles.device)
    enum[:, ENUM_ATTACK] = valid.any(dim=1)
    move = torch.ones(N, 2 * N_MOVE_ENUMS, dtype=torch.bool, device=handles.device)
    return torch.cat([enum, move, valid], dim=1)


class RndModel(nn.Module):
    """Random-network-distillation feature net (reference policy.py:298-317; unused by the reference)."""

    def __init__(self, requires_grad: bool = False):
        super().__init__()
        self.affine1 = nn.Linear(10, 64)
        self.affine2 = nn.Linear(64, 64)
        self.affine3 = nn.Linear(64, 64)
        self.affine4 = nn.Linear(64, 64)
        self.requires_grad_(requires_grad)

    def forward(self, env, allied_heroes, *unused):
        if allied_heroes.numel() == 0:
            allied_heroes = torch.zeros(1, 7)
        inputs = torch.cat([env.reshape(-1), allied_heroes.reshape(-1)])[:10]
        x = F.relu(self.affine1(inputs))
        x = F.relu(self.affine2(x))
        x = F.relu(self.affine3(x))
        return F.relu(self.affine4(x))
