"""Launch helpers of the XCD-team persistent LSTM recurrence kernels (ops/csrc/lstm_team.hip).

* ``team_fwd`` — the recurrence in ONE persistent launch (``_C.lstm_team_fwd``): 32 workgroups of ONE XCD per
  sequence chain, exchanging the step state through that XCD's L2, gates in unit-major (…, H, 4) layout; it saves the
  activated gates and cell states for the backward;
* ``team_bwd`` — the reverse recurrence in one launch (``_C.lstm_team_bwd``) producing ∂L/∂gates for every step (the
  weight gradients are the learner's split-K GEMMs, ops/csrc/gemm_tn.hip);
* ``gate_perm`` / ``team_ctl`` — the gate-major → unit-major row permutation and the per-stream control block.

(A cross-XCD "ring" recurrence — every hand-off over the Infinity Fabric — measured 2.5-3 µs per step against the
team kernel's ≈1.3-1.5 µs and was removed in round 5. The ``nn.LSTM``-shaped autograd wrapper that tests the
kernels against torch lives in tests/test_lstm_kernel.py.)
"""
from __future__ import annotations

import torch


def gate_perm(H: int, device) -> torch.Tensor:
    """Row permutation gate-major (q·H + j) → unit-major (4·j + q): W[perm] puts a unit's 4 gates together."""
    j = torch.arange(H, device=device)
    return (torch.arange(4, device=device)[None, :] * H + j[:, None]).reshape(-1)


_CTL = {}


def team_ctl(device=None, stream=None) -> torch.Tensor:
    """The persistent, self-cleaning control block for team-LSTM launches on (device, stream): zero-initialised
    once; each launch leaves it clean for the next one and advances its epoch (lstm_team.hip ``TeamCtl``). Team
    kernels on different streams must not share a block, kernels on one stream are serialised anyway."""
    dev = torch.device(device) if device is not None else torch.device('cuda', torch.cuda.current_device())
    if dev.index is None:
        dev = torch.device('cuda', torch.cuda.current_device())
    s = stream if stream is not None else torch.cuda.current_stream(dev)
    key = (dev.index, s.cuda_stream)
    t = _CTL.get(key)
    if t is None:
        t = _CTL[key] = torch.zeros(64, dtype=torch.int32, device=dev)
    return t


def team_fwd(C, xp4, whh16, h0, c0, err, want_f32_h, **kw):
    return C.lstm_team_fwd(xp4, whh16, h0.contiguous(), c0.contiguous(), err, team_ctl(xp4.device), want_f32_h,
                           **kw)


def team_bwd(C, dhs, gates4, cs, c0, dhn, dcn, whh16, err, **kw):
    return C.lstm_team_bwd(dhs, gates4, cs, c0.contiguous(), dhn, dcn, whh16, err, team_ctl(dhs.device), **kw)


