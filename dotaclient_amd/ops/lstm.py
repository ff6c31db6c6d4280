"""Autograd wrapper around the persistent LSTM recurrence kernels (ops/csrc/lstm.hip).

``lstm_sequence(x, w_ih, w_hh, b_ih, b_hh, h0, c0)`` is a drop-in for a single-layer ``nn.LSTM`` (batch_first,
PyTorch gate order i, f, g, o) returning ``(out (B,S,H) f32, h_n, c_n)``:

* the input projection ``x·W_ihᵀ + b_ih + b_hh`` for all timesteps is one bf16 GEMM with fp32 output (hipBLASLt);
* the recurrence runs in ONE persistent launch per ≤64-sequence chunk (``_C.lstm_fwd``), saving the activated gates
  and cell states for backward;
* backward runs the reverse recurrence in one launch (``_C.lstm_bwd``) producing ∂L/∂gates for every step, then the
  weight gradients are plain GEMMs over all B·S rows: dW_ih = dGᵀx, dW_hh = dGᵀh_{t-1}, db = ΣdG, dx = dG·W_ih.
"""
from __future__ import annotations

import torch

from . import require



def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 × bf16 → fp32 GEMM (hipBLASLt) — fp32 accumulation and output."""
    return torch.mm(a.to(torch.bfloat16), b.to(torch.bfloat16), out_dtype=torch.float32)


class _Recurrence(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, w_hh, h0, c0, err):
        C = require()
        whh16 = w_hh.detach().to(torch.bfloat16).contiguous()
        B = xp.shape[0]
        MAX_B = C.lstm_max_batch(w_hh.shape[1])
        outs = []
        for s in range(0, B, MAX_B):
            e = min(B, s + MAX_B)
            outs.append(C.lstm_fwd(xp[s:e].contiguous(), whh16, h0[s:e].contiguous(), c0[s:e].contiguous(), err,
                                   True))
        hs16, hsf, cs, gates, hn, cn = (torch.cat([o[i] for o in outs]) if len(outs) > 1 else outs[0][i]
                                        for i in range(6))
        ctx.save_for_backward(gates, cs, c0, whh16, hs16, h0)
        ctx.err = err
        ctx.mark_non_differentiable(hs16)
        return hsf, hn, cn, hs16

    @staticmethod
    def backward(ctx, dhs, dhn, dcn, _dhs16):
        C = require()
        gates, cs, c0, whh16, hs16, h0 = ctx.saved_tensors
        B, S, H = cs.shape
        dhs = dhs.contiguous() if dhs is not None else torch.zeros_like(cs)
        MAX_B = C.lstm_max_batch(H)
        outs = []
        for s in range(0, B, MAX_B):
            e = min(B, s + MAX_B)
            outs.append(C.lstm_bwd(dhs[s:e], gates[s:e], cs[s:e], c0[s:e].contiguous(),
                                   None if dhn is None else dhn[s:e].contiguous(),
                                   None if dcn is None else dcn[s:e].contiguous(), whh16, ctx.err))
        dgates, dh0, dc0 = (torch.cat([o[i] for o in outs]) if len(outs) > 1 else outs[0][i] for i in range(3))
        # dW_hh = Σ_t dG_tᵀ h_{t-1}
        hprev = torch.cat([h0.to(torch.bfloat16).unsqueeze(1), hs16[:, :-1]], dim=1).reshape(B * S, H)
        dg2 = dgates.reshape(B * S, 4 * H)
        dw_hh = _mm_f32(dg2.t(), hprev)
        ctx.dgates = None
        return dgates, dw_hh, dh0, dc0, None


class _InputProjection(torch.autograd.Function):
    """xp = x·W_ihᵀ + b_ih + b_hh as one bf16 GEMM with fp32 output."""

    @staticmethod
    def forward(ctx, x, w_ih, b_ih, b_hh):
        B, S, I = x.shape
        x2 = x.reshape(B * S, I).to(torch.bfloat16)
        w16 = w_ih.detach().to(torch.bfloat16)
        xp = _mm_f32(x2, w16.t()) + (b_ih + b_hh)
        ctx.save_for_backward(x2, w16)
        ctx.shape = (B, S, I)
        return xp.view(B, S, -1)

    @staticmethod
    def backward(ctx, dxp):
        x2, w16 = ctx.saved_tensors
        B, S, I = ctx.shape
        g2 = dxp.reshape(B * S, -1)
        g16 = g2.to(torch.bfloat16)
        dx = torch.mm(g16, w16, out_dtype=torch.float32).view(B, S, I)
        dw = torch.mm(g16.t(), x2, out_dtype=torch.float32)
        db = g2.sum(0)
        return dx, dw, db, db


def lstm_sequence(x, w_ih, w_hh, b_ih, b_hh, h0, c0, err):
    """Returns (out f32 (B,S,H), h_n (B,H), c_n (B,H), out_bf16 (B,S,H))."""
    xp = _InputProjection.apply(x, w_ih, b_ih, b_hh)
    return _Recurrence.apply(xp, w_hh, h0, c0, err)
