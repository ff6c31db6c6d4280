"""MI355X execution of :class:`~dotaclient_amd.models.policy.Policy` on hand-written gfx950 kernels.

Same parameters (it wraps the reference module and reads its ``nn.Parameter``s, which live in the learner's flat
buffer), different execution:

=================  =====================================================================================
stage              MI355X path
=================  =====================================================================================
entity encoder     ``ops.encoder``: fused unit-MLP + per-type GEMM + max-pool (+argmax) HIP kernel
                   (falls back to bf16 torch ops only for configurations the kernel does not cover)
pre-RNN            bf16 GEMM (fp32 out) + ReLU
LSTM               ``ops.lstm``: input projection GEMM + ONE persistent recurrence launch (fwd and bwd)
heads + loss       ``ops.heads``: one heads GEMM + the fused pointer/log-softmax/PPO/entropy/value kernel
optimizer          ``learner.optim.FlatAdam``: fused clip + Adam kernels over the flat buffer
=================  =====================================================================================
"""
from __future__ import annotations

from typing import Dict

import torch
import torch.nn.functional as F

from .policy import Policy


class FusedPolicy:
    def __init__(self, policy: Policy):
        from .. import ops
        ops.require()
        self.policy = policy
        self.cfg = policy.config
        dev = next(policy.parameters()).device
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self._zero_v = None

    def refresh(self):
        pass

    # ------------------------------------------------------------------------------------------------
    def _wcat(self, with_value: bool):
        p = self.policy
        H = self.cfg.hidden
        dev = p.affine_value.weight.device
        wv, bv = p.affine_value.weight, p.affine_value.bias
        if not with_value:
            wv, bv = torch.zeros(1, H, device=dev), torch.zeros(1, device=dev)
        from ..ops.heads import LDZ
        pad = LDZ - (128 + 3 + 9 + 9 + 1)
        w = torch.cat([p.affine_unit_attention.weight, p.affine_head_enum.weight, p.affine_move_x.weight,
                       p.affine_move_y.weight, wv, torch.zeros(pad, H, device=dev)], 0)
        b = torch.cat([p.affine_unit_attention.bias, p.affine_head_enum.bias, p.affine_move_x.bias,
                       p.affine_move_y.bias, bv, torch.zeros(pad, device=dev)], 0)
        return w, b

    def trunk(self, env: torch.Tensor, units: torch.Tensor, h0=None, c0=None):
        """Encoder + pre-RNN + recurrence. Returns (xh (B,S,H) f32, emb (B,S,U,128) bf16, hn, cn)."""
        from ..ops.encoder import encode
        p = self.policy
        x, emb = encode(p, env, units)                 # x (B,S,pre_rnn) f32, emb bf16
        B, S, _ = x.shape
        if self.cfg.rnn == 'lstm':
            from ..ops.lstm import lstm_sequence
            H = self.cfg.hidden
            if h0 is None:
                h0 = torch.zeros(B, H, device=x.device)
                c0 = torch.zeros(B, H, device=x.device)
            r = p.rnn
            xh, hn, cn, _ = lstm_sequence(x, r.weight_ih_l0, r.weight_hh_l0, r.bias_ih_l0, r.bias_hh_l0,
                                          h0.contiguous(), c0.contiguous(), self.err)
        else:
            xh = F.linear(x, p.fake_rnn.weight, p.fake_rnn.bias)
            hn = cn = None
        return xh, emb, hn, cn

    def loss(self, batch: Dict[str, torch.Tensor], cfg):
        from ..ops.heads import heads_loss
        B, S = batch['env'].shape[:2]
        xh, emb, _, _ = self.trunk(batch['env'], batch['units'], batch.get('h0'), batch.get('c0'))
        with_value = cfg.vf_coef > 0
        w, b = self._wcat(with_value)
        U = emb.shape[2]
        loss, metrics, _ = heads_loss(xh.reshape(B * S, -1), w, b, emb.reshape(B * S, U, -1), batch, cfg, S)
        return loss, metrics

    def check_error(self):
        """Raise if a persistent kernel timed out (host sync — call at iteration boundaries, not per step)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f'persistent kernel error code {e} (recurrence hand-off timed out)')
