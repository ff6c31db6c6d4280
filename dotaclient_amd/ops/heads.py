"""Autograd wrapper for the fused heads + loss kernel (ops/csrc/heads_loss.hip).

``heads_loss(xh, wcat, bcat, emb, batch, cfg, ...)`` computes, for N = B·S rows,
``z = xh·Wcatᵀ + bcat`` (ONE bf16 GEMM with fp32 output for all five heads: pointer query, enum, x, y, value), then the
fused kernel evaluates the masked log-softmaxes, the PPO (or reference VPG) objective, entropies and the value loss
and writes ∂L/∂z and ∂L/∂(pointer logits) in the same pass. Backward is two GEMMs plus the rank-1 pointer-key
gradient ∂L/∂emb[n,u] = dtl[n,u]·q[n].

Column layout of z / Wcat (``LDZ`` = 160): ``[q 0:128 | enum 128:131 | x 131:140 | y 140:149 | value 149 | pad]``.
"""
from __future__ import annotations

from typing import Dict

import torch

from . import require

LDZ = 160
Q = 128
COL_ENUM, COL_X, COL_Y, COL_V = 128, 131, 140, 149


def batch_norms(actions: torch.Tensor, ret: torch.Tensor, compat_value_bug: bool, S: int) -> torch.Tensor:
    """Experience-only normalisers (device tensor, no host sync):
    [1/n_valid, 1/total_sel, 1/n_sel[enum,x,y,target] (0 if none), ΣG_last, 0]."""
    N, A = actions.shape
    col = actions.sum(0, dtype=torch.float32)                   # (A,)
    nsel = torch.stack([col[0:3].sum(), col[3:12].sum(), col[12:21].sum(), col[21:].sum()])
    n_valid = (actions.amax(1) > 0).sum().to(torch.float32)
    total = nsel.sum()

    def inv(x):
        return torch.where(x > 0, 1.0 / x.clamp_min(1.0), torch.zeros_like(x))
    g_last = ret.view(-1, S)[-1].sum() if compat_value_bug else torch.zeros((), device=ret.device)
    return torch.cat([inv(n_valid).view(1), inv(total).view(1), inv(nsel), g_last.view(1),
                      torch.zeros(1, device=ret.device)]).contiguous()


def assemble_loss(part: torch.Tensor, norms: torch.Tensor, cfg, ret: torch.Tensor, N: int, S: int):
    """Loss scalar + metrics from the kernel's summed partials. The returned loss carries the gradient through
    ``part[15]`` (an always-zero slot): d loss / d part[15] = 1, so the custom backward receives the upstream
    gradient of the scalar loss there and scales its precomputed ∂L/∂inputs by it."""
    algo = 0 if cfg.algo == 'ppo' else 1
    B = N // S
    ent_h = part[2:6] * norms[2:6]
    entropy = ent_h.sum()
    if algo == 0:
        policy_loss = -part[0] * norms[0]
        value_loss = cfg.vf_coef * part[1] * norms[0]
        entropy_loss = -cfg.entropy_coef * entropy
        advantage = part[8] * norms[0]
    else:
        policy_loss = part[0] * norms[1]
        entropy_loss = -cfg.entropy_coef * entropy if cfg.entropy_coef > 0 else torch.zeros_like(entropy)
        if cfg.vf_coef > 0 and cfg.compat_value_bug:
            g_last = ret.view(-1, S)[-1]
            sG, sG2 = g_last.sum(), (g_last * g_last).sum()
            value_loss = cfg.vf_coef * (S * part[10] - 2 * part[9] * sG + N * sG2) / (B * S * S)
            advantage = part[9] / N - sG / S
        elif cfg.vf_coef > 0:
            value_loss = cfg.vf_coef * part[1] / N
            advantage = part[8] / N
        else:
            value_loss = torch.zeros_like(entropy)
            advantage = part[8] / N
    loss_value = (policy_loss + value_loss + entropy_loss).detach()
    loss = loss_value + (part[15] - part[15].detach())
    metrics = {'loss': loss_value, 'policy_loss': policy_loss.detach(), 'entropy_loss': entropy_loss.detach(),
               'advantage_loss': value_loss.detach(), 'entropy': entropy.detach(), 'advantage': advantage.detach()}
    if algo == 0:
        metrics['approx_kl'] = (part[6] * norms[0]).detach()
        metrics['clipfrac'] = (part[7] * norms[0]).detach()
    for k, e in zip(['enum', 'x', 'y', 'target_unit'], ent_h):
        metrics[f'entropy/{k}'] = e.detach()
    return loss, metrics


class _HeadsLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xh, wcat, bcat, emb, actions, masks, adv, ret, logp_old, nret, norms, algo, compat_value_bug,
                S, B, clip_eps, ent_coef, vf_coef):
        C = require()
        N = xh.shape[0]
        x16 = xh.to(torch.bfloat16)
        w16 = wcat.detach().to(torch.bfloat16)
        z = torch.mm(x16, w16.t(), out_dtype=torch.float32) + bcat.detach()
        dz, dtl, part, logp = C.heads_loss(z, emb.contiguous(), actions, masks, adv, ret, logp_old, nret, norms,
                                           algo, compat_value_bug, S, B, clip_eps, ent_coef, vf_coef)
        ctx.save_for_backward(dz, dtl, z, x16, w16)
        ctx.mark_non_differentiable(part, logp, z)
        return part.sum(0), logp, z

    @staticmethod
    def backward(ctx, gpart, _glogp, _gz):
        dz, dtl, z, x16, w16 = ctx.saved_tensors
        # The loss is a fixed linear functional of `part` assembled by the caller, which passes its weight
        # through gpart[15] (an unused slot) — see heads_loss(): loss = Σ part·coef, coef[15] = 1 marks it.
        g = gpart[15]
        dZ = dz * g
        d16 = dZ.to(torch.bfloat16)
        dxh = torch.mm(d16, w16, out_dtype=torch.float32)
        dw = torch.mm(d16.t(), x16, out_dtype=torch.float32)
        db = dZ.sum(0)
        demb = ((dtl * g).unsqueeze(-1) * z[:, :Q].unsqueeze(1)).to(torch.bfloat16)
        return (dxh, dw, db, demb) + (None,) * 14


def heads_loss(xh: torch.Tensor, wcat: torch.Tensor, bcat: torch.Tensor, emb: torch.Tensor,
               batch: Dict[str, torch.Tensor], cfg, S: int):
    """Returns (loss scalar, metrics dict of device scalars, per-row joint logp)."""
    N = xh.shape[0]
    actions = batch['actions'].reshape(N, -1).contiguous()
    masks = batch['masks'].reshape(N, -1).contiguous()
    algo = 0 if cfg.algo == 'ppo' else 1
    ret = batch['ret'].reshape(N).float().contiguous()
    norms = batch_norms(actions, ret, cfg.compat_value_bug and algo == 1, S)
    zeros = torch.zeros(N, device=xh.device)
    adv = batch['adv'].reshape(N).contiguous() if 'adv' in batch else zeros
    lpo = batch['logp_old'].reshape(N).contiguous() if 'logp_old' in batch else zeros
    nret = batch['norm_ret'].reshape(N).contiguous() if 'norm_ret' in batch else zeros
    B = N // S
    part, logp, z = _HeadsLoss.apply(xh, wcat, bcat, emb, actions, masks, adv, ret, lpo, nret, norms, algo,
                                     bool(cfg.compat_value_bug), S, B, float(cfg.clip_eps), float(cfg.entropy_coef),
                                     float(cfg.vf_coef))
    loss, metrics = assemble_loss(part, norms, cfg, ret, N, S)
    return loss, metrics, logp
