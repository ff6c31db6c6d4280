"""Host-side companions of the fused heads + loss kernel (ops/csrc/heads_loss.hip): the experience-only loss
normalisers (:func:`batch_norms`) and the loss / metrics assembly from the kernel's partial sums
(:func:`assemble_loss`; the learner's direct step does the same on the device, glue.hip loss_assemble). The kernel
evaluates the masked log-softmaxes, the PPO (or reference VPG) objective, entropies and the value loss for N = B·S rows
of head logits ``z = h·Wcatᵀ + bcat`` and writes ∂L/∂z and ∂L/∂(pointer logits) in the same pass.

Column layout of z / Wcat (``LDZ`` = 160): ``[q 0:128 | enum 128:131 | x 131:140 | y 140:149 | value 149 | pad]``.
"""
from __future__ import annotations

import torch

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
