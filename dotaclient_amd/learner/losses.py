"""Policy-gradient losses, written densely (mask-weighted sums instead of ``masked_select``).

Two objectives:

* :func:`vpg_loss` — the reference's live objective (optimizer.py:602-672): per-head masked log-softmax,
  ``−log p · R̂`` on the selected one-hot actions averaged over all selections of all heads, per-head entropy
  over valid entries divided by that head's selection count, and ``vf_coef · mean((V − G)²)``. With
  ``compat_value_bug=True`` the value target is the *last* sequence's returns broadcast to (B,S,S) exactly as
  optimizer.py:603 does; otherwise it is the per-sample return.
* :func:`ppo_loss` — the north-star clipped surrogate (the reference's commented-out code at optimizer.py:632-639,
  ε = ``e_clip`` = 0.1 at optimizer.py:239) on the joint log-probability of the sampled multi-head action, a value
  loss against GAE returns and the same entropy bonus.

The dense form is deterministic and CUDA/HIP-graph capturable (no data-dependent shapes). The fused
HIP kernel ``heads_loss`` (ops/csrc/heads_loss.hip) computes exactly these quantities and their gradients; these
functions are its oracle.
"""
from __future__ import annotations

from typing import Dict

import torch

from ..models.policy import masked_log_softmax


def split_heads(flat: torch.Tensor, counts: Dict[str, int]) -> Dict[str, torch.Tensor]:
    out, acc = {}, 0
    for k, n in counts.items():
        out[k] = flat[..., acc:acc + n]
        acc += n
    return out


def head_terms(logits: Dict[str, torch.Tensor], actions: Dict[str, torch.Tensor], masks: Dict[str, torch.Tensor],
               stable: bool = True):
    """Per head: log-probs, selected log-prob (B,S), selection count, entropy-sum."""
    out = {}
    for key, lg in logits.items():
        m = masks[key].bool()
        a = actions[key].to(lg.dtype)
        logp = masked_log_softmax(lg, m, dim=-1, stable=stable)
        sel_logp = (logp * a).sum(-1)                     # (B,S): log-prob of the chosen entry (0 if none)
        n_sel = a.sum()
        p = torch.exp(logp) * m
        ent_sum = -(p * torch.where(m, logp, torch.zeros_like(logp))).sum()
        out[key] = (logp, sel_logp, n_sel, ent_sum)
    return out


def _entropies(terms) -> Dict[str, torch.Tensor]:
    ents = {}
    for key, (_, _, n_sel, ent_sum) in terms.items():
        ents[key] = torch.where(n_sel > 0, ent_sum / n_sel.clamp_min(1), torch.zeros_like(ent_sum))
    return ents


def vpg_loss(logits: Dict[str, torch.Tensor], values: torch.Tensor, actions: Dict[str, torch.Tensor],
             masks: Dict[str, torch.Tensor], norm_returns: torch.Tensor, returns: torch.Tensor,
             entropy_coef: float, vf_coef: float, compat_value_bug: bool = False, stable: bool = True):
    """Reference VPG objective. ``norm_returns``/``returns`` are (B,S). Returns (loss, metrics dict)."""
    terms = head_terms(logits, actions, masks, stable=stable)
    total_sel = sum(t[2] for t in terms.values())
    pg_sum = sum((-t[1] * norm_returns).sum() for t in terms.values())
    policy_loss = pg_sum / total_sel
    ents = _entropies(terms)
    zero = torch.zeros((), device=values.device, dtype=values.dtype)
    if compat_value_bug:
        advantage = values - returns[-1]          # (B,S,1) - (S,) → (B,S,S), optimizer.py:603
    else:
        advantage = values.squeeze(-1) - returns
    entropy = torch.stack(list(ents.values())).sum()
    entropy_loss = -entropy_coef * entropy if entropy_coef > 0 else zero
    advantage_loss = vf_coef * advantage.pow(2).mean() if vf_coef > 0 else zero
    loss = policy_loss + entropy_loss + advantage_loss
    metrics = {'loss': loss, 'policy_loss': policy_loss, 'entropy_loss': entropy_loss,
               'advantage_loss': advantage_loss, 'advantage': advantage.mean(), 'entropy': entropy}
    for k, v in ents.items():
        metrics[f'entropy/{k}'] = v
    return loss, metrics


def ppo_loss(logits: Dict[str, torch.Tensor], values: torch.Tensor, actions: Dict[str, torch.Tensor],
             masks: Dict[str, torch.Tensor], advantages: torch.Tensor, returns: torch.Tensor,
             logp_old: torch.Tensor, clip_eps: float, entropy_coef: float, vf_coef: float, stable: bool = True,
             offpolicy: str = 'clip'):
    """Clipped-surrogate PPO on the joint (summed over sampled heads) log-probability. All per-step tensors (B,S).

    ``offpolicy='tis'``: the policy term is the off-policy policy gradient with the truncated importance weight
    w = min(1, π/π_old) held constant (V-trace style, for replayed experience): value −mean(w·A), gradient
    −mean(w·A·∇log π); ``clipfrac`` then counts the truncated rows (π > π_old)."""
    terms = head_terms(logits, actions, masks, stable=stable)
    logp = sum(t[1] for t in terms.values())
    valid = sum(actions[k].sum(-1) for k in actions).gt(0).to(logp.dtype)   # padded steps select nothing
    n_valid = valid.sum().clamp_min(1.0)
    log_ratio = logp - logp_old
    ratio = torch.exp(log_ratio)
    if offpolicy == 'tis':
        w = ratio.detach().clamp(max=1.0)
        policy_loss = -(w * advantages * (1.0 + logp - logp.detach()) * valid).sum() / n_valid
    else:
        surr1 = ratio * advantages
        surr2 = torch.clamp(ratio, 1.0 - clip_eps, 1.0 + clip_eps) * advantages
        policy_loss = -(torch.minimum(surr1, surr2) * valid).sum() / n_valid
    v = values.squeeze(-1)
    if vf_coef > 0:
        value_loss = vf_coef * ((v - returns).pow(2) * valid).sum() / n_valid
    else:   # keep the value head out of the graph (reference sparse-param semantics, optimizer.py:667-670)
        value_loss = torch.zeros((), device=v.device, dtype=v.dtype)
    ents = _entropies(terms)
    entropy = torch.stack(list(ents.values())).sum()
    entropy_loss = -entropy_coef * entropy
    loss = policy_loss + value_loss + entropy_loss
    with torch.no_grad():
        approx_kl = ((-log_ratio) * valid).sum() / n_valid
        hit = (ratio > 1.0) if offpolicy == 'tis' else ((ratio - 1.0).abs() > clip_eps)
        clipfrac = (hit.to(logp.dtype) * valid).sum() / n_valid
    metrics = {'loss': loss, 'policy_loss': policy_loss, 'entropy_loss': entropy_loss, 'advantage_loss': value_loss,
               'advantage': (advantages * valid).sum() / n_valid, 'entropy': entropy, 'approx_kl': approx_kl,
               'clipfrac': clipfrac}
    for k, e in ents.items():
        metrics[f'entropy/{k}'] = e
    return loss, metrics


def sampled_logp(logits: Dict[str, torch.Tensor], actions: Dict[str, torch.Tensor], masks: Dict[str, torch.Tensor],
                 stable: bool = True) -> torch.Tensor:
    """Joint log-prob of the sampled multi-head action (behaviour policy's ``logp_old``)."""
    terms = head_terms(logits, actions, masks, stable=stable)
    return sum(t[1] for t in terms.values())
