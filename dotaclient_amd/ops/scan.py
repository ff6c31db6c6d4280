"""Returns / advantages over a batch of rollouts on the device (``csrc/scan.hip``) plus its CPU reference.

All rollouts of a learner iteration are concatenated, each padded to a multiple of ``seq_len``; segment ``s`` spans
rows ``off[s]:off[s+1]`` of which the first ``seglen[s]`` are real steps. ``compute_returns`` returns per-row
``ret`` / ``adv`` / ``norm`` and per-segment ``stats`` (mean, population std of the returns), and advances the
per-team EMA state ``ema`` (``(n_keys, 3)`` = mean, std, initialised) in rollout order:

* ``mode='discount'`` — reference VPG path: ``G_t = r_t + γ G_{t+1}`` over the whole padded segment
  (optimizer.py:52-53, 382), EMA(0.99) update with the segment's (mean, std) (optimizer.py:335-343) and the normalised
  return ``(G − μ)/(σ + eps)`` (optimizer.py:185-186) in ``norm`` (= ``adv``).
* ``mode='gae'`` — PPO path: GAE(γ, λ) over the valid prefix, ``ret = adv + V``, zeros in the padded tail; the EMA is
  updated with the statistics of ``ret[:T]`` (metrics only); ``norm`` = ``adv``.
* ``mode='vtrace'`` — off-policy PPO path (Espeholt et al. 2018, V-trace): ``val`` are the LEARNER's values (its
  forward at the iteration's weights), ``lr`` = log π − log μ per row (learner vs behaviour log-prob of the sampled
  action); ρ_t = min(ρ̄, e^lr), c_t = λ·min(c̄, e^lr), A_t = ρ_t·δ_t + γ·c_t·A_{t+1}; ``ret = A + V`` is the V-trace
  value target and ``adv`` = A the off-policy-corrected GAE. Equal to ``gae`` at lr = 0.

On a GPU tensor the HIP kernel runs (and the extension is required); on CPU the torch reference below runs — it is
also the oracle of the GPU tests.
"""
from __future__ import annotations

from typing import Dict

import torch

from ..constants import EPS

MODES = {'discount': 0, 'gae': 1, 'vtrace': 2}


def _reference(rew, val, off, seglen, boot, done, keys, ema, mode, gamma, lam, factor, eps, normalize, lr=None,
               rho_bar=1.0, c_bar=1.0):
    L = rew.shape[0]
    r = rew.double().sum(1)
    v = val.double() if mode >= 1 else None
    w = torch.exp(lr.double().clamp(max=30.0)) if mode == 2 else None
    ret = torch.zeros(L, dtype=torch.float64)
    adv = torch.zeros(L, dtype=torch.float64)
    nseg = seglen.numel()
    stats = torch.zeros(nseg, 2, dtype=torch.float64)
    for s in range(nseg):
        a, b = int(off[s]), int(off[s + 1])
        T = min(int(seglen[s]), b - a)
        if mode == 1:
            acc, nv = 0.0, (0.0 if bool(done[s]) else float(boot[s]))
            for t in range(T - 1, -1, -1):
                delta = float(r[a + t]) + gamma * nv - float(v[a + t])
                acc = delta + gamma * lam * acc
                adv[a + t] = acc
                nv = float(v[a + t])
            ret[a:a + T] = adv[a:a + T] + v[a:a + T]
            seg = ret[a:a + T]
        elif mode == 2:
            acc, nv = 0.0, (0.0 if bool(done[s]) else float(boot[s]))
            for t in range(T - 1, -1, -1):
                rho, cw = min(rho_bar, float(w[a + t])), min(c_bar, float(w[a + t]))
                delta = float(r[a + t]) + gamma * nv - float(v[a + t])
                acc = rho * delta + gamma * lam * cw * acc        # A_t = v_t − V_t
                adv[a + t] = acc
                ret[a + t] = acc + float(v[a + t])
                nv = float(v[a + t])
            seg = ret[a:a + T]
        else:
            acc = 0.0
            for t in range(b - a - 1, -1, -1):
                acc = float(r[a + t]) + gamma * acc
                ret[a + t] = acc
            seg = ret[a:b]
        if seg.numel():
            stats[s, 0] = seg.mean()
            stats[s, 1] = seg.std(unbiased=False)
    ema_new = ema.clone().double()
    norm = adv.clone() if mode >= 1 else torch.zeros(L, dtype=torch.float64)
    for s in range(nseg):
        k = int(keys[s])
        if ema_new[k, 2] == 0:
            ema_new[k, 0], ema_new[k, 1], ema_new[k, 2] = stats[s, 0], stats[s, 1], 1.0
        else:
            ema_new[k, 0] = ema_new[k, 0] * factor + stats[s, 0] * (1 - factor)
            ema_new[k, 1] = ema_new[k, 1] * factor + stats[s, 1] * (1 - factor)
        if mode == 0 and normalize:
            a, b = int(off[s]), int(off[s + 1])
            norm[a:b] = (ret[a:b] - ema_new[k, 0]) / (ema_new[k, 1] + eps)
    if mode == 0:
        adv = norm if normalize else ret.clone()
    ema.copy_(ema_new.to(ema.dtype))
    f = torch.float32
    return {'ret': ret.to(f), 'adv': adv.to(f), 'norm': norm.to(f), 'stats': stats.to(f)}


def compute_returns(rew: torch.Tensor, val, off, seglen, boot, done, keys, ema: torch.Tensor, mode: str = 'gae',
                    gamma: float = 0.98, lam: float = 0.95, factor: float = 0.99, eps: float = EPS,
                    normalize: bool = True, lr=None, rho_bar: float = 1.0,
                    c_bar: float = 1.0) -> Dict[str, torch.Tensor]:
    """``rew`` (L, K) f32 sub-rewards (summed per row), ``val`` (L,) f32 or None; per-segment metadata as host
    int32/float32/uint8 tensors or sequences; ``ema`` (n_keys, 3) f32 on the same device as ``rew`` (updated in
    place); ``lr`` (L,) f32 log ratios for ``mode='vtrace'``."""
    m = MODES[mode]
    off = torch.as_tensor(off, dtype=torch.int32).contiguous()
    seglen = torch.as_tensor(seglen, dtype=torch.int32).contiguous()
    keys = torch.as_tensor(keys, dtype=torch.int32).contiguous()
    boot = torch.as_tensor(boot, dtype=torch.float32).contiguous()
    done = torch.as_tensor(done, dtype=torch.uint8).contiguous()
    if m >= 1 and val is None:
        raise ValueError('gae needs values')
    if m == 2 and lr is None:
        raise ValueError('vtrace needs the per-row log ratios')
    if rew.device.type != 'cuda':
        return _reference(rew, val, off, seglen, boot, done, keys, ema, m, gamma, lam, factor, eps, normalize, lr,
                          rho_bar, c_bar)
    from . import require
    C = require()
    L = rew.shape[0]
    rew = rew.float().contiguous()
    v = val.float().contiguous() if m >= 1 else rew.new_empty(0)
    ret = torch.empty(L, device=rew.device)
    adv = torch.empty(L, device=rew.device) if m >= 1 else ret.new_empty(L)
    norm = torch.empty(L, device=rew.device) if m == 0 else adv
    stats = torch.empty(seglen.numel(), 2, device=rew.device)
    C.returns_scan(rew, v, off, seglen, boot, done, keys, ema, ret, adv, norm, stats, m, bool(normalize and m == 0),
                   float(gamma), float(lam), float(factor), float(eps),
                   lr.float().contiguous() if m == 2 else None, float(rho_bar), float(c_bar))
    if m == 0:
        adv = norm if normalize else ret
    return {'ret': ret, 'adv': adv, 'norm': norm, 'stats': stats}


def vtrace_step(values: torch.Tensor, lp: torch.Tensor, mu: torch.Tensor, vt: torch.Tensor, B: int, S: int,
                gamma: float = 0.98, lam: float = 0.95, rho_bar: float = 1.0, c_bar: float = 1.0, z=None,
                vcol: int = 149):
    """V-trace inside the learner step over a minibatch's TIME-MAJOR rows (r = t·B + b): ``values`` (N,) the step's
    own values, ``lp`` (N,) its log-probs of the recorded actions, ``mu`` (N,) the actor's behaviour log-probs, ``vt``
    (N, 4) = {reward, bootstrap, valid, last} (``last``: the episode segment ends at this row inside its sequence; its
    successor value is ``bootstrap``). ρ_t = min(ρ̄, e^{lp − mu}), A_t = ρ_t·δ_t + γλ·min(c̄, e^{lp − mu})·A_{t+1};
    returns (adv = A, ret = A + V on valid rows, stats (B, 4) = Σ valid {ρ, [w > ρ̄], mu − lp, 1}). GPU with ``z``
    (the heads logits, value in column ``vcol``): the HIP kernel (ops/csrc/scan.hip vtrace_step_kernel); otherwise
    this torch reference (its oracle)."""
    if z is not None and z.is_cuda:
        from . import require
        return tuple(require().vtrace_step(z, vcol, lp.contiguous(), mu.contiguous(), vt.contiguous(), B, S,
                                           float(gamma), float(lam), float(rho_bar), float(c_bar)))
    V = values.reshape(S, B).double()
    dl = (lp - mu).reshape(S, B).double()
    v4 = vt.reshape(S, B, 4).double()
    w = torch.exp(dl.clamp(max=30.0))
    rho, cw = w.clamp(max=rho_bar), w.clamp(max=c_bar)
    valid = v4[..., 2] > 0
    last = v4[..., 3] > 0
    last[S - 1] = True
    nextV = torch.cat([V[1:], torch.zeros(1, B, dtype=V.dtype)], 0)
    nextV = torch.where(last, v4[..., 1], nextV)
    d = torch.where(valid, rho * (v4[..., 0] + gamma * nextV - V), torch.zeros_like(V))
    k = torch.where(valid & ~last, gamma * lam * cw, torch.zeros_like(V))
    A = torch.zeros(S, B, dtype=torch.float64)
    acc = torch.zeros(B, dtype=torch.float64)
    for t in range(S - 1, -1, -1):
        acc = d[t] + k[t] * acc
        A[t] = acc
    ret = torch.where(valid, A + V, torch.zeros_like(V))
    vf = valid.double()
    stats = torch.stack([(rho * vf).sum(0), ((w > rho_bar * (1 + 1e-6)).double() * vf).sum(0), (-dl * vf).sum(0),
                         vf.sum(0)], 1)
    f = torch.float32
    return A.reshape(-1).to(f), ret.reshape(-1).to(f), stats.to(f)
