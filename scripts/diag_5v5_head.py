#!/usr/bin/env python3
"""Diagnostic: where the 5v5 fp32-exact step's pointer-head gradient error comes from. Runs the fused exact step with
heads_loss wrapped to record its inputs / outputs, and a float64 evaluation with hooks on the attention output (E1),
the pointer query q and the pointer logits; prints relative errors of E1, q, the pointer logits' gradient (dtl) and
∂q (dz[:, :128]) — time-major rows on both sides."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402
from dotaclient_amd.learner.losses import ppo_loss, split_heads  # noqa: E402

B, S = 8, int(sys.argv[1]) if len(sys.argv) > 1 else 1400
if len(sys.argv) > 2 and sys.argv[2] == 'precise':       # the recurrence with libm-class activations
    import dotaclient_amd.models.pipelined as pl
    _tf, _tb = pl.team_fwd, pl.team_bwd
    pl.team_fwd = lambda *a, **k: _tf(*a, precise=True, **k)
    pl.team_bwd = lambda *a, **k: _tb(*a, precise=True, **k)
    print('recurrence: precise activations')
torch.manual_seed(0)
cfg = get_config('5v5')
pol = Policy(cfg)
p0 = copy.deepcopy(pol)
lc = LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01)
batch = make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=3)
L = Learner(pol, lc, device='cuda', backend='fused', dp=False, precision='fp32-exact')
C = L.model.C
rec = {}
orig = C.heads_loss


def wrap(zc, emb, *a, **k):
    out = orig(zc, emb, *a, **k)
    rec.update(z=zc.detach().clone(), emb=emb.detach().clone(), dz=out[0].detach().clone(), dtl=out[1].detach().clone())
    return out


C.heads_loss = wrap
L.dp.zero_grad()
loss, _ = L.loss(batch)
loss.backward()
torch.cuda.synchronize()
C.heads_loss = orig
g_f = {n: p.grad.detach().clone() for n, p in zip(L.flat.names, L.flat.params) if p.grad is not None}

# float64 with hooks
cap = {}
pol64 = p0.cuda()


def hook_e1(m, i, o):
    cap['E1'] = o
    o.retain_grad()


def hook_q(m, i, o):
    cap['q'] = o
    o.retain_grad()


pol64 = pol64.double()
_heads = pol64.heads


def heads_hook(x, ue):
    d, v = _heads(x, ue)
    d['target_unit'].retain_grad()
    cap['tl'] = d['target_unit']
    return d, v


pol64.heads = heads_hook
pol64.entity_attn.register_forward_hook(lambda m, i, o: hook_e1(m, i, o))
pol64.affine_unit_attention.register_forward_hook(lambda m, i, o: hook_q(m, i, o))
b = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
logits, values, _ = pol64.forward_packed(b['env'], b['units'], (b['h0'].unsqueeze(0), b['c0'].unsqueeze(0)))
counts = pol64.layout.action_counts()
l64, _ = ppo_loss(logits, values, split_heads(b['actions'], counts), split_heads(b['masks'], counts), b['adv'],
                  b['ret'], b['logp_old'], lc.clip_eps, lc.entropy_coef, lc.vf_coef, stable=True)
l64.backward()
g64 = {n: p.grad for n, p in pol64.named_parameters()}


def tm(x):          # (B, S, ...) → time-major rows (S·B, ...)
    return x.transpose(0, 1).reshape(S * B, *x.shape[2:])


def rel(a, b):
    return float((a.double() - b.double()).norm() / b.double().norm())


E1_64, q64 = tm(cap['E1'].detach()), tm(cap['q'].detach())
dq64 = tm(cap['q'].grad.detach())
print('E1 rel', rel(rec['emb'].view(S * B, -1, 128), E1_64))
print('q rel', rel(rec['z'][:, :128], q64))
print('dq rel', rel(rec['dz'][:, :128], dq64))
print('dq sum rel', rel(rec['dz'][:, :128].double().sum(0), dq64.double().sum(0)))
print('att bias grad rel', rel(g_f['affine_unit_attention.bias'], g64['affine_unit_attention.bias']))
# dq from the kernel's own dtl and E1 in float64 vs the kernel's dq: the kernel's accumulation error alone
dq_own = torch.einsum('nu,nud->nd', rec['dtl'].double(), rec['emb'].view(S * B, -1, 128).double())
print('dq accumulation rel (kernel vs fp64 of its own dtl, E1)', rel(rec['dz'][:, :128], dq_own))
print('dq from kernel dtl and fp64 E1 vs fp64 dq', rel(torch.einsum('nu,nud->nd', rec['dtl'].double(), E1_64), dq64))

dtl64 = tm(cap['tl'].grad.detach())
dtlk = rec['dtl'].double()
E1k = rec['emb'].view(S * B, -1, 128).double()
print('dtl rel per row', rel(dtlk, dtl64))
lk = torch.einsum('nd,nud->nu', rec['z'][:, :128].double(), E1k)
print('pointer logits rel (kernel q, E1 in fp64 vs fp64)', rel(lk, tm(cap['tl'].detach())))
dq64s = dq64.double().sum(0)
for name, dt, e in (('kernel dtl, kernel E1', dtlk, E1k), ('fp64 dtl, kernel E1', dtl64, E1k),
                    ('kernel dtl, fp64 E1', dtlk, E1_64.double()), ('fp64 dtl, fp64 E1', dtl64, E1_64.double())):
    print(f'Σ_n dq ({name}) rel', rel(torch.einsum('nu,nud->d', dt, e), dq64s))
print('cancellation Σ|dq| / |Σ dq|', float(dq64.double().abs().sum(0).norm() / dq64s.norm()))
err = rec['dz'][:, :128].double() - dq64
print('error coherence |Σ err| / Σ|err|', float(err.sum(0).norm() / err.abs().sum(0).norm()))
# dtl of the float64 loss evaluated AT the kernel's pointer logits: logits error vs heads_loss arithmetic
lg = {k: v.detach() for k, v in logits.items()}
lkb = lk.view(S, B, -1).transpose(0, 1).contiguous().requires_grad_(True)
lg['target_unit'] = lkb
lm, _ = ppo_loss(lg, values.detach(), split_heads(b['actions'], counts), split_heads(b['masks'], counts), b['adv'],
                 b['ret'], b['logp_old'], lc.clip_eps, lc.entropy_coef, lc.vf_coef, stable=True)
lm.backward()
dtl_mixed = tm(lkb.grad.detach())
print('dtl_mixed (fp64 loss at kernel logits) vs fp64 dtl', rel(dtl_mixed, dtl64), '; vs kernel dtl', rel(dtlk, dtl_mixed))
print('Σ_n dq (dtl_mixed, fp64 E1) rel', rel(torch.einsum('nu,nud->d', dtl_mixed, E1_64.double()), dq64s))
