"""heads_loss kernel (F32, PRECISE) vs float64 autograd of the same loss on the same fp32 logits: ∂L/∂z per head.
Isolates the fused heads/loss pass of the fp32-exact learner from the rest of the step. python scripts/heads_diag.py"""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.constants import LAYOUT_1V1  # noqa: E402
from dotaclient_amd.learner.losses import ppo_loss, split_heads, vpg_loss  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.ops.heads import batch_norms  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


C = ops.require()
B, S = 8, 1400
N = B * S
lay = LAYOUT_1V1
U = lay.max_units
bt = make_batch(B, S, lay, 512, device='cuda', seed=3)
g = torch.Generator(device='cuda').manual_seed(0)
z = torch.randn(N, 160, device='cuda', generator=g)
emb = torch.randn(N, U, 128, device='cuda', generator=g) * 0.1
act = bt['actions'].reshape(N, -1).contiguous()
msk = bt['masks'].reshape(N, -1).contiguous()
adv = bt['adv'].reshape(N).float().contiguous()
ret = bt['ret'].reshape(N).float().contiguous()
lpo = bt['logp_old'].reshape(N).float().contiguous()
nret = bt['norm_ret'].reshape(N).float().contiguous()
for algo in ('ppo', 'vpg'):
    a = 0 if algo == 'ppo' else 1
    norms = batch_norms(act, ret, False, S)
    dz, dtl, part, lp = C.heads_loss(z, emb, act, msk, adv, ret, lpo, nret, norms, a, False, S, B, 0.2, 0.01, 0.5,
                                     dz_bf16=False, precise=True)
    res = {}
    for dt in (torch.float64, torch.float32):
        zz = z.to(dt).requires_grad_()
        ee = emb.to(dt)
        logits = {'enum': zz[:, 128:131], 'x': zz[:, 131:140], 'y': zz[:, 140:149],
                  'target_unit': torch.einsum('nd,nud->nu', zz[:, :128], ee)}
        counts = lay.action_counts()
        acts, msks = split_heads(act, counts), split_heads(msk, counts)
        if a == 0:
            loss, _ = ppo_loss(logits, zz[:, 149:150], acts, msks, adv.to(dt), ret.to(dt), lpo.to(dt), 0.2, 0.01, 0.5)
        else:
            loss, _ = vpg_loss(logits, zz[:, 149:150], acts, msks, nret.to(dt), ret.to(dt), 0.01, 0.5)
        res[dt] = torch.autograd.grad(loss, zz)[0]
        if dt == torch.float64:
            from dotaclient_amd.learner.losses import head_terms
            lp64 = sum(t[1] for t in head_terms({k: v.detach() for k, v in logits.items()}, acts, msks).values())
    d64, d32 = res[torch.float64], res[torch.float32]
    print(algo, 'logp rel', rel(lp, lp64), 'max abs', float((lp.double() - lp64).abs().max()), flush=True)
    if a == 0:
        r64 = torch.exp(lp64 - lpo.double())
        A = adv.double()
        print('   ratio range', float(r64.min()), float(r64.max()), 'min |r-1.2| (A>0)',
              float((r64 - 1.2).abs()[A > 0].min()), 'min |r-0.8| (A<0)', float((r64 - 0.8).abs()[A < 0].min()))
    for name, sl in (('q', slice(0, 128)), ('enum', slice(128, 131)), ('x', slice(131, 140)), ('y', slice(140, 149)),
                     ('value', slice(149, 150))):
        print(f'   dz {name:6s} kernel {rel(dz[:, sl], d64[:, sl]):.3e}  torch-fp32 {rel(d32[:, sl], d64[:, sl]):.3e}',
              flush=True)
        if name == 'enum':
            e = (dz[:, sl].double() - d64[:, sl]).abs().sum(1)
            top = torch.topk(e, 5)
            print('      worst rows', top.indices.tolist(), [f'{v:.2e}' for v in top.values.tolist()],
                  'row |dz|', [f'{float(d64[i, sl].abs().sum()):.2e}' for i in top.indices.tolist()], flush=True)
