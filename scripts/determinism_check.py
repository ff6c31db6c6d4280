#!/usr/bin/env python3
"""Run-to-run determinism of the fused learner step: the same minibatch through two fresh learners from the same
weights must give bitwise-identical gradients (every reduction in the kernels is fixed-order). Prints the tensors
that differ per (preset, precision, B, S)."""
import copy
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402


def grads(pol, batch, prec, direct):
    L = Learner(copy.deepcopy(pol), LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01), device='cuda',
                backend='fused', dp=False, precision=prec)
    if direct:
        L.train_step(batch)
        torch.cuda.synchronize()
        return {'flat': L.flat.flat.detach().clone()}
    L.dp.zero_grad()
    loss, _ = L.loss(batch)
    loss.backward()
    torch.cuda.synchronize()
    return {n: p.grad.detach().clone() for n, p in zip(L.flat.names, L.flat.params) if p.grad is not None}


bad = 0
for preset, prec, B, S in [('lstm128', 'fp32-exact', 2, 48), ('lstm128', 'fp32', 2, 48), ('lstm512', 'fp32-exact', 8, 280),
                           ('lstm512', 'fp32-exact', 16, 140), ('lstm128', 'fp32-exact', 4, 96)]:
    torch.manual_seed(0)
    cfg = get_config(preset)
    pol = Policy(cfg).cuda()
    batch = make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=3)
    for direct in (False, True):
        a = grads(pol, batch, prec, direct)
        b = grads(pol, batch, prec, direct)
        diff = [n for n in a if not torch.equal(a[n], b[n])]
        print(f'{preset} {prec} B={B} S={S} direct={direct}: {"OK" if not diff else "DIFFER " + str(diff[:8])}',
              flush=True)
        bad += bool(diff)
sys.exit(1 if bad else 0)
