"""Run-to-run determinism of the fused learner step (every reduction in the kernels is fixed-order): the same
minibatch through two fresh learners from the same weights gives bitwise-identical gradients and, through the direct
(graph) step, identical weights. Covers H = 128 (a team workgroup's 4 units on one of its 4 waves — the round-5
regression where the idle waves of the exact forward published other workgroups' units) and H = 512 with 1 / 2 rows
per chain. scripts/determinism_check.py is the standalone form."""
import copy

import pytest
import torch

pytestmark = pytest.mark.gpu


def _run(pol, batch, prec, direct):
    from dotaclient_amd.learner.engine import Learner, LossConfig
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


@pytest.mark.parametrize('preset,prec,B,S', [('lstm128', 'fp32-exact', 2, 48), ('lstm128', 'fp32', 4, 96),
                                             ('lstm512', 'fp32-exact', 8, 280), ('lstm512', 'fp32-exact', 16, 140)])
def test_fused_step_is_deterministic(gpu_ops, preset, prec, B, S):
    from dotaclient_amd.learner.synthetic import make_batch
    from dotaclient_amd.models.policy import Policy, get_config
    torch.manual_seed(0)
    cfg = get_config(preset)
    pol = Policy(cfg).cuda()
    batch = make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=3)
    for direct in (False, True):
        a, b = _run(pol, batch, prec, direct), _run(pol, batch, prec, direct)
        diff = [n for n in a if not torch.equal(a[n], b[n])]
        assert not diff, (direct, diff[:8])
