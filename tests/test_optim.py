"""FlatAdam (fused clip + Adam over the flat buffer) vs torch.optim.Adam + clip_grad_norm_ (reference
optimizer.py:281, 680-681)."""
import pytest
import torch

from dotaclient_amd.learner.optim import FlatAdam
from dotaclient_amd.models.policy import Policy
from dotaclient_amd.parallel.dp import FlatParams


def _grads(model, seed):
    g = torch.Generator().manual_seed(seed)
    return [torch.randn(p.shape, generator=g) * (0.5 + i % 3) for i, p in enumerate(model.parameters())]


def _run_reference(model, grads_seq, lr, max_norm, skip=()):
    opt = torch.optim.Adam(model.parameters(), lr=lr)
    params = list(model.parameters())
    for grads in grads_seq:
        for i, (p, g) in enumerate(zip(params, grads)):
            p.grad = None if i in skip else g.clone()
        torch.nn.utils.clip_grad_norm_([p for p in params if p.grad is not None], max_norm)
        opt.step()


def _run_flat(model, grads_seq, lr, max_norm, skip=(), device='cpu', kernels=False, ranks=1):
    """ranks > 1: the gradient buffer holds the SUM over that many identical ranks (what DataParallel.sync(
    scale=False) leaves) and the optimizer takes the has-grad average itself (step(divide=True))."""
    model = model.to(device)
    flat = FlatParams(model, device=device)
    opt = FlatAdam(flat, lr=lr, max_grad_norm=max_norm, use_kernels=kernels)
    counts = torch.full((len(flat.params),), float(ranks), device=device)
    for i in skip:
        counts[i] = 0
    for grads in grads_seq:
        flat.zero_grad()
        for i, (p, g) in enumerate(zip(flat.params, grads)):
            if i not in skip:
                p.grad.copy_(g.to(device) * ranks)
        opt.step(counts, divide=ranks > 1)
    return model


@pytest.mark.parametrize('skip', [(), (3, 28)])
def test_flat_adam_matches_torch(skip):
    torch.manual_seed(0)
    a = Policy('compat')
    b = Policy('compat')
    b.load_state_dict(a.state_dict())
    seq = [_grads(a, s) for s in range(4)]
    _run_reference(a, seq, 1e-3, 0.5, skip)
    _run_flat(b, seq, 1e-3, 0.5, skip)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.gpu
def test_adam_kernel_matches_reference(gpu_ops):
    torch.manual_seed(0)
    a = Policy('lstm512')
    b = Policy('lstm512')
    b.load_state_dict(a.state_dict())
    seq = [_grads(a, s) for s in range(3)]
    _run_flat(a, seq, 1e-3, 0.5, skip=(5,))
    b = _run_flat(b, seq, 1e-3, 0.5, skip=(5,), device='cuda', kernels=True)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb.cpu(), rtol=1e-5, atol=2e-6, msg=n)


@pytest.mark.parametrize('skip', [(), (3, 28)])
def test_flat_adam_divide_equals_presummed_average(skip):
    """step(divide=True) on rank SUMS == step() on the already averaged gradients (the DP fold)."""
    torch.manual_seed(0)
    a = Policy('compat')
    b = Policy('compat')
    b.load_state_dict(a.state_dict())
    seq = [_grads(a, s) for s in range(3)]
    _run_flat(a, seq, 1e-3, 0.5, skip)
    _run_flat(b, seq, 1e-3, 0.5, skip, ranks=3)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb, rtol=1e-5, atol=1e-6, msg=n)


@pytest.mark.gpu
def test_adam_kernel_divide_mode(gpu_ops):
    torch.manual_seed(0)
    a = Policy('lstm512')
    b = Policy('lstm512')
    b.load_state_dict(a.state_dict())
    seq = [_grads(a, s) for s in range(3)]
    _run_flat(a, seq, 1e-3, 0.5, skip=(5,))
    b = _run_flat(b, seq, 1e-3, 0.5, skip=(5,), device='cuda', kernels=True, ranks=4)
    for (n, pa), pb in zip(a.named_parameters(), b.parameters()):
        torch.testing.assert_close(pa, pb.cpu(), rtol=1e-5, atol=2e-6, msg=n)


def test_adam_state_remaps_across_flat_layouts():
    """the flat layout (header + offsets) is recorded with the moments; a state written under another
    layout is remapped parameter by parameter, and an unversioned state of the wrong length is rejected."""
    from dotaclient_amd.models.policy import get_config
    torch.manual_seed(0)
    model = Policy(get_config('lstm128'))
    flat = FlatParams(model)
    opt = FlatAdam(flat, use_kernels=False)
    for i in range(len(flat.params)):
        o, n = flat.offsets[i], flat.numel[i]
        opt.exp_avg[o:o + n] = float(i + 1)
        opt.exp_avg_sq[o:o + n] = float(10 * (i + 1))
    sd = opt.state_dict()
    # the same moments under a different layout (header 0, parameters packed): remapped by parameter
    old = {'header': 0, 'offsets': [], 'numel': list(sd['layout']['numel'])}
    off = 0
    for n in old['numel']:
        old['offsets'].append(off)
        off += n
    legacy = dict(sd, layout=old, exp_avg=torch.cat([torch.full((n,), float(i + 1)) for i, n in enumerate(old['numel'])]),
                  exp_avg_sq=torch.cat([torch.full((n,), float(10 * (i + 1))) for i, n in enumerate(old['numel'])]))
    opt2 = FlatAdam(FlatParams(Policy(get_config('lstm128'))), use_kernels=False)
    opt2.load_state_dict(legacy)
    torch.testing.assert_close(opt2.exp_avg, opt.exp_avg)
    torch.testing.assert_close(opt2.exp_avg_sq, opt.exp_avg_sq)
    unversioned = {k: v for k, v in legacy.items() if k != 'layout'}
    with pytest.raises(ValueError, match='older layout'):
        opt2.load_state_dict(unversioned)


def _nonfinite_case(device, kernels):
    torch.manual_seed(0)
    model = Policy('compat').to(device)
    flat = FlatParams(model, device=device)
    opt = FlatAdam(flat, lr=1e-3, max_grad_norm=0.5, use_kernels=kernels)
    counts = torch.ones(len(flat.params), device=device)
    for p in flat.params:
        p.grad.normal_()
    opt.step(counts)
    opt.check_nonfinite()
    before = (flat.flat.clone(), opt.exp_avg.clone(), opt.steps.clone())
    flat.params[3].grad[0] = float('inf')
    opt.step(counts)
    assert not bool(torch.isfinite(opt.last_grad_norm))
    # nothing applied and Adam's bias-correction clock did not move
    assert torch.equal(flat.flat, before[0]) and torch.equal(opt.exp_avg, before[1])
    assert torch.equal(opt.steps, before[2])
    with pytest.raises(FloatingPointError):
        opt.check_nonfinite()
    opt.check_nonfinite()                      # the flag was cleared by the raise
    flat.params[3].grad[0] = 0.0
    opt.step(counts)
    assert torch.equal(opt.steps, before[2] + 1)


def test_nonfinite_step_is_skipped_and_raises_cpu():
    _nonfinite_case('cpu', False)


@pytest.mark.gpu
def test_nonfinite_step_is_skipped_and_raises_gpu(gpu_ops):
    _nonfinite_case('cuda', True)


def test_learner_grad_norm_is_per_step():
    """Every step's returned grad_norm is its own tensor (the optimizer's norm buffer is rewritten by the
    next step, so a list of references would hold only the last value)."""
    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.learner.synthetic import make_batch
    from dotaclient_amd.models.policy import get_config
    cfg = get_config('lstm128')
    torch.manual_seed(0)
    L = Learner(Policy(cfg), LossConfig(algo='ppo'), device='cpu', backend='torch')
    ms = [L.train_step(make_batch(2, 8, cfg.layout, cfg.hidden, device='cpu', seed=s)) for s in range(3)]
    vals = [float(m['grad_norm']) for m in ms]
    assert len({m['grad_norm'].data_ptr() for m in ms}) == 3
    assert float(L.opt.last_grad_norm) == vals[-1] and len(set(vals)) == 3
