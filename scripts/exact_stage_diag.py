"""Where does the fp32-exact fused step leave float64? Captures the heads-loss inputs of one fused step (the logits
z, time-major) and compares them with the float64 policy's logits, and the step's gradients per tensor.
python scripts/exact_stage_diag.py [precision]"""
import copy
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.learner.engine import Learner, LossConfig  # noqa: E402
from dotaclient_amd.learner.synthetic import make_batch  # noqa: E402
from dotaclient_amd.models.policy import Policy, get_config  # noqa: E402


def rel(a, b):
    a, b = a.double(), b.double()
    return float((a - b).norm() / (b.norm() + 1e-30))


prec = sys.argv[1] if len(sys.argv) > 1 else 'fp32-exact'
C = ops.require()
seen = {}


class Spy:
    def __getattr__(self, k):
        f = getattr(C, k)
        if k not in ('heads_loss', 'encoder_fwd', 'lstm_team_fwd'):
            return f

        def w(*a, **kw):
            out = f(*a, **kw)
            seen.setdefault(k, []).append((a, out))
            return out
        return w


torch.manual_seed(0)
B, S = 8, 1400
cfg = get_config('lstm512')
pol = Policy(cfg)
p64 = copy.deepcopy(pol).double().cuda()
lc = LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01)
L = Learner(pol, lc, device='cuda', backend='fused', dp=False, precision=prec)
L.model.C = Spy()
batch = make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=3)
L.dp.zero_grad()
loss, _ = L.loss(batch)
loss.backward()
torch.cuda.synchronize()
print('captured', {k: len(v) for k, v in seen.items()}, flush=True)
b = {k: (v.double() if v.is_floating_point() else v) for k, v in batch.items()}
with torch.no_grad():
    logits, values, _ = p64.forward_packed(b['env'], b['units'], (b['h0'].unsqueeze(0), b['c0'].unsqueeze(0)))
tm = lambda x: x.transpose(0, 1).reshape(B * S, *x.shape[2:])   # noqa: E731  (B,S,…) → time-major rows
if 'heads_loss' in seen:
    z = seen['heads_loss'][0][0][0]
    for name, sl, ref in (('enum', slice(128, 131), logits['enum']), ('x', slice(131, 140), logits['x']),
                          ('y', slice(140, 149), logits['y']), ('value', slice(149, 150), values)):
        print(f'z {name:6s} vs fp64: {rel(z[:, sl], tm(ref.reshape(B, S, -1))):.3e}', flush=True)
if 'heads_loss' in seen:
    from dotaclient_amd.ops.heads import batch_norms
    a = seen['heads_loss'][0][0]
    N = B * S
    act_t = tm(batch['actions']).reshape(N, -1)
    print('act equal', torch.equal(a[2], act_t), 'msk equal', torch.equal(a[3], tm(batch['masks']).reshape(N, -1)),
          flush=True)
    for i, k in ((4, 'adv'), (5, 'ret'), (6, 'logp_old'), (7, 'norm_ret')):
        ref = tm(batch[k].reshape(B, S)).reshape(N).float()
        print(f'{k}: max abs diff {float((a[i].float() - ref).abs().max()):.3e} dtype {a[i].dtype}', flush=True)
    nref = batch_norms(act_t.contiguous(), tm(batch['ret'].reshape(B, S)).reshape(N).float(), False, S)
    print('norms fused', a[8].tolist(), flush=True)
    print('norms ref  ', nref.tolist(), flush=True)
if 'lstm_team_fwd' in seen:
    a, kw_out = seen['lstm_team_fwd'][0]
    xp4, out = a[0], kw_out
    print('xp4 dtype', xp4.dtype, 'whh dtype', a[1].dtype, flush=True)
    with torch.no_grad():
        x, _ = p64.encode(b['env'], b['units'])
        xp = x @ p64.rnn.weight_ih_l0.t() + p64.rnn.bias_ih_l0 + p64.rnn.bias_hh_l0
        hseq, _ = p64.recurrent(x, (b['h0'].unsqueeze(0), b['c0'].unsqueeze(0)))
    H = cfg.hidden
    ref4 = xp.view(B, S, 4, H).transpose(2, 3).transpose(0, 1)          # (S, B, H, 4)
    got = xp4.double()
    bias4 = None
    for v in (list(a) + [None]):
        pass
    print('xp4 (no bias) vs fp64 x·W_ihᵀ: rel', rel(got, ref4 - (p64.rnn.bias_ih_l0 + p64.rnn.bias_hh_l0).view(4, H).t()),
          flush=True)
    hs = out[0].double()
    print('h (kernel) vs fp64 h: rel', rel(hs, hseq.transpose(0, 1)), flush=True)
if 'heads_loss' in seen and 'lstm_team_fwd' in seen:
    from tests.test_fp32_kernels import _fp64_grads
    dz = seen['heads_loss'][0][1][0].double()                      # (N, 160) time-major
    h = seen['lstm_team_fwd'][0][1][0].double().reshape(B * S, -1)  # (S·B, H) time-major rows
    mine = dz.t() @ h
    grads = {n: p.grad for n, p in zip(L.flat.names, L.flat.params)}
    _, g64 = _fp64_grads(copy.deepcopy(pol).cuda(), batch, lc)
    for nm, sl in (('affine_head_enum.weight', slice(128, 131)), ('affine_move_x.weight', slice(131, 140)),
                   ('affine_value.weight', slice(149, 150))):
        print(f'{nm}: fused grad vs fp64 {rel(grads[nm], g64[nm]):.3e}; fused vs dzᵀh(captured, fp64 sum) '
              f'{rel(grads[nm], mine[sl]):.3e}; dzᵀh(captured) vs fp64 {rel(mine[sl], g64[nm]):.3e}', flush=True)
