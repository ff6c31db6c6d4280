"""GPU actor inference kernels (fused sampling, LSTM cell) and the graph-captured batched actor vs torch fp32."""
import numpy as np
import pytest
import torch

from dotaclient_amd.models.policy import Policy, batched_action_masks, get_config, masked_log_softmax

pytestmark = pytest.mark.gpu

HEADS = (('enum', 0, 3), ('x', 3, 9), ('y', 12, 9))


def _torch_logps(z, emb, handles):
    """Per-head masked log-softmax (fp32) from the packed head logits z (N,160) and unit embeddings."""
    U = emb.shape[1]
    valid = batched_action_masks(handles)
    out = {}
    for k, o, w in HEADS:
        out[k] = masked_log_softmax(z[:, 128 + o:128 + o + w], valid[:, o:o + w], dim=-1)
    tl = torch.einsum('nd,nud->nu', z[:, :128], emb.float())
    out['target'] = masked_log_softmax(tl, valid[:, 21:21 + U], dim=-1)
    return out, valid


def _run_sample(C, z, emb, handles, seed=7, ctr=0):
    N, U = handles.shape
    dev = z.device
    c = torch.tensor([ctr], dtype=torch.long, device=dev)
    idx = torch.empty(N, 4, dtype=torch.int32, device=dev)
    act = torch.empty(N, 21 + U, dtype=torch.uint8, device=dev)
    msk = torch.empty_like(act)
    logp = torch.empty(N, device=dev)
    val = torch.empty(N, device=dev)
    C.sample_actions(z, emb, handles, seed, c, idx, act, msk, logp, val)
    return idx.long(), act, msk, logp, val


def test_sample_actions_consistency(gpu_ops):
    torch.manual_seed(0)
    N, U = 3000, 40
    z = torch.randn(N, 160, device='cuda') * 2
    emb = (torch.randn(N, U, 128, device='cuda') * 0.2).to(torch.bfloat16)
    handles = torch.where(torch.rand(N, U, device='cuda') < 0.3, torch.randint(1, 999, (N, U), device='cuda'),
                          torch.full((N, U), -1, device='cuda'))
    handles[:200] = -1                              # rows with nothing attackable
    idx, act, msk, logp, val = _run_sample(gpu_ops, z, emb, handles)
    lps, valid = _torch_logps(z, emb, handles)
    r = torch.arange(N, device='cuda')
    enum, x, y, t = idx.unbind(1)
    assert int(enum.max()) <= 2 and int(x.max()) <= 8 and int(y.max()) <= 8 and int(t.max()) < U
    assert not bool((enum[:200] == 2).any()), 'ATTACK sampled with no valid target'
    att = enum == 2
    mv = enum == 1
    assert bool(valid[r[att], 21 + t[att]].all()), 'sampled an invalid target'
    ref_lp = lps['enum'][r, enum] + mv * (lps['x'][r, x] + lps['y'][r, y]) + torch.where(att, lps['target'][r, t], 0.)
    torch.testing.assert_close(logp, ref_lp, atol=2e-3, rtol=1e-3)
    torch.testing.assert_close(val, z[:, 149])
    # experience record: one-hot of the sampled heads; masks = selected heads ∧ valid
    A = 21 + U
    ra = torch.zeros(N, A, dtype=torch.uint8, device='cuda')
    ra[r, enum] = 1
    ra[r[mv], 3 + x[mv]] = 1
    ra[r[mv], 12 + y[mv]] = 1
    ra[r[att], 21 + t[att]] = 1
    head = torch.zeros(N, A, dtype=torch.bool, device='cuda')
    head[:, :3] = True
    head[:, 3:21] = mv[:, None]
    head[:, 21:] = att[:, None]
    assert torch.equal(act, ra)
    assert torch.equal(msk, (head & valid).to(torch.uint8))


def test_sample_actions_distribution(gpu_ops):
    """Gumbel-max draws follow the masked softmax (many rows sharing one set of logits)."""
    torch.manual_seed(1)
    N, U = 40000, 40
    z1 = torch.randn(1, 160, device='cuda')
    e1 = (torch.randn(1, U, 128, device='cuda') * 0.3).to(torch.bfloat16)
    h1 = torch.full((1, U), -1, device='cuda', dtype=torch.long)
    h1[0, 1:6] = torch.arange(10, 15, device='cuda')
    z, emb, handles = z1.expand(N, -1).contiguous(), e1.expand(N, -1, -1).contiguous(), h1.expand(N, -1).contiguous()
    idx, *_ = _run_sample(gpu_ops, z, emb, handles, seed=11, ctr=3)
    lps, valid = _torch_logps(z1, e1, h1)
    for col, k, o, w in ((0, 'enum', 0, 3), (1, 'x', 3, 9), (3, 'target', 21, U)):
        freq = torch.bincount(idx[:, col], minlength=w).float() / N
        p = lps[k][0].exp() * valid[0, o:o + w]
        assert (freq - p).abs().max() < 0.015, (k, freq, p)
    # a different counter gives different draws; the same counter reproduces them
    idx2, *_ = _run_sample(gpu_ops, z, emb, handles, seed=11, ctr=4)
    idx3, *_ = _run_sample(gpu_ops, z, emb, handles, seed=11, ctr=3)
    assert not torch.equal(idx, idx2) and torch.equal(idx, idx3)


def test_lstm_cell_kernel(gpu_ops):
    torch.manual_seed(2)
    N, H = 300, 512
    g = torch.randn(N, 4 * H, device='cuda') * 3
    h = torch.randn(N, H, device='cuda')
    c = torch.randn(N, H, device='cuda')
    i, f, gg, o = g.chunk(4, 1)
    cr = torch.sigmoid(f) * c + torch.sigmoid(i) * torch.tanh(gg)
    hr = torch.sigmoid(o) * torch.tanh(cr)
    h16 = torch.empty(N, H, dtype=torch.bfloat16, device='cuda')
    gpu_ops.lstm_cell(g, h, c, h16)
    torch.testing.assert_close(c, cr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(h, hr, atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(h16.float(), hr, atol=1e-2, rtol=1e-2)


# bf16 operands: loose bounds; IEEE fp32 (the reference actor's precision): log-probs within 1e-5 of torch fp32
TOL = {'bf16': dict(logp=5e-2, value=2e-2, h=2e-2), 'fp32': dict(logp=1e-5, value=1e-5, h=1e-5)}


@pytest.mark.parametrize('preset,precision', [('lstm512', 'bf16'), ('lstm128', 'bf16'), ('compat', 'bf16'),
                                              ('5v5', 'bf16'), ('lstm512', 'fp32'), ('lstm128', 'fp32'),
                                              ('compat', 'fp32'), ('5v5', 'fp32')])
@pytest.mark.parametrize('graph', [True, False])
def test_gpu_actor_matches_policy(gpu_ops, preset, precision, graph):
    """Graph-captured batched actor (hand-written kernels only: encoder → [attention block] → actor_core →
    sampler): values and log-probs of the sampled actions match the torch fp32 policy, with the recurrent state
    carried across steps and reset per slot. fp32: every product an fp32 FMA, log-probs within 1e-5 of torch."""
    from dotaclient_amd.actor.batched import F32ActorPolicy, GpuActorPolicy, _synthetic_states
    from dotaclient_amd.features.featurizer import featurize
    from dotaclient_amd.protos import pb
    torch.manual_seed(3)
    cfg = get_config(preset)
    pol = Policy(cfg).cuda().eval()
    n = 64
    cls = F32ActorPolicy if precision == 'fp32' else GpuActorPolicy
    gp = cls(pol, n, device='cuda', seed=5, use_graph=graph)
    tol = TOL[precision]
    worst = [0.0, 0.0, 0.0]
    states = _synthetic_states(2 * n + 8)
    lay = cfg.layout
    hidden = pol.initial_hidden(n, device='cuda') if cfg.rnn == 'lstm' else None
    for step in range(4):
        feats = []
        for i in range(n):
            j = (i + step * n) % len(states)     # even entries are Radiant's view, odd ones Dire's
            ws = pb.CMsgBotWorldState.FromString(states[j])
            team = 2 if j % 2 == 0 else 3
            feats.append(featurize(ws, 0 if team == 2 else 5, team, lay))
        env = np.stack([f.env for f in feats]).astype(np.float32)
        units = np.stack([f.units for f in feats]).astype(np.float32)
        handles = np.stack([f.handles for f in feats]).astype(np.int64)
        reset = np.zeros(n, bool)
        if step == 2:
            reset[::3] = True
            if hidden is not None:
                keep = torch.as_tensor(~reset, device='cuda', dtype=torch.float32)[None, :, None]
                hidden = (hidden[0] * keep, hidden[1] * keep)
        out = gp.step(env, units, handles, reset=reset)
        with torch.no_grad():
            e = torch.as_tensor(env, device='cuda')[:, None]
            u = torch.as_tensor(units, device='cuda')[:, None]
            logits, value, hidden = pol.forward_packed(e, u, hidden)
            th = torch.as_tensor(handles, device='cuda')
            valid = batched_action_masks(th)
            lps = {k: masked_log_softmax(logits[k][:, 0].reshape(n, -1).float(), valid[:, o:o + w], dim=-1)
                   for k, o, w in (('enum', 0, 3), ('x', 3, 9), ('y', 12, 9), ('target_unit', 21, lay.max_units))}
        idx = torch.as_tensor(out['idx'], device='cuda').long()
        r = torch.arange(n, device='cuda')
        enum, x, y, t = idx.unbind(1)
        mv, att = enum == 1, enum == 2
        ref = lps['enum'][r, enum] + mv * (lps['x'][r, x] + lps['y'][r, y]) + torch.where(
            att, lps['target_unit'][r, t], 0.)
        got = torch.as_tensor(out['logp'], device='cuda')
        worst[0] = max(worst[0], float((got - ref).abs().max()))
        assert (got - ref).abs().max() < tol['logp'], (step, (got - ref).abs().max())
        v = torch.as_tensor(out['value'], device='cuda')
        vr = value[:, 0, 0].float()
        worst[1] = max(worst[1], float((v - vr).abs().max()))
        assert (v - vr).abs().max() < tol['value'] + tol['value'] * vr.abs().max(), (step, v[:4], vr[:4])
        if hidden is not None:
            hg, _ = gp.hidden()
            rel = float((hg - hidden[0][0]).norm() / hidden[0][0].norm())
            worst[2] = max(worst[2], rel)
            assert rel < tol['h'], (step, rel)
    print(f'[actor {preset} {precision} graph={graph}] max |dlogp| {worst[0]:.3e}  max |dvalue| {worst[1]:.3e}  '
          f'h rel {worst[2]:.3e}')

