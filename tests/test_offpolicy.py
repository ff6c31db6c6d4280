"""Learner-side old log-probs / values (the reference's ``policy_old``, optimizer.py:279, 474) and the off-policy
corrections of stale and replayed experience:

* ``old_logp='learner'``: once per iteration the learner evaluates the iteration's experience at its starting weights
  (``Learner.evaluate_sequences``) — at weight age 0 that IS the actor's log-prob (the actor ran the same fp32 policy);
* V-trace GAE (ops/scan.py ``'vtrace'``) from the learner's values with truncated importance weights against the
  actor's behaviour log-probs;
* ``LossConfig.offpolicy='tis'`` (replayed experience): the truncated-importance-weight policy gradient, torch oracle
  vs the fused heads kernel (algo 2).
"""
import copy

import numpy as np
import pytest
import torch

from dotaclient_amd import native
from dotaclient_amd.learner.engine import Learner, LossConfig
from dotaclient_amd.learner.synthetic import make_batch
from dotaclient_amd.models.policy import Policy, get_config
from dotaclient_amd.transport.codec import decode


def _actor_rollouts(cfg, n_games=3, finished=3, seed=5):
    from dotaclient_amd.actor.vec import VecActor
    from dotaclient_amd.actor.weights import WeightStore
    ws = WeightStore(cfg, device='cpu')
    torch.manual_seed(seed)
    ws.add(0, {k: t.detach().clone() for k, t in Policy(cfg).state_dict().items()})
    sent = []
    va = VecActor(ws, n_games, sent.append, device='cpu', seed=seed, rollout_size=40, max_dota_time=20.0,
                  hidden_stride=8, threads=2, groups=1)
    while va.games_finished < finished:
        va.step()
    return ws, [decode(b) for b in sent]


@pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
def test_learner_old_logp_equals_the_actors_at_weight_age_zero(tmp_path):
    """At weight age 0 the learner's policy_old evaluation reproduces the fp32 actor's log-probs of its own sampled
    actions (and its values) within 1e-5 on every valid row — the learner and the actor run the same fp32 policy, the
    actor step by step with its LSTM state carried across rollout chunks (stored hidden states), the learner over
    whole sequences. The V-trace GAE then equals the actor-side GAE (ρ = 1 up to rounding)."""
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.broker import InProcBroker
    cfg = get_config('lstm128')
    ws, rs = _actor_rollouts(cfg)
    assert len(rs) >= 4
    out = {}
    for mode in ('learner', 'actor'):
        oc = OptimizerConfig(log_dir=str(tmp_path / mode), batch_size=2, seq_len=32, seq_per_epoch=4, epochs=1,
                             model='lstm128', device='cpu', backend='torch', ingest='device', old_logp=mode,
                             advantages='vtrace-iteration' if mode == 'learner' else 'gae')
        opt = DotaOptimizer(oc, InProcBroker())
        opt.policy.load_state_dict(ws.latest_weights()[1])
        opt.learner.after_load_weights()
        n_seq = sum(-(-r.length // 32) for r in rs)
        d = opt._ingest_device(rs, n_seq - n_seq % 2)
        out[mode] = (d, d.pop('_prox', None))
    (dl, prox), (da, _) = out['learner'], out['actor']
    v = dl['valid'] > 0
    assert int(v.sum()) > 100
    err = (dl['logp_old'] - da['logp_old'])[v].abs().max().item()
    assert err < 1e-5, err
    assert float(prox['offpolicy/max_abs_logratio']) < 1e-5
    assert abs(float(prox['offpolicy/rho_mean']) - 1.0) < 1e-5
    torch.testing.assert_close(dl['ret'][v], da['ret'][v], rtol=1e-4, atol=1e-4)


def test_truncated_is_policy_term_gradient():
    """ppo_loss(offpolicy='tis'): value −mean(w·A) and gradient −mean(w·A·∇logπ) with w = min(1, π/π_old) held
    constant; clipfrac counts the truncated rows."""
    from dotaclient_amd.learner.losses import ppo_loss, sampled_logp, split_heads
    torch.manual_seed(0)
    cfg = get_config('lstm128')
    pol = Policy(cfg)
    b = make_batch(2, 12, cfg.layout, cfg.hidden, device='cpu', seed=3)
    counts = pol.layout.action_counts()
    acts, msks = split_heads(b['actions'], counts), split_heads(b['masks'], counts)
    logits, values, _ = pol.forward_packed(b['env'], b['units'], (b['h0'][None], b['c0'][None]))
    logp_old = b['logp_old']
    loss, m = ppo_loss(logits, values, acts, msks, b['adv'], b['ret'], logp_old, 0.1, 0.0, 0.0, offpolicy='tis')
    g = torch.autograd.grad(loss, [pol.affine_head_enum.weight])[0]
    logits2, _, _ = pol.forward_packed(b['env'], b['units'], (b['h0'][None], b['c0'][None]))
    lp = sampled_logp(logits2, acts, msks)
    valid = sum(acts[k].sum(-1) for k in acts).gt(0).float()
    w = torch.exp(lp - logp_old).detach().clamp(max=1.0)
    ref = -(w * b['adv'] * lp * valid).sum() / valid.sum()
    g_ref = torch.autograd.grad(ref, [pol.affine_head_enum.weight])[0]
    torch.testing.assert_close(g, g_ref, rtol=1e-5, atol=1e-7)
    torch.testing.assert_close(m['policy_loss'], -(w * b['adv'] * valid).sum() / valid.sum(), rtol=1e-5, atol=1e-7)
    frac = ((torch.exp(lp - logp_old) > 1).float() * valid).sum() / valid.sum()
    torch.testing.assert_close(m['clipfrac'], frac.detach())


@pytest.mark.gpu
@pytest.mark.parametrize('preset,precision', [('lstm512', 'fp32-exact'), ('lstm128', 'fp32'), ('5v5', 'fp32-exact')])
def test_fused_evaluate_sequences_matches_torch_fp32(gpu_ops, preset, precision):
    """Learner.evaluate_sequences on the fused forward kernels (the policy_old pass) vs the torch fp32 module: the
    sampled-action log-prob and the value of every step, fp32-exact within 1e-5 (bf16x3: 1e-3)."""
    torch.manual_seed(0)
    cfg = get_config(preset)
    pol = Policy(cfg)
    ref = copy.deepcopy(pol)
    fused = Learner(pol, LossConfig(), device='cuda', backend='fused', dp=False, precision=precision)
    oracle = Learner(ref, LossConfig(), device='cuda', backend='torch', dp=False, precision='fp32')
    n, S = 5, 70
    data = make_batch(n, S, cfg.layout, cfg.hidden, device='cuda', seed=7)
    data['reset'] = (torch.rand(n, S, device='cuda') < 0.02).to(torch.uint8)
    lp_f, v_f = fused.evaluate_sequences(data, n, chunk=3)
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        lp_t, v_t = oracle.evaluate_sequences(data, n)
    torch.cuda.synchronize()
    fused.model.check_error()
    tol = 1e-5 if precision == 'fp32-exact' else 1e-3
    valid = data['actions'].sum(-1) > 0
    assert (lp_f - lp_t)[valid].abs().max().item() < tol * max(1.0, lp_t.abs().max().item())
    assert (v_f - v_t).abs().max().item() < tol * max(1.0, v_t.abs().max().item())


@pytest.mark.gpu
def test_fused_truncated_is_step_matches_torch(gpu_ops):
    """The fused step with LossConfig(offpolicy='tis') (heads_loss algo 2) vs the torch oracle: loss, metrics and
    the whole gradient."""
    torch.manual_seed(0)
    cfg = get_config('lstm512')
    pol = Policy(cfg)
    ref = copy.deepcopy(pol)
    lc = LossConfig(algo='ppo', offpolicy='tis')
    fused = Learner(pol, lc, device='cuda', backend='fused', dp=False, precision='fp32-exact')
    oracle = Learner(ref, lc, device='cuda', backend='torch', dp=False, precision='fp32')
    batch = make_batch(4, 40, cfg.layout, cfg.hidden, device='cuda', seed=3)
    batch['logp_old'] = batch['logp_old'] + 0.3 * torch.randn_like(batch['logp_old'])
    for L in (fused, oracle):
        L.dp.zero_grad()
    lf, mf = fused.loss(batch)
    lf.backward()
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        lr_, mr = oracle.loss(batch)
        lr_.backward()
    torch.cuda.synchronize()
    for k in ('loss', 'policy_loss', 'approx_kl', 'clipfrac'):
        assert abs(float(mf[k]) - float(mr[k])) <= 1e-4 * max(1.0, abs(float(mr[k]))), (k, float(mf[k]), float(mr[k]))
    rel = ((fused.flat.grad - oracle.flat.grad).norm() / oracle.flat.grad.norm()).item()
    assert rel < 1e-4, rel


@pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
def test_snapshot_evaluation_and_league_matrix_cpu():
    """Head-to-head evaluation against frozen snapshots (actor/validate.py): every game a league game of the current
    weights against the snapshot; results counted per game; the league matrix is antisymmetric around ½."""
    from dotaclient_amd.actor.validate import evaluate_vs_snapshot, league_matrix
    cfg = get_config('lstm128')
    torch.manual_seed(1)
    a, b = Policy(cfg), Policy(cfg)
    r = evaluate_vs_snapshot(a, b.state_dict(), n_games=6, device='cpu', seed=3, max_dota_time=12.0, threads=2)
    assert r['games'] >= 6 and 0.0 <= r['win_rate'] <= 1.0
    assert r['wins'] + r['losses'] + r['draws'] == r['games']
    m = league_matrix([('v0', a.state_dict()), ('v1', b.state_dict())], cfg, n_games=4, device='cpu',
                      max_dota_time=12.0, threads=2)
    w = m['win_rate']
    assert m['labels'] == ['v0', 'v1'] and w[0][0] == 0.5 and abs(w[0][1] + w[1][0] - 1.0) < 1e-9


@pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
def test_in_step_vtrace_rows_and_weight_age_zero(tmp_path):
    """advantages='vtrace-step': the ingest lays out the per-row {reward, bootstrap, valid, last} field (an episode
    segment ends at its rollout's last row — bootstrap 0 if done, else the actor's bootstrap value — and at every
    sequence boundary it runs past — bootstrap the actor's value of the next row); at weight age 0 the in-step V-trace
    of a minibatch (the step's own values and log-probs, torch oracle) reproduces the ingest's GAE returns, and a
    training step runs and reports the off-policy metrics (ρ = 1, behaviour KL ≈ 0)."""
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.ops.scan import vtrace_step
    from dotaclient_amd.transport.broker import InProcBroker
    cfg = get_config('lstm128')
    ws, rs = _actor_rollouts(cfg)
    S = 32
    oc = OptimizerConfig(log_dir=str(tmp_path), batch_size=2, seq_len=S, seq_per_epoch=4, epochs=1, model='lstm128',
                         device='cpu', backend='torch', ingest='device', advantages='vtrace-step')
    opt = DotaOptimizer(oc, InProcBroker())
    assert opt.vtrace_step and opt.learner.cfg.vtrace
    opt.policy.load_state_dict(ws.latest_weights()[1])
    opt.learner.after_load_weights()
    n_seq = sum(-(-r.length // S) for r in rs)
    n = n_seq - n_seq % 2
    d = opt._ingest_device(rs, n)
    vt = d['vt']
    assert vt.shape == (n, S, 4)
    flat = vt.reshape(-1, 4)
    # (unpacked layout: every rollout padded to a multiple of S) — last rows: rollout ends and inner boundaries
    row = 0
    for r in rs:
        T = r.length
        k = -(-T // S) * S
        if row + k > n * S:
            break
        last = flat[row:row + k, 3]
        want = torch.zeros(k)
        want[T - 1] = 1.0
        for b in range(S - 1, T - 1, S):
            want[b] = 1.0
        assert torch.equal(last, want), r.game_id
        assert float(flat[row + T - 1, 1]) == pytest.approx(0.0 if r.done else float(r.bootstrap_value), abs=1e-6)
        for b in range(S - 1, T - 1, S):
            assert float(flat[row + b, 1]) == pytest.approx(float(r.values[b + 1]), abs=1e-6)
        assert torch.equal(flat[row:row + k, 2], (torch.arange(k) < T).float())
        row += k
    # weight age 0: the in-step V-trace returns of a minibatch equal the ingest's GAE returns (actor values) on every
    # sequence that holds its episodes' ends (a sequence cut inside a rollout bootstraps from the actor's value of the
    # next row — truncated there, like any V-trace unroll — where the ingest scan runs over the whole rollout)
    B = 4
    batch = {k: v[:B] for k, v in d.items() if torch.is_tensor(v)}
    with torch.no_grad():
        hid = (batch['h0'][None], batch['c0'][None])
        logits, values, _ = opt.policy.forward_packed(batch['env'], batch['units'], hid)
        from dotaclient_amd.learner.losses import sampled_logp, split_heads
        counts = opt.policy.layout.action_counts()
        lp = sampled_logp(logits, split_heads(batch['actions'], counts), split_heads(batch['masks'], counts))
    tm = lambda x: x.transpose(0, 1).reshape(B * S, *x.shape[2:])  # noqa: E731
    adv, ret, st = vtrace_step(tm(values.squeeze(-1)), tm(lp), tm(batch['logp_old']), tm(batch['vt']), B, S)
    cut = (batch['vt'][:, S - 1, 2] > 0) & (batch['vt'][:, S - 1, 3] > 0)     # a rollout runs past the sequence end
    whole = (~cut).view(1, B).expand(S, B).reshape(-1)
    v = (tm(batch['vt'])[:, 2] > 0) & whole
    assert int(v.sum()) > 10
    torch.testing.assert_close(ret[v], tm(batch['ret'])[v], rtol=1e-4, atol=1e-4)
    s_ = st.sum(0)
    assert abs(float(s_[0] / s_[3]) - 1.0) < 1e-5 and abs(float(s_[2] / s_[3])) < 1e-5
    m = opt.learner.train_step(batch)
    assert float(m['offpolicy/rho_mean']) == pytest.approx(1.0, abs=1e-5)
    assert abs(float(m['offpolicy/behaviour_kl'])) < 1e-5 and torch.isfinite(m['loss'])


def _vt_batch(cfg, B, S, seed):
    b = make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=seed)
    g = torch.Generator(device='cuda').manual_seed(seed)
    valid = (b['actions'].sum(-1) > 0).float()
    last = (torch.rand(B, S, device='cuda', generator=g) < 0.04).float()
    last[:, -1] = 1.0
    b['vt'] = torch.stack([torch.randn(B, S, device='cuda', generator=g) * 0.3,
                           torch.randn(B, S, device='cuda', generator=g) * last, valid, last], -1).contiguous()
    b['logp_old'] = b['logp_old'] + 0.4 * torch.randn(B, S, device='cuda', generator=g)
    return b


@pytest.mark.gpu
@pytest.mark.parametrize('precision,tol', [('fp32-exact', 2e-5), ('fp32', 2e-3)])
def test_fused_in_step_vtrace_matches_torch(gpu_ops, precision, tol):
    """The fused step with LossConfig(vtrace=True) — a forward-only heads pass for the step's log-probs, the V-trace
    kernel over its own values (ops/csrc/scan.hip vtrace_step_kernel), the advantage normalisation, then the usual
    heads / loss / backward — against the torch oracle (Learner._vtrace_torch + ppo_loss): loss, the off-policy
    metrics and the whole gradient."""
    torch.manual_seed(0)
    cfg = get_config('lstm512')
    pol = Policy(cfg)
    ref = copy.deepcopy(pol)
    lc = LossConfig(algo='ppo', vtrace=True)
    fused = Learner(pol, lc, device='cuda', backend='fused', dp=False, precision=precision)
    oracle = Learner(ref, lc, device='cuda', backend='torch', dp=False, precision='fp32')
    batch = _vt_batch(cfg, 4, 50, 3)
    for L in (fused, oracle):
        L.dp.zero_grad()
    lf, mf = fused.loss(batch)
    lf.backward()
    with torch.backends.cudnn.flags(enabled=False):
        torch.backends.cuda.matmul.allow_tf32 = False
        lr_, mr = oracle.loss(batch)
        lr_.backward()
    torch.cuda.synchronize()
    for k in ('loss', 'policy_loss', 'advantage_loss', 'approx_kl', 'offpolicy/rho_mean', 'offpolicy/rho_truncated',
              'offpolicy/behaviour_kl'):
        assert abs(float(mf[k]) - float(mr[k])) <= 10 * tol * max(1.0, abs(float(mr[k]))), (k, float(mf[k]),
                                                                                         float(mr[k]))
    rel = ((fused.flat.grad - oracle.flat.grad).norm() / oracle.flat.grad.norm()).item()
    assert rel < 10 * tol, rel


@pytest.mark.gpu
def test_in_step_vtrace_direct_graph_step_matches_eager(gpu_ops):
    """The graph-captured direct step (replay gather of the vt field inside the graph) equals the eager step."""
    from dotaclient_amd.learner.replay import HbmReplay
    torch.manual_seed(0)
    cfg = get_config('lstm512')
    pol = Policy(cfg)
    ref = copy.deepcopy(pol)
    lc = LossConfig(algo='ppo', vtrace=True)
    a = Learner(pol, lc, device='cuda', backend='fused', dp=False, precision='fp32-exact')
    b = Learner(ref, lc, device='cuda', backend='fused', dp=False, precision='fp32-exact')
    assert b.enable_graph(warmup=1)
    rep = HbmReplay(6, 40, cfg.layout, cfg.hidden, 'cuda', seed=5, vtrace=True)
    rep.add(_vt_batch(cfg, 6, 40, 9))
    for step in range(3):
        idx = torch.randperm(6, device='cuda')[:4]
        ma = a.train_step_indices(rep, idx)
        mb = b.train_step_indices(rep, idx)
        torch.cuda.synchronize()
        for k in ('loss', 'offpolicy/rho_mean', 'grad_norm'):
            torch.testing.assert_close(mb[k], ma[k], rtol=1e-5, atol=1e-6, msg=f'step {step} {k}')
    torch.testing.assert_close(b.flat.flat, a.flat.flat, rtol=1e-5, atol=1e-6)
