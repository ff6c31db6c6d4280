"""Does the framework learn?

* CPU: the learning-curve loop (learner/curve.py: VecActor self-play → DotaOptimizer → periodic evaluation against
  the scripted default bot, the reference's validation agent /root/reference/agent.py:905-927) runs end to end and
  reports the reference's validation metrics;
* GPU: thirty seconds of training with the fused IEEE-fp32 learner at the reference deploy shape (8 × 1400) raise
  ``game/rewards_sum`` and the win rate against the default bot;
* GPU: the fused fp32-exact optimizer trajectory follows the plain torch-fp32 learner (nn.LSTM autograd + the same
  Adam) step by step on the same batches — losses and the parameter updates, not just one gradient."""
import copy

import pytest
import torch

from dotaclient_amd.learner.curve import run_learning_curve
from dotaclient_amd.learner.engine import Learner, LossConfig
from dotaclient_amd.learner.synthetic import make_batch
from dotaclient_amd.models.policy import Policy, get_config

KEYS = ('game/rewards_sum', 'game/win_rate', 'game/loss_rate', 'game/steps', 'games')


def test_learning_curve_loop_cpu():
    rows = run_learning_curve(budget=3, eval_every=1.5, eval_games=8, model='lstm128', precision='fp32', games=16,
                              threads=2, seq_len=32, batch_size=2, seq_per_epoch=2, max_dota_time=20.0,
                              device='cpu', pack=False)
    assert len(rows) >= 2
    assert rows[0]['iteration'] == 0 and rows[-1]['iteration'] > 0 and rows[-1]['samples'] > 0
    assert rows[-1]['actor_steps'] > 0
    for r in rows:
        assert all(k in r for k in KEYS), sorted(r)
        assert r['games'] == 8.0
        assert 0.0 <= r['game/win_rate'] <= 1.0 and 0.0 <= r['game/loss_rate'] <= 1.0
    assert rows[0]['t_train'] == 0.0 and rows[-1]['t_train'] >= 3


def test_learning_curve_resumes_from_log_dir_cpu(tmp_path):
    """A long curve as several jobs: the second job resumes the checkpointed learner and the curve's counters."""
    kw = dict(eval_every=1.0, eval_games=4, model='lstm128', precision='fp32', games=8, threads=2, seq_len=16,
              batch_size=2, seq_per_epoch=2, max_dota_time=10.0, device='cpu', pack=False, log_dir=str(tmp_path))
    first = run_learning_curve(budget=1.5, **kw)
    second = run_learning_curve(budget=3.0, **kw)
    assert first[0]['t_train'] == 0.0 and second[0].get('resumed')
    assert second[0]['iteration'] > first[-1]['iteration'] and second[0]['t_train'] > first[-1]['t_train']
    assert second[-1]['samples'] > first[-1]['samples'] and second[-1]['t_train'] >= 3.0
    assert second[-1]['actor_steps'] > first[-1]['actor_steps']


@pytest.mark.gpu
def test_short_training_beats_the_untrained_policy_vs_default_bot(gpu_ops):
    """30 s of fused fp32-exact training in the node loop, evaluated with the fp32 actor against the default bot:
    the shaped reward AND the win rate go up (round-4 curve at 30 s: rewards_sum −2.0 → 2.8, win rate 0.02 → 0.20)."""
    rows = run_learning_curve(budget=30, eval_every=30, eval_games=128, games=1024, threads=12)
    first, last = rows[0], rows[-1]
    print('learning: rewards_sum', first['game/rewards_sum'], '->', last['game/rewards_sum'], 'win_rate',
          first['game/win_rate'], '->', last['game/win_rate'], 'iterations', last['iteration'])
    assert last['iteration'] >= 100
    assert last['game/rewards_sum'] >= first['game/rewards_sum'] + 1.5, (first, last)
    assert last['game/win_rate'] >= first['game/win_rate'] + 0.05, (first, last)


def _rel(a, b):
    return float((a - b).norm() / b.norm().clamp_min(1e-30))


@pytest.mark.gpu
def test_exact_fused_trajectory_follows_torch_fp32(gpu_ops):
    """Eight PPO optimizer steps on eight different batches from the same initial weights: the fused fp32-exact
    learner and the torch-fp32 learner (autograd nn.LSTM, same FlatAdam) stay together — per-step loss within 1e-5
    and the accumulated parameter update within 1e-3 of its own size (Adam's m/√v maps the ≈1e-6 gradient round-off
    differences of near-zero-gradient elements to larger relative update differences; a wrong gradient anywhere
    is O(1))."""
    torch.manual_seed(0)
    cfg = get_config('lstm512')
    pol = Policy(cfg)
    lc = LossConfig(algo='ppo', learning_rate=1e-4)
    fused = Learner(copy.deepcopy(pol), lc, device='cuda', backend='fused', dp=False, precision='fp32-exact')
    ref = Learner(copy.deepcopy(pol), lc, device='cuda', backend='torch', dp=False, precision='fp32')
    w0 = {n: p.detach().to('cuda').clone() for n, p in pol.named_parameters()}
    batches = [make_batch(4, 96, cfg.layout, cfg.hidden, device='cuda', seed=100 + s) for s in range(8)]
    lf, lr_ = [], []
    for bt in batches:
        lf.append(float(fused.train_step(bt)['loss']))
        lr_.append(float(ref.train_step(bt)['loss']))
    fused.model.check_error()
    torch.cuda.synchronize()
    print('losses fused', lf, 'torch', lr_)
    for a, b in zip(lf, lr_):
        assert abs(a - b) <= 1e-5 * max(0.1, abs(b)), (lf, lr_)
    pf, pr = dict(fused.policy.named_parameters()), dict(ref.policy.named_parameters())
    upd_f = torch.cat([(pf[n].detach() - w0[n]).reshape(-1) for n in w0])
    upd_r = torch.cat([(pr[n].detach() - w0[n]).reshape(-1) for n in w0])
    assert upd_r.norm() > 0
    assert _rel(upd_f, upd_r) < 1e-3, _rel(upd_f, upd_r)
    # per parameter tensor, looser (small tensors carry few elements)
    for n in w0:
        uf, ur = pf[n].detach() - w0[n], pr[n].detach() - w0[n]
        if ur.norm() > 0:
            assert _rel(uf, ur) < 1e-2, (n, _rel(uf, ur))
