"""Device return / GAE scan (ops/csrc/scan.hip) and the device ingest path of the learner.

* CPU: the torch reference of ``compute_returns`` equals the host numpy path (``discount`` / ``gae`` /
  ``RunningMeanStd``, themselves pinned to scipy.lfilter and the reference formula in test_runtime.py), and the
  learner's device-ingest batch equals the host ``experiences_from_rollout`` + ``_to_device`` batch.
* GPU: the HIP kernel equals the fp64 torch reference over ragged segments, both modes, incl. long rollouts.
"""
import numpy as np
import pytest
import torch

from dotaclient_amd.learner.returns import RunningMeanStd, discount, gae
from dotaclient_amd.ops.scan import compute_returns
from dotaclient_amd.transport.codec import Rollout


def _segments(rng, lens, S, K=9):
    padded = [-(-T // S) * S for T in lens]
    off = np.concatenate([[0], np.cumsum(padded)]).astype(np.int32)
    L = int(off[-1])
    rew = np.zeros((L, K), np.float32)
    val = np.zeros(L, np.float32)
    for T, a in zip(lens, off[:-1]):
        rew[a:a + T] = rng.randn(T, K) * 0.1
        val[a:a + T] = rng.randn(T)
    return off, rew, val


@pytest.mark.parametrize('mode', ['discount', 'gae'])
def test_reference_matches_host_numpy(mode):
    rng = np.random.RandomState(3)
    S = 64
    lens = [50, 64, 130, 7, 200]
    keys = [0, 1, 0, 0, 1]
    boot = rng.randn(len(lens)).astype(np.float32)
    done = [True, False, False, True, False]
    off, rew, val = _segments(rng, lens, S)
    ema = torch.zeros(4, 3)
    out = compute_returns(torch.from_numpy(rew), torch.from_numpy(val), off, lens, boot, done, keys, ema, mode)
    rms = RunningMeanStd(0.99)
    for i, (T, a, b) in enumerate(zip(lens, off[:-1], off[1:])):
        summed = rew[a:b].astype(np.float64).sum(1)
        if mode == 'gae':
            adv, ret = gae(summed[:T], val[a:a + T], boot[i], 0.98, 0.95, done=done[i])
            np.testing.assert_allclose(out['adv'][a:a + T].numpy(), adv, rtol=1e-5, atol=1e-5)
            np.testing.assert_allclose(out['ret'][a:a + T].numpy(), ret, rtol=1e-5, atol=1e-5)
            assert (out['ret'][a + T:b] == 0).all() and (out['adv'][a + T:b] == 0).all()
            rms.update(ret, keys[i])
        else:
            ret = discount(summed, 0.98)
            np.testing.assert_allclose(out['ret'][a:b].numpy(), ret, rtol=1e-5, atol=1e-5)
            rms.update(ret, keys[i])
            np.testing.assert_allclose(out['norm'][a:b].numpy(), rms.normalize(ret, keys[i]), rtol=1e-4, atol=1e-4)
    for k in (0, 1):
        assert float(ema[k, 0]) == pytest.approx(rms.mean[k], rel=1e-5, abs=1e-6)
        assert float(ema[k, 1]) == pytest.approx(rms.std[k], rel=1e-5, abs=1e-6)
        assert float(ema[k, 2]) == 1.0
    assert float(ema[2, 2]) == 0.0


def _rollouts(n, U=40, H=16, seed=0):
    rng = np.random.RandomState(seed)
    out = []
    for i in range(n):
        T = int(rng.randint(20, 150))
        out.append(Rollout(game_id=f'g{i}', team_id=2 + i % 2, player_id=0, env=rng.randn(T, 3).astype(np.float32),
                           units=rng.randn(T, U, 10).astype(np.float32),
                           actions=(rng.rand(T, 21 + U) > 0.9).astype(np.uint8),
                           masks=(rng.rand(T, 21 + U) > 0.5).astype(np.uint8), rewards=rng.randn(T, 9) * 0.1,
                           weight_version=1, logp=rng.randn(T).astype(np.float32),
                           values=rng.randn(T).astype(np.float32), hiddens=rng.randn(8, 2, H).astype(np.float32),
                           hidden_stride=32, bootstrap_value=float(rng.randn()), done=bool(i % 3 == 0)))
    return out


@pytest.mark.parametrize('algo', ['ppo', 'vpg'])
def test_device_ingest_equals_host_ingest(tmp_path, algo):
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.broker import InProcBroker

    def make(ingest, sub):
        cfg = OptimizerConfig(log_dir=str(tmp_path / sub), batch_size=2, seq_len=32, seq_per_epoch=8, epochs=1,
                              algo=algo, model='lstm128', device='cpu', backend='torch', ingest=ingest,
                              advantages='gae')     # (the host ingest: GAE from the actor's values)
        return DotaOptimizer(cfg, InProcBroker())
    host, dev = make('host', 'h'), make('device', 'd')
    for it in range(2):                                  # two rounds: the EMA state carries over
        rs = _rollouts(5, H=host.policy_cfg.hidden, seed=it)
        seqs = []
        for r in rs:
            seqs.extend(host.experiences_from_rollout(r))
        n = len(seqs) - len(seqs) % 2
        a = host._to_device(seqs[:n])
        b = dev._ingest_device(rs, n)
        assert set(a) == set(b)
        for k in a:
            assert a[k].shape == b[k].shape, k
            torch.testing.assert_close(b[k].float(), a[k].float(), rtol=1e-4, atol=1e-4, msg=k)
        dev._sync_running()
        for team in (2, 3):
            assert dev.running.mean[team] == pytest.approx(host.running.mean[team], rel=1e-5, abs=1e-6)
            assert dev.running.std[team] == pytest.approx(host.running.std[team], rel=1e-5, abs=1e-6)


def _vtrace_np(r, v, lr, boot, gamma, lam, rho_bar=1.0, c_bar=1.0):
    """V-trace (Espeholt et al. 2018, eq. 1) written out as the explicit sum, independently of the recursion:
    v_s = V_s + Σ_{t≥s} γ^{t−s} (Π_{i=s}^{t−1} c_i) ρ_t δ_t, c_i = λ·min(c̄, w_i), ρ_t = min(ρ̄, w_t); the advantage is
    v_s − V_s."""
    T = len(r)
    w = np.exp(lr)
    vn = np.append(v[1:], boot)
    delta = r + gamma * vn - v
    rho, c = np.minimum(rho_bar, w), lam * np.minimum(c_bar, w)
    vs = np.zeros(T)
    for s_ in range(T):
        acc, prod = 0.0, 1.0
        for t in range(s_, T):
            acc += gamma ** (t - s_) * prod * rho[t] * delta[t]
            prod *= c[t]
        vs[s_] = v[s_] + acc
    return vs, vs - v


def test_vtrace_reference_matches_explicit_sum_and_equals_gae_on_policy():
    rng = np.random.RandomState(5)
    S = 32
    lens = [30, 32, 70, 5]
    keys = [0, 1, 0, 1]
    boot = rng.randn(len(lens)).astype(np.float32)
    done = [False, True, False, False]
    off, rew, val = _segments(rng, lens, S)
    lr = (rng.randn(int(off[-1])) * 0.7).astype(np.float32)
    out = compute_returns(torch.from_numpy(rew), torch.from_numpy(val), off, lens, boot, done, keys, torch.zeros(2, 3),
                          'vtrace', lr=torch.from_numpy(lr))
    for i, (T, a, b) in enumerate(zip(lens, off[:-1], off[1:])):
        r = rew[a:a + T].astype(np.float64).sum(1)
        vs, pg = _vtrace_np(r, val[a:a + T].astype(np.float64), lr[a:a + T].astype(np.float64),
                            0.0 if done[i] else float(boot[i]), 0.98, 0.95)
        np.testing.assert_allclose(out['ret'][a:a + T].numpy(), vs, rtol=1e-5, atol=1e-5)
        np.testing.assert_allclose(out['adv'][a:a + T].numpy(), pg, rtol=1e-5, atol=1e-5)
        assert (out['ret'][a + T:b] == 0).all() and (out['adv'][a + T:b] == 0).all()
    # on-policy (π = μ): V-trace's value target is GAE's return and its advantage GAE's advantage
    gae_out = compute_returns(torch.from_numpy(rew), torch.from_numpy(val), off, lens, boot, done, keys,
                              torch.zeros(2, 3), 'gae')
    on = compute_returns(torch.from_numpy(rew), torch.from_numpy(val), off, lens, boot, done, keys, torch.zeros(2, 3),
                         'vtrace', lr=torch.zeros(int(off[-1])))
    torch.testing.assert_close(on['ret'], gae_out['ret'], rtol=1e-5, atol=1e-5)
    torch.testing.assert_close(on['adv'], gae_out['adv'], rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
@pytest.mark.parametrize('mode', ['discount', 'gae', 'vtrace'])
def test_scan_kernel_matches_reference(gpu_ops, mode):
    rng = np.random.RandomState(11)
    S = 1400
    lens = [1380, 1400, 2900, 1, 700, 9999, 3000, 64]
    keys = [0, 1, 0, 1, 1, 0, 2, 0]
    boot = rng.randn(len(lens)).astype(np.float32)
    done = [True, False, False, True, False, True, False, False]
    off, rew, val = _segments(rng, lens, S)
    ema_c = torch.zeros(3, 3)
    ema_c[1] = torch.tensor([0.3, 1.5, 1.0])            # a resumed team state
    ema_g = ema_c.clone().cuda()
    lr = torch.from_numpy((rng.randn(int(off[-1])) * 0.5).astype(np.float32))
    ref = compute_returns(torch.from_numpy(rew), torch.from_numpy(val), off, lens, boot, done, keys, ema_c, mode, lr=lr)
    got = compute_returns(torch.from_numpy(rew).cuda(), torch.from_numpy(val).cuda(), off, lens, boot, done, keys,
                          ema_g, mode, lr=lr.cuda())
    torch.cuda.synchronize()
    for k in ('ret', 'adv', 'norm', 'stats'):
        torch.testing.assert_close(got[k].cpu(), ref[k], rtol=2e-4, atol=2e-4, msg=k)
    torch.testing.assert_close(ema_g.cpu(), ema_c, rtol=1e-5, atol=1e-5)


@pytest.mark.gpu
def test_multi_copy_matches_per_tensor_copies(gpu_ops):
    """ops multi_copy (the learner's one-launch pool fill): every segment byte-exact, including byte tails of
    uint8 fields whose sizes are not multiples of 16."""
    g = torch.Generator(device='cuda').manual_seed(0)
    srcs = [torch.randn(1000, 7, device='cuda', generator=g), torch.randint(0, 255, (333, 61), device='cuda',
                                                                             dtype=torch.uint8, generator=g),
            torch.randn(5, device='cuda', generator=g), torch.randint(0, 2, (1401,), device='cuda', dtype=torch.uint8,
                                                                      generator=g)]
    dsts = [torch.full_like(t, 7) for t in srcs]
    gpu_ops.multi_copy(dsts, srcs)
    torch.cuda.synchronize()
    for d, s in zip(dsts, srcs):
        assert torch.equal(d, s)


@pytest.mark.gpu
def test_ingest_scatter_and_adv_normalize_match_torch(gpu_ops):
    """ops ingest_scatter (the look-ahead expand's one launch) against zero_() + index_copy_() per field, incl. byte
    rows (uint8, 61 B) and out-of-range inv entries (zeros, never read); adv_normalize against the torch expression."""
    g = torch.Generator(device='cuda').manual_seed(1)
    L, Lv = 500, 321
    rows = torch.randperm(L, device='cuda', generator=g)[:Lv].sort().values
    inv = torch.full((L,), -1, dtype=torch.int32, device='cuda')
    inv[rows] = torch.arange(Lv, dtype=torch.int32, device='cuda')
    inv[rows[-1]] = Lv + 5                                   # out of range: must come out as a padding row
    srcs = [torch.randn(Lv, 40, 10, device='cuda', generator=g),
            torch.randint(0, 255, (Lv, 61), dtype=torch.uint8, device='cuda', generator=g),
            torch.randn(Lv, device='cuda', generator=g), torch.randn(Lv, 9, device='cuda', generator=g)]
    dsts = [torch.full((L,) + tuple(t.shape[1:]), 7, dtype=t.dtype, device='cuda') for t in srcs]
    valid = torch.full((L,), 7.0, device='cuda')
    gpu_ops.ingest_scatter(dsts, srcs, inv, valid)
    keep = rows[:-1]
    for d, s in zip(dsts, srcs):
        ref = torch.zeros_like(d)
        ref.index_copy_(0, keep, s[:Lv - 1])
        assert torch.equal(d, ref)
    vref = torch.zeros(L, device='cuda')
    vref[keep] = 1.0
    assert torch.equal(valid, vref)
    adv = torch.randn(8, 64, device='cuda', generator=g) * 3 + 1
    v = (torch.rand(8, 64, device='cuda', generator=g) > 0.3).float()
    out = torch.empty_like(adv)
    gpu_ops.adv_normalize(adv, v, out, 1e-8)
    n = v.sum().clamp_min(1.0)
    mu = (adv * v).sum() / n
    sd = (((adv - mu) ** 2 * v).sum() / n).sqrt()
    torch.testing.assert_close(out, ((adv - mu) / (sd + 1e-8)) * v, rtol=1e-5, atol=1e-6)
