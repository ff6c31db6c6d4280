"""Sequence packing (learner/ingest.py SequencePacker, ``OptimizerConfig.pack_sequences``): several episodes per
``seq_len`` sequence with episode-start reset flags instead of padding every rollout (the reference pads,
/root/reference/optimizer.py:355-378).

* the packer's placement: first fit into free tails, long / stored-state rollouts aligned, reset rows, h0 sources;
* the CPU oracle (torch LSTM with resets, models/policy.py) — a packed sequence [A | B] gives the same PPO loss and
  parameter gradients as the padded sequences [A], [B];
* GPU: the fused learner step with the team recurrence's reset flags (ops/csrc/lstm_team.hip) against the same
  padded evaluation, fp32 (bf16x3) and IEEE fp32."""
import copy

import numpy as np
import pytest
import torch

from dotaclient_amd.learner.engine import Learner, LossConfig
from dotaclient_amd.learner.ingest import IngestPipeline, SequencePacker
from dotaclient_amd.learner.synthetic import make_batch
from dotaclient_amd.models.policy import Policy, get_config
from dotaclient_amd.transport.codec import Rollout


def _rollout(T, seed, hidden=None, stride=0):
    rng = np.random.default_rng(seed)
    U = 40
    A = 21 + U
    act = np.zeros((T, A), np.uint8)
    act[np.arange(T), rng.integers(0, 3, T)] = 1
    return Rollout(game_id=f'g{seed}', team_id=2, player_id=0, env=rng.standard_normal((T, 3)).astype(np.float32),
                   units=rng.standard_normal((T, U, 10)).astype(np.float32), actions=act, masks=act.copy(),
                   rewards=rng.standard_normal((T, 9)), weight_version=0, logp=np.zeros(T, np.float32),
                   values=np.zeros(T, np.float32), hiddens=hidden, hidden_stride=stride)


def test_packer_first_fit_and_resets():
    S = 10
    pk = SequencePacker(S)
    starts = [pk.add(_rollout(T, i)) for i, T in enumerate([4, 3, 12, 2, 9, 5])]
    # 4 → seq 0 [0,4); 3 → seq 0 [4,7) reset; 12 → seqs 1-2 aligned, tail 2 in seq 2; 2 → seq 0 [7,9) reset;
    # 9 → new seq 3; 5 → seq 2 tail [22, 27) reset
    assert starts == [0, 4, 10, 7, 30, 22]
    assert pk.n_seq == 4
    assert sorted(pk.resets) == [4, 7, 22]
    assert pk.seq_src == [(0, 0), (2, 0), (2, 1), (4, 0)]
    # a rollout that starts from a stored non-zero state is never placed mid-sequence
    h = np.ones((1, 2, 8), np.float32)
    r = _rollout(1, 9, hidden=h, stride=S)
    assert not pk.fits(r) and pk.add(r) == 40 and pk.n_seq == 5
    # padding mode: the reference layout (every rollout at a sequence start)
    pp = SequencePacker(S, pack=False)
    assert [pp.add(_rollout(T, i)) for i, T in enumerate([4, 3, 12])] == [0, 10, 20] and pp.resets == []


def test_ingest_stage_packs_rows_in_row_order():
    S = 16
    pl = IngestPipeline(None, S, 2, 'ppo', 8, 'cpu', pack=True)
    rs = [_rollout(5, 1), _rollout(20, 2), _rollout(7, 3)]
    st = pl.stage(rs)
    # 5 → [0,5); 20 → [16,36) (seqs 1-2, tail 4 rows); 7 → seq 0 [5,12) reset
    assert st.n_seq == 3 and st.L == 48 and st.Lv == 32
    assert list(st.off) == [0, 5, 16, 48] and st.lens == [5, 7, 20]
    x = pl.expand(st, {})
    rst = x['reset'].numpy()
    assert rst.sum() == 1 and rst[5] == 1
    v = x['valid'].numpy()
    assert v[:12].all() and not v[12:16].any() and v[16:36].all() and not v[36:].any()
    np.testing.assert_array_equal(x['env'][5:12].numpy(), rs[2].env)


def test_stager_stages_ring_resident_rollouts_and_releases_them():
    """Zero-copy consumption (learner/optimizer.py ``_consume_decode(claim=True)``): the stager thread receives
    rollouts whose arrays view their messages inside the shared-memory ring, copies every field straight into its
    upload slot, and gives the regions back (Rollout.detach_shared) — the staged rows equal the rollouts, the bulk
    arrays are dropped afterwards, the last canvas is kept, and the ring has its space back."""
    import threading
    import uuid
    from dotaclient_amd import native
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.codec import encode
    from dotaclient_amd.transport.shm import ShmBroker
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    S = 16
    b = ShmBroker(f'dca_zc_{uuid.uuid4().hex[:8]}', capacity=1 << 24, create=True)
    try:
        cfg = OptimizerConfig(log_dir='', model='lstm128', seq_len=S, seq_per_epoch=2, batch_size=2,
                              pack_sequences=True, run_local=True)
        opt = DotaOptimizer.__new__(DotaOptimizer)      # only the consumption path: no learner, no GPU
        opt.cfg, opt.broker, opt.corrupt_rollouts = cfg, b, 0
        rs = [_rollout(5, 1), _rollout(20, 2), _rollout(7, 3)]
        for r in rs:
            r.canvas = np.full((4, 4, 3), r.length, np.uint8)
            b.publish_experience(encode(r))
        stop = threading.Event()
        got = [opt._consume_decode(stop, claim=True) for _ in rs]
        assert all(g.release is not None for g in got) and opt._claim_budget.held > 0
        pl = IngestPipeline(None, S, 2, 'ppo', 8, 'cpu', pack=True)
        st = pl.stage(got)
        assert opt._claim_budget.held == 0 and all(g.release is None and g.units is None for g in got)
        assert st.rollouts[-1].canvas is not None and all(g.canvas is None for g in st.rollouts[:-1])
        x = pl.expand(st, {})
        np.testing.assert_array_equal(x['env'][5:12].numpy(), rs[2].env)
        np.testing.assert_array_equal(x['units'][16:36].numpy(), rs[1].units)
        assert [g.length for g in st.rollouts] == [5, 7, 20]
        # the ring is empty and its space reusable: a half-ring message goes through (wherever the cursor stands)
        big = b'x' * ((1 << 23) - 4096)
        b.publish_experience(big, timeout=5.0)
        assert b.consume_experience(1.0) == big
    finally:
        b.close(unlink=True)


def _ppo_grads(pol, batch):
    lrn = Learner(pol, LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01), device='cpu', backend='torch', dp=False)
    pol.zero_grad()
    loss, _ = lrn.loss(batch)
    loss.backward()
    return float(loss.detach()), {n: p.grad.clone() for n, p in pol.named_parameters() if p.grad is not None}


def _packed_and_padded(cfg, S, la, lb, device='cpu', seed=3):
    """Padded: two sequences [A | pad], [B | pad]; packed: one sequence [A | B | pad] with a reset at |A|."""
    src = make_batch(2, S, cfg.layout, cfg.hidden, device='cpu', seed=seed, pad_frac=0.0)
    pad = {k: v.clone() for k, v in src.items()}
    for k, v in pad.items():
        if v.dim() >= 2 and v.shape[1] == S:
            v[0, la:] = 0
            v[1, lb:] = 0
    pad['h0'].zero_()
    pad['c0'].zero_()
    packed = {}
    for k, v in pad.items():
        if v.dim() >= 2 and v.shape[1] == S:
            p = torch.zeros_like(v[:1])
            p[0, :la] = v[0, :la]
            p[0, la:la + lb] = v[1, :lb]
            packed[k] = p
        else:
            packed[k] = v[:1].clone()
    rst = torch.zeros(1, S, dtype=torch.uint8)
    rst[0, la] = 1
    packed['reset'] = rst
    mv = lambda d: {k: v.to(device) for k, v in d.items()}     # noqa: E731
    return mv(pad), mv(packed)


def test_packed_sequence_matches_padded_sequences_cpu():
    torch.manual_seed(0)
    cfg = get_config('lstm128')
    pol = Policy(cfg)
    pad, packed = _packed_and_padded(cfg, 24, 9, 11)
    l_pad, g_pad = _ppo_grads(copy.deepcopy(pol), pad)
    l_pack, g_pack = _ppo_grads(copy.deepcopy(pol), packed)
    assert abs(l_pad - l_pack) < 1e-5, (l_pad, l_pack)
    assert set(g_pad) == set(g_pack)
    for n in g_pad:
        torch.testing.assert_close(g_pack[n], g_pad[n], rtol=1e-4, atol=1e-6, msg=n)
    # without the reset the packed sequence would carry A's state into B: the loss differs
    no_reset = dict(packed, reset=torch.zeros_like(packed['reset']))
    assert abs(_ppo_grads(copy.deepcopy(pol), no_reset)[0] - l_pack) > 1e-7


@pytest.mark.gpu
@pytest.mark.parametrize('precision', ['fp32', 'fp32-exact'])
def test_fused_packed_sequence_matches_padded_on_gpu(gpu_ops, precision):
    """The fused step (team recurrence with reset flags, masked h_{t-1} operand of ∂W_hh) on [A | B] against the
    padded [A], [B] — loss and every parameter gradient."""
    torch.manual_seed(0)
    cfg = get_config('lstm512')
    pol = Policy(cfg)
    S = 64
    pad, packed = _packed_and_padded(cfg, S, 23, 37, device='cuda')

    def run(batch):
        p = copy.deepcopy(pol)
        lrn = Learner(p, LossConfig(algo='ppo', vf_coef=0.5, entropy_coef=0.01), device='cuda', backend='fused',
                      dp=False, precision=precision)
        lrn.dp.zero_grad()
        loss, _ = lrn.loss(batch)
        loss.backward()
        torch.cuda.synchronize()
        return float(loss), {n: q.grad.detach().clone() for n, q in p.named_parameters() if q.grad is not None}
    l_pad, g_pad = run(pad)
    l_pack, g_pack = run(packed)
    assert abs(l_pad - l_pack) <= 1e-5 * max(1.0, abs(l_pad)), (l_pad, l_pack)
    for n, g in g_pad.items():
        rel = ((g_pack[n] - g).norm() / g.norm().clamp_min(1e-12)).item()
        assert rel < (1e-5 if precision == 'fp32-exact' else 1e-3), (n, rel)


def test_zero_copy_stager_keeps_up_with_a_faster_drop_oldest_producer():
    """The node loop's consumption under overload: a producer publishing into the drop_oldest ring faster than the
    stager takes rollouts, three claiming decode threads, packed staging. A consumer that holds claimed regions for a
    whole gather pins the ring's reclaim point; the ring used to keep dropping every new message behind it (space it
    could never reclaim) until the stager, one rollout short of its batch, waited forever (native/core.h
    drop_head_locked now drops only what it can reclaim and otherwise lets the producer wait)."""
    import threading
    import time
    import uuid
    from dotaclient_amd import native
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig, _RolloutPrefetcher
    from dotaclient_amd.transport.codec import encode
    from dotaclient_amd.transport.shm import ShmBroker
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    S = 256
    rng = np.random.default_rng(0)
    msgs = [encode(_rollout(int(T), i)) for i, T in enumerate(rng.integers(50, 400, 32))]
    b = ShmBroker(f'dca_zf_{uuid.uuid4().hex[:8]}', capacity=1 << 26, create=True, drop_oldest=True)
    stop = threading.Event()
    err = []

    def produce():
        i = 0
        try:
            while not stop.is_set():
                b.publish_experience(msgs[i % len(msgs)], timeout=5.0)
                i += 1
        except BaseException as e:
            if not stop.is_set():       # (at the end: the closed consumer no longer releases space)
                err.append(e)
    th = threading.Thread(target=produce, daemon=True)
    th.start()
    cfg = OptimizerConfig(log_dir='', model='lstm128', seq_len=S, seq_per_epoch=8, batch_size=8,
                          pack_sequences=True, run_local=True)
    opt = DotaOptimizer.__new__(DotaOptimizer)
    opt.cfg, opt.broker, opt.corrupt_rollouts, opt._xp_broker = cfg, b, 0, b
    pf = _RolloutPrefetcher(lambda s: opt._consume_decode(s, claim=True), 32, threads=3)
    pl = IngestPipeline(pf.get_until, S, 8, 'ppo', 128, 'cpu', pack=True)
    n, t0 = 0, time.monotonic()
    try:
        # (before the ring fix the stager starved for good within ≈10 iterations; 60 pass in seconds on an idle host
        # and well within the limit on a loaded one)
        while n < 60 and time.monotonic() - t0 < 90.0:
            st = pl.get()
            pl.expand(st, {})
            n += 1
    finally:
        stop.set()
        pl.close()
        pf.close()
        th.join(10.0)
    try:
        assert not err, err
        assert n == 60
        assert opt._claim_budget.held == 0 and opt.ingest_stats()['claimed'] > 0
    finally:
        b.close(unlink=True)


def test_stager_rejects_an_iteration_whose_claim_was_abandoned():
    """Zero-copy staging vs the ring's claim abandonment (native/core.h claim_abandon_s_): a learner that holds claimed
    rollouts past the deadline while producers need the space loses them to the producers — the ring reclaims the
    regions and new messages overwrite the bytes. The stager checks every claim after copying and drops the iteration
    instead of training on the overwritten rows; releases of the abandoned tokens are ignored; the next iteration is
    staged normally."""
    import threading
    import time
    import uuid
    from dotaclient_amd import native
    from dotaclient_amd.learner.ingest import _ClaimsAbandoned
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.codec import encode
    from dotaclient_amd.transport.shm import ShmBroker
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    S = 64
    msgs = [encode(_rollout(60, i)) for i in range(3)]
    b = ShmBroker(f'dca_ca_{uuid.uuid4().hex[:8]}', capacity=4 * len(msgs[0]) + 4096, create=True, drop_oldest=True)
    try:
        cfg = OptimizerConfig(log_dir='', model='lstm128', seq_len=S, seq_per_epoch=2, batch_size=2, run_local=True)
        opt = DotaOptimizer.__new__(DotaOptimizer)
        opt.cfg, opt.broker, opt.corrupt_rollouts, opt._xp_broker = cfg, b, 0, b
        stop = threading.Event()
        pl = IngestPipeline(None, S, 2, 'ppo', 128, 'cpu')
        # control: claimed, staged, released — accepted
        for m in msgs[:2]:
            b.publish_experience(m, timeout=1.0)
        rs = [opt._consume_decode(stop, claim=True) for _ in range(2)]
        assert all(getattr(r, 'release', None) is not None for r in rs)
        st = pl.stage(rs)
        assert st.n_seq == 2
        pl.expand(st, {})
        assert opt._claim_budget.held == 0
        # now hold two claims while a producer fills the ring and waits for space: after 0.3 s the claim at the
        # reclaim point is abandoned and overwritten
        b.ring.set_claim_abandon(0.3)
        for m in msgs[:2]:
            b.publish_experience(m, timeout=1.0)
        rs = [opt._consume_decode(stop, claim=True) for _ in range(2)]
        d0 = b.ring.dropped()
        t0 = time.monotonic()
        for i in range(6):                  # more than fits behind the held claims: the last ones wait for abandonment
            b.publish_experience(msgs[2], timeout=5.0)
        assert time.monotonic() - t0 > 0.2 and b.ring.dropped() > d0
        assert not all(r.release.valid() for r in rs)
        with pytest.raises(_ClaimsAbandoned):
            pl.stage(rs)
        assert all(getattr(r, 'release', None) is None for r in rs)     # every claim given back (late: ignored)
        assert opt._claim_budget.held == 0
        # the ring and the stager still work: drain, then one more accepted iteration
        b.ring.set_claim_abandon(60.0)
        while b.consume_experience(0.0) is not None:
            pass
        for m in msgs[:2]:
            b.publish_experience(m, timeout=1.0)
        rs = [opt._consume_decode(stop, claim=True) for _ in range(2)]
        st = pl.stage(rs)
        pl.expand(st, {})
        assert st.n_seq == 2 and opt._claim_budget.held == 0
    finally:
        b.close(unlink=True)
