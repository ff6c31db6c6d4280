"""On-HBM replay ring buffer (learner/replay.py): ring semantics, newest-window sampling, byte budgeting, and the
optimizer training from it."""
import pytest
import torch

from dotaclient_amd.constants import LAYOUT_1V1
from dotaclient_amd.learner.replay import HbmReplay, bytes_per_sequence
from dotaclient_amd.learner.synthetic import make_batch


def _batch(n, S, seed, hidden=128):
    b = make_batch(n, S, LAYOUT_1V1, hidden, device='cpu', seed=seed)
    b['ret'] = torch.full((n, S), float(seed))        # tag rows by their batch seed
    return b


def test_ring_wraps_and_keeps_newest():
    r = HbmReplay(5, 8, LAYOUT_1V1, 128, 'cpu')
    for seed in range(3):                              # 3 adds of 2 → 6 rows into capacity 5
        r.add(_batch(2, 8, seed), version=seed)
    assert len(r) == 5 and r.inserted == 6 and r.cursor == 1
    tags = r.data['ret'][:, 0].tolist()
    assert sorted(tags) == [0.0, 1.0, 1.0, 2.0, 2.0]  # the oldest row was overwritten
    assert r.version.tolist().count(2) == 2


def test_prefill_replicates_to_capacity_and_new_rows_overwrite_copies():
    r = HbmReplay(11, 4, LAYOUT_1V1, 32, 'cpu')
    r.add(_batch(3, 4, 7, hidden=32), version=5)
    assert r.fill_fraction == pytest.approx(3 / 11)
    assert r.prefill() == 8 and len(r) == 11 and r.fill_fraction == 1.0
    for k, v in r.data.items():                        # every row is a copy of one of the 3 added sequences
        for i in range(11):
            assert torch.equal(v[i], v[i % 3]), k
    assert r.version.tolist() == [5, 5, 5] + [-1] * 8
    r.add(_batch(2, 4, 9, hidden=32), version=6)        # lands at the cursor, over the oldest copies
    assert r.cursor == 5 and r.version.tolist()[3:5] == [6, 6] and len(r) == 11
    assert r.prefill() == 0


def test_recent_window_sampling_only_returns_newest():
    r = HbmReplay(16, 4, LAYOUT_1V1, None, 'cpu', seed=1)
    for seed in range(8):
        r.add(_batch(2, 4, seed, hidden=None), version=seed)
    s = r.sample(64, recent=2)
    assert set(s['ret'][:, 0].tolist()) == {7.0}
    s = r.sample(256)
    assert set(s['ret'][:, 0].tolist()) == set(float(i) for i in range(8))
    assert s['units'].shape == (256, 4, LAYOUT_1V1.max_units, 10) and s['actions'].dtype == torch.uint8


def test_capacity_for_bytes_matches_allocation():
    S, H = 1400, 512
    per = bytes_per_sequence(S, LAYOUT_1V1, H)
    assert 2.0e6 < per < 3.0e6                        # ≈2.4 MB per 1400-step LSTM-512 sequence
    cap = HbmReplay.capacity_for_bytes(10 * per + 5, S, LAYOUT_1V1, H)
    assert cap == 10
    r = HbmReplay(3, 16, LAYOUT_1V1, 64, 'cpu')
    assert r.nbytes == 3 * bytes_per_sequence(16, LAYOUT_1V1, 64)


def test_replay_keeps_packed_episode_starts():
    """Packed sequences (learner/ingest.py SequencePacker) keep their episode-start flags in the ring; unpacked
    batches added to a packing ring get none; the time-major gather hands them to the step."""
    from dotaclient_amd.learner.engine import Learner
    S = 6
    r = HbmReplay(4, S, LAYOUT_1V1, 64, 'cpu', reset=True)
    assert r.nbytes == 4 * bytes_per_sequence(S, LAYOUT_1V1, 64, reset=True)
    b = _batch(2, S, 1, hidden=64)
    b['reset'] = torch.zeros(2, S, dtype=torch.uint8)
    b['reset'][1, 3] = 1
    r.add(b)
    r.add(_batch(1, S, 2, hidden=64))                  # no flags: zero-filled
    assert r.data['reset'][:3].sum().item() == 1 and r.data['reset'][1, 3].item() == 1
    import types
    out = Learner.gather_time_major(types.SimpleNamespace(STEP_FIELDS=Learner.STEP_FIELDS), r, torch.tensor([1, 2]), S)
    rst = out['reset'].view(S, 2)                      # time-major rows t·B + b
    assert rst[3, 0].item() == 1 and rst.sum().item() == 1
    assert 'reset' not in HbmReplay(2, S, LAYOUT_1V1, 64, 'cpu').data


def test_optimizer_trains_from_replay(tmp_path):
    import numpy as np
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.broker import InProcBroker
    from dotaclient_amd.transport.codec import Rollout, encode
    br = InProcBroker()
    cfg = OptimizerConfig(log_dir=str(tmp_path), model='lstm128', epochs=2, seq_per_epoch=4, batch_size=2,
                          seq_len=16, device='cpu', replay_capacity=6, xp_timeout=30)
    opt = DotaOptimizer(cfg, br)
    rng = np.random.default_rng(0)
    U, A = LAYOUT_1V1.max_units, 21 + LAYOUT_1V1.max_units
    for i in range(8):
        T = 16
        act = np.zeros((T, A), np.uint8)
        act[:, 0] = 1
        msk = np.zeros((T, A), np.uint8)
        msk[:, :3] = 1
        br.publish_experience(encode(Rollout(
            game_id=f'g{i}', team_id=2 + i % 2, player_id=0, weight_version=0, env=rng.standard_normal((T, 3)).astype(np.float32),
            units=rng.standard_normal((T, U, 10)).astype(np.float32), actions=act, masks=msk,
            rewards=rng.standard_normal((T, 9)), logp=np.full(T, -1.0, np.float32),
            values=np.zeros(T, np.float32), done=True)))
    opt.run(iterations=2)
    assert len(opt.replay) == 6 and opt.replay.inserted == 8
    assert np.isfinite(opt.last_metrics['loss/sum']) and opt.last_metrics['replay/size'] == 6.0


@pytest.mark.gpu
def test_replay_on_hbm_large(gpu_ops):
    """A multi-GB on-device buffer: add/sample stay on the GPU and return the right rows."""
    S, H = 1400, 512
    cap = HbmReplay.capacity_for_bytes(8e9, S, LAYOUT_1V1, H)
    r = HbmReplay(cap, S, LAYOUT_1V1, H, 'cuda')
    assert r.nbytes > 7e9
    b = {k: v.cuda() for k, v in _batch(4, S, 3, hidden=H).items()}
    r.add(b, version=1)
    s = r.sample(8)
    assert s['units'].is_cuda and torch.equal(s['ret'][:, 0].cpu(), torch.full((8,), 3.0))


@pytest.mark.gpu
def test_replay_200gb_on_hbm_accounting_and_training(gpu_ops):
    """BASELINE config 5's on-HBM replay at scale: a 200 GB buffer of 1400-step LSTM-512 sequences. The bytes the
    driver reports as taken match ``nbytes`` (and ``bytes_per_sequence`` × capacity), writes across the ring's wrap
    point land where expected, and the fused learner trains from it."""
    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.learner.replay import bytes_per_sequence
    from dotaclient_amd.models.policy import Policy, get_config
    S, H, budget = 1400, 512, 200e9
    torch.cuda.synchronize()
    torch.cuda.empty_cache()                       # earlier tests' cached blocks must not be reused here
    free0, total = torch.cuda.mem_get_info()
    alloc0 = torch.cuda.memory_allocated()
    if free0 < budget + 20e9:
        pytest.skip(f'needs {budget / 1e9 + 20:.0f} GB free HBM, have {free0 / 1e9:.0f}')
    cap = HbmReplay.capacity_for_bytes(budget, S, LAYOUT_1V1, H)
    r = HbmReplay(cap, S, LAYOUT_1V1, H, 'cuda')
    torch.cuda.synchronize()
    free1, _ = torch.cuda.mem_get_info()
    assert 0.995 * budget <= r.nbytes <= budget
    assert abs(r.nbytes - (cap * bytes_per_sequence(S, LAYOUT_1V1, H) + cap * 8)) < 1e6
    # the allocator's and the driver's view: the buffer really is resident HBM of that size
    assert abs((torch.cuda.memory_allocated() - alloc0) - r.nbytes) < 1e-3 * r.nbytes
    assert free0 - free1 >= 0.99 * r.nbytes, (free0 - free1, r.nbytes)
    # fill up to the wrap point, then write across it
    r.cursor = cap - 2
    b = {k: v.cuda() for k, v in _batch(4, S, 7, hidden=H).items()}
    r.add(b, version=5)
    assert r.cursor == 2 and int(r.version[cap - 1]) == 5 and int(r.version[1]) == 5
    assert torch.equal(r.data['ret'][cap - 2, 0].cpu(), torch.tensor(7.0)) and float(r.data['ret'][1, 0]) == 7.0
    L = Learner(Policy(get_config('lstm512')), LossConfig(algo='ppo'), device='cuda', backend='fused', dp=False)
    m = L.train_step_replay(r, 4, recent=4)
    torch.cuda.synchronize()
    assert torch.isfinite(m['loss'])
    del r


@pytest.mark.gpu
def test_sample_into_host_ring(gpu_ops):
    """sample_into: host-sampled positions written into a device index buffer by one pinned copy per call (the
    captured learner step's index buffer), newest-first window like sample_indices, ring slots reused safely."""
    rep = HbmReplay(10, 8, LAYOUT_1V1, 32, 'cuda', seed=3)
    rep.add(make_batch(7, 8, LAYOUT_1V1, 32, device='cuda', seed=1))
    out = torch.empty(5, dtype=torch.long, device='cuda')
    seen = set()
    for _ in range(12):                                  # > ring size: slots are recycled behind their copies
        rep.sample_into(out, recent=3)
        v = out.cpu().tolist()
        assert all(i in (4, 5, 6) for i in v), v          # the 3 newest of the 7 written positions
        seen.update(v)
    assert seen == {4, 5, 6}
    rep.add(make_batch(6, 8, LAYOUT_1V1, 32, device='cuda', seed=2))   # wraps: newest are 12 mod 10 = 2 … back
    rep.sample_into(out)
    assert all(0 <= i < 10 for i in out.cpu().tolist())
