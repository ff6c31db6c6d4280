"""Multi-process data parallelism on CPU (gloo): the flat-bucket DP wrapper reproduces the reference's
``DistributedDataParallelSparseParamCPU`` semantics (distributed.py:16-79) and single-process large-batch math."""
import os
import socket

import pytest
import torch
import torch.distributed as dist
import torch.multiprocessing as mp


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _init(rank, world, port):
    os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
    torch.set_num_threads(1)               # up to 8 ranks share the 8 CPUs of the test box
    dist.init_process_group('gloo', rank=rank, world_size=world)


class Toy(torch.nn.Module):
    def __init__(self):
        super().__init__()
        self.a = torch.nn.Linear(4, 4)
        self.b = torch.nn.Linear(4, 4)
        self.c = torch.nn.Linear(4, 4)   # never used: must stay untouched


def _toy_worker(rank, world, port, q, split=False):
    try:
        _init(rank, world, port)
        from dotaclient_amd.parallel.dp import DataParallel
        torch.manual_seed(100 + rank)          # different init per rank → broadcast must equalise
        m = Toy()
        dp = DataParallel(m, bucket_cap_mb=0.0001, overlap=False)
        if split:     # the learner's two-phase layout: b, c early (own buckets), a last with the counts
            assert dp.split_buckets([2, 3, 4, 5], cap_mb=0.0001)
            assert dp.buckets[-1] == [1, 0]
        x = torch.full((2, 4), float(rank + 1))
        out = m.a(x).sum()
        if rank == 0:
            out = out + m.b(x).sum()           # only rank 0 produces a gradient for b
        dp.zero_grad()
        out.backward()
        if split:
            dp.launch_early()
        dp.sync()
        # numpy, not torch tensors: torch.multiprocessing shares tensors by fd through the child's resource sharer,
        # which is gone once the child exits — the parent may unpickle later (flaky FileNotFoundError)
        q.put((rank, {k: v.detach().numpy().copy() for k, v in m.state_dict().items()},
               {n: p.grad.numpy().copy() for n, p in m.named_parameters()}, dp.counts.numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None, None))


@pytest.mark.parametrize('world,split', [(2, False), (2, True), (4, True), (8, False), (8, True)])
def test_sparse_param_semantics(world, split):
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_toy_worker, args=(r, world, port, q, split)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, sd, grads, counts = q.get(timeout=120)
        assert grads is not None, sd
        res[r] = ({k: torch.from_numpy(v) for k, v in sd.items()}, {k: torch.from_numpy(v) for k, v in grads.items()},
                  torch.from_numpy(counts))
    for p in ps:
        p.join(timeout=60)
    sd0, g0, c0 = res[0]
    for r in range(1, world):
        sdr, gr, _ = res[r]
        for k in sd0:
            assert torch.equal(sd0[k], sdr[k]), k      # rank-0 broadcast at construction
        for k in g0:
            assert torch.equal(g0[k], gr[k]), k        # identical reduced grads on every rank (fixes §2.10-8)
    names = list(g0)
    counts = dict(zip(names, c0.tolist()))
    assert counts['a.weight'] == world and counts['b.weight'] == 1 and counts['c.weight'] == 0
    # a: mean over ranks of per-rank grads (x = rank + 1) → column sums 2·mean(1..world) = world + 1
    assert torch.allclose(g0['a.weight'], torch.full((4, 4), float(world + 1)))
    # b: only rank 0 had it → divided by its count 1
    assert torch.allclose(g0['b.weight'], torch.full((4, 4), 2.0))
    assert torch.count_nonzero(g0['c.weight']) == 0


def _learner_worker(rank, world, port, q, batch_seed):
    try:
        _init(rank, world, port)
        from dotaclient_amd.learner.engine import Learner, LossConfig
        from dotaclient_amd.learner.synthetic import make_batch
        from dotaclient_amd.models.policy import Policy, get_config
        torch.manual_seed(0)
        cfg = get_config('lstm128')
        L = Learner(Policy(cfg), LossConfig(algo='ppo', vf_coef=0.0), device='cpu', backend='torch', overlap=False)
        b = make_batch(4, 16, cfg.layout, cfg.hidden, seed=batch_seed + rank)
        L.train_step(b)
        q.put((rank, L.flat.flat.numpy().copy(), L.dp.counts.numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


@pytest.mark.parametrize('world', [2, 4, 8])
def test_dp_step_equals_single_process_average(world):
    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.learner.synthetic import make_batch
    from dotaclient_amd.models.policy import Policy, get_config
    port, seed = _free_port(), 11
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_learner_worker, args=(r, world, port, q, seed)) for r in range(world)]
    for p in ps:
        p.start()
    out = {}
    for _ in range(world):
        r, flat, counts = q.get(timeout=180)
        assert counts is not None, flat
        out[r] = (torch.from_numpy(flat), torch.from_numpy(counts))
    for p in ps:
        p.join(timeout=60)
    for r in range(1, world):
        assert torch.equal(out[0][0], out[r][0])
    # single-process oracle: average of the two per-rank gradients, same optimizer step
    torch.manual_seed(0)
    cfg = get_config('lstm128')
    L = Learner(Policy(cfg), LossConfig(algo='ppo', vf_coef=0.0), device='cpu', backend='torch', dp=False)
    grads = []
    for r in range(world):
        L.dp.zero_grad()
        loss, _ = L.loss(make_batch(4, 16, cfg.layout, cfg.hidden, seed=seed + r))
        loss.backward()
        grads.append(L.flat.grad.clone())
    L.flat.grad.copy_(sum(grads) / world)
    counts = out[0][1]
    names = L.flat.names
    assert counts[names.index('affine_value.weight')] == 0      # vf_coef = 0: value head has no grad anywhere
    L.opt.step(counts)
    torch.testing.assert_close(L.flat.flat, out[0][0], rtol=1e-5, atol=1e-6)


def _resume_worker(rank, world, port, root, q):
    try:
        _init(rank, world, port)
        from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
        from dotaclient_amd.transport.broker import InProcBroker
        # rank 0 sees the run's checkpoint directory, rank 1 a fresh, empty node-local directory
        ld = os.path.join(root, 'run') if rank == 0 else os.path.join(root, f'empty{rank}')
        cfg = OptimizerConfig(log_dir=ld, batch_size=2, seq_len=16, seq_per_epoch=2, epochs=1, model='lstm128',
                              device='cpu', backend='torch')
        opt = DotaOptimizer(cfg, InProcBroker(), checkpoint=rank == 0)
        q.put((rank, opt.iteration_start, opt.learner.opt.exp_avg.numpy().copy(),
               opt.learner.opt.steps.numpy().copy(), opt.learner.flat.flat.numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None, None, None))


def test_resume_equalises_iteration_and_optimizer_state(tmp_path):
    """Only rank 0 can read the checkpoint (reference workers restart at iteration 1 with fresh Adam state,
    §2.10-7): every rank must resume at rank 0's iteration with rank 0's weights AND optimizer moments."""
    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.models.policy import Policy, get_config
    from dotaclient_amd.utils import checkpoint as ckpt
    torch.manual_seed(3)
    pol = Policy(get_config('lstm128'))
    L = Learner(pol, LossConfig(), device='cpu', backend='torch', dp=False)
    L.opt.exp_avg.normal_()
    L.opt.steps.fill_(41)
    run = tmp_path / 'run'
    ckpt.save_model(pol.state_dict(), str(run), 41)
    ckpt.save_trainer_state({'learner': L.state_dict(), 'running': {'factor': 0.99, 'mean': {}, 'std': {}},
                             'iteration': 41}, str(run), 41)
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_resume_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = dict((r[0], tuple(torch.from_numpy(x) if hasattr(x, 'dtype') else x for x in r[1:]))
               for r in (q.get(timeout=300) for _ in range(world)))
    for p in ps:
        p.join(timeout=60)
    assert all(isinstance(v[0], int) for v in res.values()), res
    assert res[0][0] == res[1][0] == 42
    torch.testing.assert_close(res[1][1], res[0][1])
    torch.testing.assert_close(res[0][1], L.opt.exp_avg)
    assert (res[1][2] == 41).all()
    torch.testing.assert_close(res[1][3], res[0][3])


@pytest.mark.parametrize('preset', ['lstm512', '5v5'])
def test_split_buckets_on_policy_layout(preset):
    """The learner's DP split (recurrence / pre-RNN / heads early, encoder last with the counts) is a valid bucket
    layout on the real policy's flat buffer (64-element aligned offsets): two disjoint contiguous ranges."""
    from dotaclient_amd.models.policy import Policy, get_config
    from dotaclient_amd.parallel.dp import DataParallel
    pol = Policy(get_config(preset))
    dp = DataParallel(pol, overlap=False, broadcast=False)
    names = [n for n, _ in pol.named_parameters()]
    pre = ('affine_pre_rnn.', 'rnn.', 'affine_head_enum.', 'affine_move_', 'affine_unit_attention.', 'affine_value.')
    early = [i for i, n in enumerate(names) if n.startswith(pre)]
    assert dp.split_buckets(early)
    late = sorted(dp.buckets[-1])
    assert set(late) == set(range(len(names))) - set(early)
    assert all(n.startswith(('affine_env', 'affine_unit_basic', 'entity_attn')) or
               (n.startswith('affine_unit_') and 'attention' not in n) for n in (names[i] for i in late))
    (llo, lhi) = dp.bucket_ranges[-1]
    for lo, hi in dp.bucket_ranges[:-1]:
        assert hi <= llo or lo >= lhi


def _uneven_worker(rank, world, port, root, q):
    """Every rank gets rollouts of different lengths: 5 and 7 sequences of 16 steps → 4 and 6 full minibatch rows
    of 2. Without the MIN agreement rank 1 would run a third train_step (and all-reduce) that rank 0 never joins."""
    try:
        _init(rank, world, port)
        import numpy as np
        from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
        from dotaclient_amd.transport.broker import InProcBroker
        from dotaclient_amd.transport.codec import Rollout, encode
        cfg = OptimizerConfig(log_dir=os.path.join(root, f'r{rank}'), batch_size=2, seq_len=16, seq_per_epoch=4,
                              epochs=1, model='lstm128', device='cpu', backend='torch', xp_timeout=30)
        br = InProcBroker()
        opt = DotaOptimizer(cfg, br, checkpoint=rank == 0)
        rng = np.random.default_rng(rank)
        U = opt.policy_cfg.layout.max_units
        for T in ((16 * 5 - 3,) if rank == 0 else (16 * 7 - 1,)):
            act = np.zeros((T, 21 + U), np.uint8)
            act[:, 0] = 1
            br.publish_experience(encode(Rollout(
                game_id=f'g{rank}', team_id=2, player_id=0, weight_version=0,
                env=rng.standard_normal((T, 3)).astype(np.float32),
                units=rng.standard_normal((T, U, 10)).astype(np.float32), actions=act,
                masks=np.ones((T, 21 + U), np.uint8), rewards=rng.standard_normal((T, 9)),
                logp=np.full(T, -1.0, np.float32), values=np.zeros(T, np.float32), done=True)))
        opt.run(iterations=1)
        q.put((rank, opt.learner.flat.flat.numpy().copy(), opt.learner.n_steps))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None))


def test_ranks_with_uneven_rollouts_run_the_same_steps(tmp_path):
    world, port = 2, _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_uneven_worker, args=(r, world, port, str(tmp_path), q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    for _ in range(world):
        r, flat, steps = q.get(timeout=300)
        assert steps is not None, flat
        res[r] = (flat, steps)
    for p in ps:
        p.join(timeout=60)
    assert res[0][1] == res[1][1] == 2            # min(5, 7) sequences → 4 rows → 2 minibatches on both ranks
    assert (res[0][0] == res[1][0]).all()
