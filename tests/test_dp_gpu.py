"""The fused data-parallel learner step at world > 1 on the one available GPU.

RCCL cannot place two ranks on one device, so 2 and 4 ranks share ``cuda:0`` over the **gloo** backend on device
tensors — the same DataParallel code path as RCCL (bucketed async all-reduce on the comm stream, the count-carrying
last bucket with the has-grad flags and the kernel error flag, the split two-graph step whose early buckets are
launched between the graphs, has-grad division folded into the fused Adam). Every rank must end with identical
parameters, equal to a single-process oracle that sums the per-rank gradients and applies the same Adam step
(reference semantics: distributed.py:16-79).
"""
import os
import socket

import pytest
import torch

pytestmark = pytest.mark.gpu

STEPS, B, S = 3, 4, 32


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _batch(cfg, step, rank):
    from dotaclient_amd.learner.synthetic import make_batch
    return make_batch(B, S, cfg.layout, cfg.hidden, device='cuda', seed=1000 * step + rank)


def _worker(rank, world, port, precision, q):
    import torch.distributed as dist
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world))
        torch.cuda.set_device(0)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from dotaclient_amd.learner.engine import Learner, LossConfig
        from dotaclient_amd.models.policy import Policy, get_config
        cfg = get_config('lstm128')
        torch.manual_seed(100 + rank)          # different init per rank: the DP broadcast must equalise
        L = Learner(Policy(cfg), LossConfig(algo='ppo'), device='cuda', backend='fused', precision=precision)
        assert L.dp.enabled and L.enable_graph(warmup=1)
        for step in range(STEPS):
            L.train_step(_batch(cfg, step, rank))
        torch.cuda.synchronize()
        L.model.check_error()
        q.put((rank, L.flat.flat.cpu().numpy(), bool(L._split), L.graph is not None,
               L.dp.counts.cpu().numpy().copy()))
        dist.barrier()
        dist.destroy_process_group()
    except Exception as e:  # pragma: no cover
        q.put((rank, repr(e), None, None, None))


@pytest.mark.parametrize('world,precision', [(2, 'fp32'), (4, 'fp32'), (2, 'fp32-exact')])
def test_fused_dp_split_graph_step_multi_rank(gpu_ops, world, precision):
    import torch.multiprocessing as mp
    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.models.policy import Policy, get_config
    port = _free_port()
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    ps = [ctx.Process(target=_worker, args=(r, world, port, precision, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            r, flat, split, graphed, counts = q.get(timeout=240)
            assert split is not None, flat
            res[r] = (torch.from_numpy(flat), split, graphed, torch.from_numpy(counts))
    finally:
        for p in ps:
            p.join(timeout=60)
            if p.is_alive():
                p.kill()
    for r in range(world):
        assert res[r][1] and res[r][2], 'split two-graph step not used'
        assert torch.equal(res[r][0], res[0][0]), r
    cfg = get_config('lstm128')
    assert (res[0][3] == world).all()          # every parameter had a gradient on every rank
    # oracle: rank 0's initial weights, per-rank gradients summed, has-grad division inside the same fused Adam
    torch.manual_seed(100)
    L = Learner(Policy(cfg), LossConfig(algo='ppo'), device='cuda', backend='fused', dp=False, precision=precision)
    for step in range(STEPS):
        grads = []
        for r in range(world):
            bt, B_, S_ = L.batch_to_time_major(_batch(cfg, step, r))
            L._direct_body(bt, B_, S_)
            grads.append(L.flat.grad.clone())
        L.flat.grad.copy_(torch.stack(grads).sum(0))
        L.opt.step(L.dp.counts, divide=True)
    torch.cuda.synchronize()
    torch.testing.assert_close(res[0][0], L.flat.flat.cpu(), rtol=1e-5, atol=1e-6)
