"""The reference's node topology on CPU (gloo): N DotaOptimizer ranks consume DISJOINT rollouts from ONE experience
queue fed by actor processes (competing consumers, /root/reference/optimizer.py:144-150), average gradients (DDP,
:274-277), and only rank 0 checkpoints and publishes the model (:284-287, ks-app/components/optimizer.jsonnet:79-174).
Exercised through ``learner.e2e.measure_e2e_node`` — the same code bench.py runs on every GPU rank — with both node
transports: the shared-memory ring and a TCP broker served from rank 0."""
import hashlib
import os
import socket

import pytest
import torch.multiprocessing as mp

from dotaclient_amd import native

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def _report(opt):
    flat = opt.learner.flat.flat.detach().cpu().numpy()
    files = sorted(os.listdir(opt.cfg.log_dir)) if os.path.isdir(opt.cfg.log_dir) else []
    return {'consumed': list(opt.consumed), 'weights': hashlib.sha256(flat.tobytes()).hexdigest(),
            'published': opt.n_published, 'models': [f for f in files if f.startswith('model_') and f.endswith('.pt')],
            'n_steps': opt.learner.n_steps}


def _worker(rank, world, port, transport, q):
    try:
        os.environ.update(MASTER_ADDR='127.0.0.1', MASTER_PORT=str(port), RANK=str(rank), WORLD_SIZE=str(world),
                          LOCAL_RANK=str(rank), LOCAL_WORLD_SIZE=str(world), OMP_NUM_THREADS='1')
        import torch
        import torch.distributed as dist
        torch.set_num_threads(1)
        dist.init_process_group('gloo', rank=rank, world_size=world)
        from dotaclient_amd.learner.e2e import measure_e2e_node
        r = measure_e2e_node(model='lstm128', device='cpu', backend='torch', duration=120.0, max_iterations=3,
                             warmup_iterations=1, games=6, threads=1, seq_len=16, batch_size=2, seq_per_epoch=4,
                             max_dota_time=12.0, prefetch=2, transport=transport, idle_probe=0.5, report=_report,
                             record_consumed=10000)
        q.put((rank, r))
        dist.barrier()
        dist.destroy_process_group()
    except BaseException as e:  # pragma: no cover
        import traceback
        q.put((rank, traceback.format_exc() + repr(e)))


@pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
@pytest.mark.parametrize('world,transport', [(2, 'shm'), (2, 'tcp'), (4, 'shm'), (4, 'tcp'), (8, 'shm'), (8, 'tcp')])
def test_learner_ranks_share_one_experience_queue(world, transport):
    import glob
    ctx = mp.get_context('spawn')
    q = ctx.Queue()
    port = _free_port()
    ps = [ctx.Process(target=_worker, args=(r, world, port, transport, q)) for r in range(world)]
    for p in ps:
        p.start()
    res = {}
    try:
        for _ in range(world):
            rank, r = q.get(timeout=600)
            assert isinstance(r, dict), r
            res[rank] = r
    finally:
        for p in ps:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
    assert all(p.exitcode == 0 for p in ps), [p.exitcode for p in ps]
    out = res[0]
    assert out['ranks'] == world and out['iterations'] == 3
    reports = out['reports']
    assert len(reports) == world
    # every rank ran the same DP steps and ends with the same weights
    assert len({rep['n_steps'] for rep in reports}) == 1 and reports[0]['n_steps'] > 0
    assert len({rep['weights'] for rep in reports}) == 1
    # competing consumers: no rollout was consumed by two ranks, every rank got some
    keys = [k for rep in reports for k in rep['consumed']]
    assert len(keys) == len(set(keys))
    assert all(len(rep['consumed']) > 0 for rep in reports)
    # only rank 0 checkpoints and publishes (model 0 at start + one per iteration)
    assert reports[0]['published'] >= 4 and len(reports[0]['models']) > 0
    assert all(rep['published'] == 0 and rep['models'] == [] for rep in reports[1:])
    assert out['steps_per_s'] > 0 and len(out['steps_per_s_per_rank']) == world
    assert out['actor_steps_per_s'] > 0 and out['queue_dropped'] >= 0
    assert glob.glob(f'/dev/shm/dca_e2e_{ps[0].pid}_*') == []      # rank 0 removed the node's ring + model slot
    # per-rank consumption counts and their skew (max / min rollouts per rank over the window)
    cons = out['rollouts_consumed_per_rank']
    assert len(cons) == world and all(c > 0 for c in cons)
    assert out['consumption_skew'] == max(cons) / min(cons)


@pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
def test_config5_node_loop_league_and_replay_cpu():
    """BASELINE config 5 through the node loop (bench.py league_replay): a PFSP league of published versions on the
    actor side and learners sampling every minibatch from the on-device replay ring (the fp8 actor step is the GPU
    part, tests/test_actor_fp8.py)."""
    from dotaclient_amd.learner.e2e import measure_e2e_node

    def report(opt):
        return {'replay': len(opt.replay), 'inserted': opt.replay.inserted, 'capacity': opt.replay.capacity,
                'n_steps': opt.learner.n_steps}
    r = measure_e2e_node(model='lstm128', device='cpu', backend='torch', duration=120.0, max_iterations=3,
                         warmup_iterations=1, games=6, threads=1, seq_len=16, batch_size=2, seq_per_epoch=4,
                         max_dota_time=12.0, prefetch=2, transport='shm', idle_probe=0.0, report=report,
                         league='pfsp', latest_weights_prob=0.5, replay_gb=0.002)
    rep = r['reports'][0]
    assert r['config']['league'] == 'pfsp' and r['config']['replay_gb'] == 0.002
    assert rep['capacity'] > 4 and rep['inserted'] >= 4 and rep['n_steps'] > 0
    assert r['steps_per_s'] > 0 and r['actor_steps_per_s'] > 0
