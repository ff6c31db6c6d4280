"""Learner runtime on the GPU with the overlapped host work: decode-ahead thread (``prefetch_rollouts``) and the
device-snapshot model publish + checkpoint writer (``async_checkpoint``). The published model, the checkpoint file
and the resumed trainer state must all be the weights of the iteration they are labelled with."""
import io
import os

import numpy as np
import pytest
import torch

from dotaclient_amd.constants import LAYOUT_1V1
from dotaclient_amd.transport.broker import InProcBroker
from dotaclient_amd.transport.codec import Rollout, encode

pytestmark = pytest.mark.gpu


def _rollout(i, T=48):
    rng = np.random.default_rng(i)
    U, A = LAYOUT_1V1.max_units, 21 + LAYOUT_1V1.max_units
    act = np.zeros((T, A), np.uint8)
    act[:, 0] = 1
    msk = np.zeros((T, A), np.uint8)
    msk[:, :3] = 1
    return Rollout(game_id=f'g{i}', team_id=2 + i % 2, player_id=0, weight_version=0,
                   env=rng.standard_normal((T, 3)).astype(np.float32),
                   units=rng.standard_normal((T, U, 10)).astype(np.float32), actions=act, masks=msk,
                   rewards=rng.standard_normal((T, 9)), logp=np.full(T, -1.0, np.float32),
                   values=np.zeros(T, np.float32), done=True)


def test_prefetch_and_async_publish_on_gpu(tmp_path):
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.utils import checkpoint as ckpt
    br = InProcBroker()
    for i in range(12):
        br.publish_experience(encode(_rollout(i)))
    cfg = OptimizerConfig(log_dir=str(tmp_path), model='lstm128', epochs=1, seq_per_epoch=4, batch_size=2,
                          seq_len=48, device='cuda', xp_timeout=30, async_checkpoint=True, prefetch_rollouts=3)
    opt = DotaOptimizer(cfg, br)
    opt.run(iterations=2)                       # run() joins the writer and stops the decode-ahead thread
    assert getattr(opt, '_prefetcher', None) is None
    assert np.isfinite(opt.last_metrics['loss/sum'])
    live = {k: v.detach().cpu() for k, v in opt.policy.state_dict().items()}
    version, body = br.latest_model()
    assert version == 2
    pub = torch.load(io.BytesIO(body), weights_only=True)
    disk = ckpt.load_model_file(os.path.join(str(tmp_path), 'model_000000002.pt'))
    for k, v in live.items():
        assert torch.equal(pub[k], v), k
        assert torch.equal(disk[k], v), k
    opt2 = DotaOptimizer(cfg, InProcBroker())
    assert opt2.iteration_start == 3
    torch.testing.assert_close(opt2.learner.opt.exp_avg, opt.learner.opt.exp_avg)
    torch.testing.assert_close(opt2.learner.opt.exp_avg_sq, opt.learner.opt.exp_avg_sq)


def test_e2e_actor_process_on_gpu():
    """bench.py's default e2e mode on the GPU: VecActor in a spawned process (its own HIP context on the same GPU)
    over the shared-memory broker, the learner here; rollouts flow, models flow back, the ring is unlinked."""
    import glob
    from dotaclient_amd.learner.e2e import measure_e2e_procs
    mine = f'/dev/shm/dca_e2e_{os.getpid()}_*'
    r = measure_e2e_procs(model='lstm128', device='cuda', duration=30.0, max_iterations=3, games=64, threads=4,
                          seq_len=128, batch_size=4, seq_per_epoch=8, max_dota_time=30.0, warmup_iterations=1)
    assert r['iterations'] == 3
    assert r['steps_per_s'] > 0 and r['actor_steps_per_s'] > 0
    assert 0 <= r['avg_weight_age'] < 16
    assert r['queue_dropped'] >= 0 and r['actor_idle_steps_per_s'] > 0
    assert glob.glob(mine) == []


def test_pipelined_ingest_matches_inline_on_gpu(tmp_path):
    """The stager thread (valid rows packed into a pinned slot, uploaded on a copy stream one iteration ahead,
    expanded to the padded layout on the device) trains on exactly what the inline ingest builds: same rollouts in
    the same order → bitwise-identical weights and reward statistics after three iterations (slots reused)."""
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    outs = []
    for prefetch in (0, 4):
        br = InProcBroker()
        for i in range(24):
            br.publish_experience(encode(_rollout(i, T=17 + 13 * i)))
        cfg = OptimizerConfig(log_dir=str(tmp_path / f'p{prefetch}'), model='lstm128', epochs=1, seq_per_epoch=4,
                              batch_size=2, seq_len=48, device='cuda', xp_timeout=30, prefetch_rollouts=prefetch,
                              graph=False)
        opt = DotaOptimizer(cfg, br)
        opt.run(iterations=3)
        assert opt._pipelined() == (prefetch > 0)
        outs.append((opt.learner.flat.flat.detach().cpu().clone(), opt.ema.detach().cpu().clone()))
    assert torch.equal(outs[0][0], outs[1][0])
    assert torch.equal(outs[0][1], outs[1][1])


def test_deferred_metrics_pool_growth_and_grad_norm(tmp_path):
    """with deferred metrics (the previous iteration's replays may still run when the next iteration
    starts) the per-iteration pool grows (a 10-sequence rollout after 4-sequence iterations): the growth waits for the
    pending replays before it frees their graphs and storage, and the run trains exactly like the non-deferred one.
    Every step's grad_norm is its own tensor (not the optimizer's one persistent norm), so the iteration mean is the
    mean over that iteration's steps."""
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    outs, norms = [], []
    for defer in (False, True):
        br = InProcBroker()
        lens = [48] * 8 + [480] + [48] * 16
        for i, T in enumerate(lens):
            br.publish_experience(encode(_rollout(i, T=T)))
        cfg = OptimizerConfig(log_dir=str(tmp_path / f'd{int(defer)}'), model='lstm128', epochs=1, seq_per_epoch=4,
                              batch_size=2, seq_len=48, device='cuda', xp_timeout=30, prefetch_rollouts=4,
                              async_checkpoint=True, defer_metrics=defer, graph=True)
        opt = DotaOptimizer(cfg, br)
        assert opt._defer_metrics() == defer
        seen = []
        fin = opt._finalize_iteration

        def spy(p, fin=fin, seen=seen):
            g = p['metrics_acc']['grad_norm']
            seen.append(([t.data_ptr() for t in g], [float(t) for t in g]))
            return fin(p)
        opt._finalize_iteration = spy
        opt.run(iterations=4)
        outs.append(opt.learner.flat.flat.detach().cpu().clone())
        norms.append([v for _, v in seen])
        for ptrs, _ in seen:
            assert len(set(ptrs)) == len(ptrs)
    assert torch.equal(outs[0], outs[1])
    assert norms[0] == norms[1]
