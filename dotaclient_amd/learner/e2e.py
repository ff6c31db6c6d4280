"""End-to-end node measurement: actors → experience queue → learner → model broadcast → actors, on one GPU.

The reference's only published number is the optimizer's ``steps per s`` — sequence steps consumed per wall second
*including the wait for experience* (optimizer.py:485-486, README.md:35: ~1000 with 40 agents per optimizer). This
runs that loop for real, in one process:

* a :class:`~dotaclient_amd.actor.vec.VecActor` thread (native vectorised self-play + hipGraph batched policy)
  publishes whole-game DCX1 rollouts (the deploy's ``--rollout-size 9999``, params.libsonnet:19) into a bounded
  :class:`~dotaclient_amd.transport.broker.InProcBroker` (oldest dropped when full), with staggered first games so
  the lockstep games do not all publish on the same step;
* :class:`~dotaclient_amd.learner.optimizer.DotaOptimizer` (the learner runtime, unchanged: decode, device ingest
  with the return / GAE scan, hipGraph PPO steps, checkpoint + model publish every iteration) consumes them with
  the deploy's shape — batch 8 × seq_len 1400, 16 sequences per iteration, 1 epoch (params.libsonnet:7-24), with
  experience decoded ``prefetch`` messages ahead on a background thread (``prefetch_rollouts``) so the next
  iteration's decode overlaps this one's GPU training;
* every published model reaches the actor's :class:`~dotaclient_amd.actor.weights.WeightStore` and is hot-swapped
  into the actor graphs between steps, so ``avg_weight_age`` is real.

Both run on the same GPU (their kernels share the CUs). Reported: the reference metric (``steps per s``, padded
sequences as the reference counts them), the unpadded experience steps/s actually trained on, ``avg_weight_age``,
the actor's player-steps/s during the window and the queue drops.
"""
from __future__ import annotations

import logging
import shutil
import tempfile
import threading
import time
from typing import Dict, Optional

import numpy as np
import torch

logger = logging.getLogger(__name__)


def measure_e2e(model: str = 'lstm512', device='cuda', duration: float = 20.0, games: int = 1024,
                threads: int = 14, seq_len: int = 1400, batch_size: int = 8, seq_per_epoch: int = 16,
                epochs: int = 1, precision: str = 'fp32', max_dota_time: float = 600.0, rollout_size: int = 9999,
                queue_size: int = 64, warmup_iterations: int = 2, max_iterations: Optional[int] = None,
                log_dir: Optional[str] = None, prefetch: int = 32) -> Dict[str, float]:
    from ..actor.vec import VecActor
    from ..actor.weights import WeightStore
    from ..transport.broker import InProcBroker
    from .optimizer import DotaOptimizer, OptimizerConfig

    tmp = log_dir or tempfile.mkdtemp(prefix='dca_e2e_')
    broker = InProcBroker(maxsize=queue_size, drop_oldest=True)
    cfg = OptimizerConfig(log_dir=tmp, epochs=epochs, seq_per_epoch=seq_per_epoch, batch_size=batch_size,
                          seq_len=seq_len, model=model, precision=precision, device=str(device), checkpoint_keep=2,
                          run_local=True, xp_timeout=300.0, histogram_freq=10 ** 9, async_checkpoint=True,
                          prefetch_rollouts=prefetch)
    opt = DotaOptimizer(cfg, broker)                       # publishes model version 0
    ws = WeightStore(model, device='cpu')
    from concurrent.futures import ThreadPoolExecutor
    loader = ThreadPoolExecutor(1, thread_name_prefix='weights')
    # decode + load of a published model on its own thread (the in-proc broker calls subscribers synchronously)
    broker.subscribe_model(lambda v, b: loader.submit(ws.add_bytes, v, b))
    loader.submit(lambda: None).result()
    va = VecActor(ws, games, broker.publish_experience, device=device, seed=11, rollout_size=rollout_size,
                  max_dota_time=max_dota_time, hidden_stride=seq_len, threads=threads, stagger=True)
    for _ in range(3):                                     # capture the actor graphs before the learner's
        va.step()
    stop = threading.Event()
    err = []

    def actor_loop():
        try:
            while not stop.is_set():
                va.step()
        except BaseException as e:                         # surfaced on the main thread
            err.append(e)

    th = threading.Thread(target=actor_loop, name='vec-actor', daemon=True)
    th.start()
    try:
        rows, wall, (actor_steps, dropped) = _learner_loop(
            opt, duration, warmup_iterations, max_iterations,
            counters=lambda: (va.steps_taken, broker.n_dropped), check=lambda: err and err[0])
    finally:
        stop.set()
        opt.close()
        th.join(timeout=60)
        va.close()
        opt.flush_checkpoints()
        loader.shutdown(wait=True)
        if log_dir is None:
            shutil.rmtree(tmp, ignore_errors=True)
    return _summary(rows, wall, actor_steps, dropped, games, dict(
        batch_size=batch_size, seq_len=seq_len, seq_per_epoch=seq_per_epoch, epochs=epochs, rollout_size=rollout_size,
        max_dota_time=max_dota_time, precision=precision, prefetch_rollouts=prefetch, actor='thread'))


def _learner_loop(opt, duration, warmup_iterations, max_iterations, counters, check):
    """Run learner iterations for ``duration`` seconds after ``warmup_iterations``; per-iteration metric rows, the
    wall time and the (actor steps, dropped rollouts) deltas of the window."""
    from .optimizer import DotaOptimizer
    rows = []
    it = opt.iteration_start
    for _ in range(warmup_iterations):
        opt.run_iteration(it)
        it += 1
        e = check()
        if e:
            raise e
    t0 = time.perf_counter()
    c0 = counters()
    opt.time_last_step = time.time()
    while time.perf_counter() - t0 < duration and (max_iterations is None or len(rows) < max_iterations):
        opt.run_iteration(it)
        it += 1
        m = opt.last_metrics
        rows.append((m[DotaOptimizer.SPEED_KEY], m['avg_weight_age'], m['avg_rollout_len'],
                     m.get('time/train', float('nan')), m.get('time/ingest', float('nan')), m['experience_steps'],
                     m.get('time/h2d', float('nan')), m.get('time/log', float('nan')),
                     m.get('time/publish', float('nan'))))
        e = check()
        if e:
            raise e
    if opt.device.type == 'cuda':
        torch.cuda.synchronize(opt.device)
    wall = time.perf_counter() - t0
    c1 = counters()
    return rows, wall, (c1[0] - c0[0], c1[1] - c0[1])


def _summary(rows, wall, actor_steps, dropped, games, config):
    seq_per_epoch, seq_len = config['seq_per_epoch'], config['seq_len']
    a = np.asarray(rows, dtype=np.float64)
    n_it = len(rows)
    padded = n_it * seq_per_epoch * seq_len
    valid = float(a[:, 5].sum()) if n_it else 0.0         # unpadded experience steps consumed
    return {
        'steps_per_s': padded / wall if n_it else 0.0,          # the reference's 'steps per s' (padded, incl. wait)
        'valid_steps_per_s': valid / wall if n_it else 0.0,
        'iterations': n_it, 'wall_s': wall,
        'avg_weight_age': float(a[:, 1].mean()) if n_it else float('nan'),
        'avg_rollout_len': float(a[:, 2].mean()) if n_it else float('nan'),
        'train_ms_per_iteration': 1e3 * float(a[:, 3].mean()) if n_it else float('nan'),
        'ingest_ms_per_iteration': 1e3 * float(a[:, 4].mean()) if n_it else float('nan'),
        'h2d_ms_per_iteration': 1e3 * float(a[:, 6].mean()) if n_it else float('nan'),
        'log_ms_per_iteration': 1e3 * float(a[:, 7].mean()) if n_it else float('nan'),
        'publish_ms_per_iteration': 1e3 * float(a[:, 8].mean()) if n_it else float('nan'),
        'actor_steps_per_s': actor_steps / wall,
        'queue_dropped': int(dropped), 'games': games, 'config': config,
    }


def _actor_process_main(name: str, model: str, games: int, threads: int, seq_len: int, rollout_size: int,
                        max_dota_time: float, device: str, seed: int, stop, ready, steps, failed):
    """Actor role of :func:`measure_e2e_procs`: a process of its own (own interpreter and GIL) that plays ``games``
    VecActor games on the GPU, pushes whole-game rollouts into the node's shared-memory experience ring and hot-swaps
    every model the learner publishes into that broker's model slot."""
    try:
        from ..actor.vec import VecActor
        from ..actor.weights import WeightStore
        from ..transport.shm import ShmBroker
        br = ShmBroker(name, create=False, drop_oldest=True)
        ws = WeightStore(model, device='cpu')
        m = br.latest_model(timeout=120.0)
        if m is None:
            raise TimeoutError('no model published by the learner')
        ws.add_bytes(*m)
        br.subscribe_model(lambda v, b: ws.add_bytes(v, b), poll=0.005)
        va = VecActor(ws, games, br.publish_experience, device=device, seed=seed, rollout_size=rollout_size,
                      max_dota_time=max_dota_time, hidden_stride=seq_len, threads=threads, stagger=True)
        for _ in range(3):
            va.step()
        ready.set()
        while not stop.is_set():
            va.step()
            steps.value = va.steps_taken
        va.close()
        br.close()
    except BaseException:
        import traceback
        traceback.print_exc()
        failed.set()
        ready.set()


def measure_e2e_procs(model: str = 'lstm512', device='cuda', duration: float = 20.0, games: int = 1024,
                      threads: int = 14, seq_len: int = 1400, batch_size: int = 8, seq_per_epoch: int = 16,
                      epochs: int = 1, precision: str = 'fp32', max_dota_time: float = 600.0,
                      rollout_size: int = 9999, warmup_iterations: int = 2, max_iterations: Optional[int] = None,
                      log_dir: Optional[str] = None, prefetch: int = 32, ring_bytes: int = 1 << 26
                      ) -> Dict[str, float]:
    """:func:`measure_e2e` with the deploy's process split: the actor in a process of its own (spawned, same GPU)
    and the learner here, exchanging rollouts and models through the node-local shared-memory broker
    (``transport/shm.py``: native MPMC ring + model slot) instead of in-process queues — no GIL shared between the
    actor's host loop and the learner's ingest / publish threads. The ring holds ``ring_bytes`` (64 MB ≈ the thread
    variant's 64-rollout queue at the deploy's mean rollout size; the oldest rollouts are dropped when it is full),
    which bounds the experience's weight age."""
    import multiprocessing as mp
    import os
    from ..transport.shm import ShmBroker
    from .optimizer import DotaOptimizer, OptimizerConfig

    tmp = log_dir or tempfile.mkdtemp(prefix='dca_e2e_')
    name = f'dca_e2e_{os.getpid()}_{int(time.time() * 1e3) % 10 ** 9}'
    broker = ShmBroker(name, capacity=ring_bytes, create=True, drop_oldest=True)
    ctx = mp.get_context('spawn')
    stop, ready, failed = ctx.Event(), ctx.Event(), ctx.Event()
    steps = ctx.Value('q', 0)
    proc = None
    try:
        cfg = OptimizerConfig(log_dir=tmp, epochs=epochs, seq_per_epoch=seq_per_epoch, batch_size=batch_size,
                              seq_len=seq_len, model=model, precision=precision, device=str(device),
                              checkpoint_keep=2, run_local=True, xp_timeout=60.0, histogram_freq=10 ** 9,
                              async_checkpoint=True, prefetch_rollouts=prefetch)   # (a live actor sends ~1000/s)
        opt = DotaOptimizer(cfg, broker)                   # publishes model version 0 into the shm model slot
        proc = ctx.Process(target=_actor_process_main, name='e2e-actor', daemon=True,
                           args=(name, model, games, threads, seq_len, rollout_size, max_dota_time, str(device), 11,
                                 stop, ready, steps, failed))
        proc.start()
        if not ready.wait(timeout=600) or failed.is_set():
            raise RuntimeError('e2e actor process failed to start')

        def check():
            if failed.is_set() or not proc.is_alive():
                return RuntimeError('e2e actor process died')
            return None
        try:
            rows, wall, (actor_steps, _) = _learner_loop(opt, duration, warmup_iterations, max_iterations,
                                                         counters=lambda: (steps.value, 0), check=check)
        finally:
            opt.close()
            opt.flush_checkpoints()
    finally:
        stop.set()
        if proc is not None:
            proc.join(timeout=60)
            if proc.is_alive():
                proc.kill()
                proc.join(timeout=10)
        broker.close(unlink=True)
        if log_dir is None:
            shutil.rmtree(tmp, ignore_errors=True)
    out = _summary(rows, wall, actor_steps, -1, games, dict(
        batch_size=batch_size, seq_len=seq_len, seq_per_epoch=seq_per_epoch, epochs=epochs, rollout_size=rollout_size,
        max_dota_time=max_dota_time, precision=precision, prefetch_rollouts=prefetch, actor='process (shm broker)'))
    return out
