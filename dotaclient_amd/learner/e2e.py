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
import os
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
                log_dir: Optional[str] = None, prefetch: int = 32, pack: bool = False,
                old_logp: str = 'actor', advantages: str = 'vtrace-step') -> Dict[str, float]:
    from ..actor.vec import VecActor
    from ..actor.weights import WeightStore
    from ..transport.broker import InProcBroker
    from .optimizer import DotaOptimizer, OptimizerConfig

    tmp = log_dir or tempfile.mkdtemp(prefix='dca_e2e_')
    broker = InProcBroker(maxsize=queue_size, drop_oldest=True)
    cfg = OptimizerConfig(log_dir=tmp, epochs=epochs, seq_per_epoch=seq_per_epoch, batch_size=batch_size,
                          seq_len=seq_len, model=model, precision=precision, device=str(device), checkpoint_keep=2,
                          run_local=True, xp_timeout=300.0, histogram_freq=10 ** 9, async_checkpoint=True,
                          prefetch_rollouts=prefetch, pack_sequences=pack, old_logp=old_logp,
                          advantages=advantages)
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


def _learner_loop(opt, duration, warmup_iterations, max_iterations, counters, check, agree=None):
    """Run learner iterations for ``duration`` seconds after ``warmup_iterations``; per-iteration metric rows, the
    wall time and the (actor steps, dropped rollouts) deltas of the window. ``agree(local_continue) -> bool``
    makes data-parallel ranks stop on the same iteration (every rank runs the same number of DP steps)."""
    from .optimizer import DotaOptimizer
    rows = []
    _learner_loop.metrics = {}
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
    while True:
        cont = time.perf_counter() - t0 < duration and (max_iterations is None or len(rows) < max_iterations)
        if agree is not None:
            cont = agree(cont)
        if not cont:
            break
        opt.run_iteration(it)
        it += 1
        m = opt.last_metrics
        rows.append((m[DotaOptimizer.SPEED_KEY], m['avg_weight_age'], m['avg_rollout_len'],
                     m.get('time/train', float('nan')), m.get('time/ingest', float('nan')), m['experience_steps'],
                     m.get('time/h2d', float('nan')), m.get('time/log', float('nan')),
                     m.get('time/publish', float('nan')), m.get('time/lookahead', 0.0),
                     m.get('time/gpu_train_ms_per_step', float('nan')), m.get('rollouts_consumed', float('nan')),
                     m.get('time/stage', float('nan')), m.get('time/gather', float('nan')),
                     m.get('time/stage_wait', float('nan')), m.get('time/stage_copy', float('nan')),
                     m.get('time/stage_release', float('nan'))))
        for k, v in m.items():      # PPO / off-policy diagnostics of the window (means, _learner_loop.metrics)
            if k in ('approx_kl', 'clipfrac', 'avg_weight_age') or k.startswith('offpolicy/'):
                acc = _learner_loop.metrics.setdefault(k, [0.0, 0])
                acc[0] += float(v)
                acc[1] += 1
        e = check()
        if e:
            raise e
    if opt.device.type == 'cuda':
        torch.cuda.synchronize(opt.device)
    wall = time.perf_counter() - t0
    c1 = counters()
    opt.flush_metrics()            # the last iteration's deferred metrics / logs (outside the timed window)
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
        # taking + expanding the next iteration's rollouts while this one's steps run (look-ahead ingest)
        'lookahead_ms_per_iteration': 1e3 * float(a[:, 9].mean()) if n_it else float('nan'),
        # GPU time from the first to the last training step of an iteration, per step, INSIDE the node loop (actor
        # graph replays and host enqueue gaps included) — compare with the learner-alone ms_per_step
        'learner_gpu_ms_per_step': float(np.nanmean(a[:, 10])) if n_it and np.isfinite(a[:, 10]).any() else float('nan'),
        # the slowest iteration's steps (a device-wide stall — queue preemption, memory eviction — shows here)
        'learner_gpu_ms_per_step_max': float(np.nanmax(a[:, 10])) if n_it and np.isfinite(a[:, 10]).any() else float('nan'),
        'rollouts_consumed': int(np.nansum(a[:, 11])) if n_it else 0,
        # the stager thread per iteration: packing + upload issue, and waiting for the decoded rollouts
        'stage_ms_per_iteration': 1e3 * float(np.nanmean(a[:, 12])) if n_it and np.isfinite(a[:, 12]).any() else float('nan'),
        'gather_ms_per_iteration': 1e3 * float(np.nanmean(a[:, 13])) if n_it and np.isfinite(a[:, 13]).any() else float('nan'),
        # part of stage_ms spent waiting for a free upload slot (the stager ahead of the learner)
        'stage_wait_ms_per_iteration': 1e3 * float(np.nanmean(a[:, 14])) if n_it and np.isfinite(a[:, 14]).any() else float('nan'),
        'stage_copy_ms_per_iteration': 1e3 * float(np.nanmean(a[:, 15])) if n_it and np.isfinite(a[:, 15]).any() else float('nan'),
        'stage_release_ms_per_iteration': 1e3 * float(np.nanmean(a[:, 16])) if n_it and np.isfinite(a[:, 16]).any() else float('nan'),
        'actor_steps_per_s': actor_steps / wall,
        'queue_dropped': int(dropped), 'games': games, 'config': config,
    }


def open_node_broker(addr: str, drop_oldest: bool = True):
    """Client of the node's experience / model broker: ``shm://name`` (native ring + model slot in /dev/shm) or
    ``tcp://host:port`` (TcpBrokerServer)."""
    if addr.startswith('shm://'):
        from ..transport.shm import ShmBroker
        return ShmBroker(addr[6:], create=False, drop_oldest=drop_oldest)
    from ..transport.broker import make_broker
    return make_broker(addr)


def _actor_process_main(addr: str, model: str, games: int, threads: int, seq_len: int, rollout_size: int,
                        max_dota_time: float, device: str, seed: int, stop, ready, steps, failed, tag: str = 'a0',
                        league: Optional[str] = None, latest_weights_prob: float = 1.0,
                        precision: str = 'bf16'):
    """Actor role of :func:`measure_e2e_node`: a process of its own (own interpreter and GIL) that plays ``games``
    VecActor games on its GPU, pushes whole-game rollouts into the node's experience queue and hot-swaps every model
    the learner's rank 0 publishes (reference agent.py:855-902 with the model subscription of 198-223). It tears its
    threads down before returning, so the process exits with status 0.

    The process runs at a lower CPU priority (nice 5): actor and learner share the rank's
    CPU share, and when the learner's decode / stager threads lose the CPU to the actor's workers the queue
    overflows (drops) while the learner waits for its next staged iteration — actor work that is thrown away."""
    br = None
    try:
        try:
            os.nice(5)
        except OSError:
            pass
        from ..actor.vec import VecActor
        from ..actor.weights import WeightStore
        if device.startswith('cuda') and torch.device(device).index is not None:
            torch.cuda.set_device(torch.device(device))
        br = open_node_broker(addr, drop_oldest=True)
        ws = WeightStore(model, device='cpu')
        m = br.latest_model(timeout=600.0)
        if m is None:
            raise TimeoutError('no model published by the learner')
        ws.add_bytes(*m)
        br.subscribe_model(lambda v, b: ws.add_bytes(v, b), poll=0.005 if addr.startswith('shm://') else 0.25)
        lg = None
        if league:
            # self-play league (reference agent.py:760-765 mini-league; PFSP opponents by default): the latest
            # weights play the sampled opponent version with probability 1 - latest_weights_prob
            from ..actor.league import League
            lg = League(ws, mode=league)
        from ..models.policy import get_config
        mode = '5v5' if get_config(model).layout.counts[0] > 1 else '1v1'   # (BASELINE config 4: 5v5 self-play)
        # on the node's shared-memory ring the engine encodes finished rollouts straight into it (VecActor ring_sink)
        sink = br if hasattr(br, 'ring') else None
        # (DCA_E2E_ACTOR_GROUPS: software-pipelined game groups of the actor, default 2 — A/B of the launch shape)
        groups = int(os.environ.get('DCA_E2E_ACTOR_GROUPS', '2'))
        va = VecActor(ws, games, br.publish_experience, device=device, mode=mode, seed=seed,
                      rollout_size=rollout_size, max_dota_time=max_dota_time, hidden_stride=seq_len, threads=threads,
                      stagger=True, tag=f'{tag}.vec', league=lg, latest_weights_prob=latest_weights_prob,
                      precision=precision, ring_sink=sink, groups=groups)   # (game ids unique across the node)
        for _ in range(3):
            va.step()
        ready.set()
        while not stop.is_set():
            va.step()
            steps.value = va.steps_taken
        va.close()
    except BaseException:
        import traceback
        traceback.print_exc()
        failed.set()
        ready.set()
    finally:
        if br is not None:
            br.close()                  # joins the model subscriber thread


def _feeder_process_main(addr: str, model: str, seq_len: int, stop, ready, steps, failed, seed: int = 0):
    """Diagnostic stand-in for the actor process (DCA_E2E_FEEDER=1): republishes a fixed set of synthetic raw
    rollouts (random records, whole games of 300-900 steps) into the node's experience queue as fast as the ring takes
    them, with no GPU work at all — the learner's in-loop step without the actor's kernels beside it."""
    br = None
    try:
        import numpy as np
        from ..models.policy import get_config
        from ..transport.codec import Rollout, encode
        br = open_node_broker(addr, drop_oldest=True)
        U = get_config(model).layout.max_units
        A = 21 + U
        rng = np.random.default_rng(seed)
        msgs = []
        for i in range(48):
            T = int(rng.integers(300, 900))
            raw = np.zeros((T, U, 8), np.int32)
            f = raw.view(np.float32)
            f[..., :2] = rng.uniform(-7000, 7000, (T, U, 2))
            f[..., 2] = 128.0
            f[..., 3] = rng.uniform(0, 360, (T, U))
            f[..., 4] = rng.uniform(0, 1, (T, U))
            raw[..., 5] = rng.integers(1, 5000, (T, U))
            raw[..., 6] = np.where(rng.random((T, U)) < 0.4, 1, 0)
            hero = np.zeros((T, 4), np.float32)
            hero[:, :2] = rng.uniform(-7000, 7000, (T, 2))
            hero[:, 2] = 600.0
            act = np.zeros((T, A), np.uint8)
            act[np.arange(T), rng.integers(0, 3, T)] = 1
            msk = np.zeros((T, A), np.uint8)
            msk[:, :3] = 1
            r = Rollout(game_id=f'feed{seed}_{i}', team_id=2 + i % 2, player_id=0, weight_version=0,
                        env=rng.standard_normal((T, 3)).astype(np.float32), units=None, units_raw=raw, hero=hero,
                        actions=act, masks=msk, rewards=rng.standard_normal((T, 9)) * 0.1,
                        logp=np.full(T, -1.1, np.float32), values=np.zeros(T, np.float32), done=True)
            msgs.append((encode(r), T))
        ready.set()
        k = 0
        while not stop.is_set():
            b, T = msgs[k % len(msgs)]
            br.publish_experience(b)
            steps.value += T
            k += 1
    except BaseException:
        import traceback
        traceback.print_exc()
        failed.set()
        ready.set()
    finally:
        if br is not None:
            br.close()


def measure_e2e_node(model: str = 'lstm512', device='cuda', duration: float = 20.0, games: int = 1024,
                     threads: int = 14, seq_len: int = 1400, batch_size: int = 8, seq_per_epoch: int = 16,
                     epochs: int = 1, precision: str = 'fp32', max_dota_time: float = 600.0,
                     rollout_size: int = 9999, warmup_iterations: int = 2, max_iterations: Optional[int] = None,
                     log_dir: Optional[str] = None, prefetch: int = 32, ring_bytes: int = 1 << 29,
                     transport: str = 'auto', backend: str = 'auto', idle_probe: float = 3.0,
                     report=None, record_consumed: int = 0, progress=None, pack: bool = False,
                     league: Optional[str] = None, latest_weights_prob: float = 1.0, actor_precision: str = 'bf16',
                     replay_gb: float = 0.0, actor_procs: int = 1, replay_prefill: bool = False,
                     old_logp: str = 'actor', advantages: str = 'vtrace-step') -> Dict[str, float]:
    """The reference's node topology end to end (optimizer.py:144-150, 274-287; ks-app/components/optimizer.jsonnet:
    79-174): ONE experience queue per node fed by actor processes, ``WORLD_SIZE`` learner ranks (one per GPU, DDP
    over RCCL) consuming disjoint rollouts from it as competing consumers, and rank 0 alone checkpointing and
    publishing the model every iteration, which every actor hot-swaps. Works at any world size (1 = one GPU).

    Rank 0 creates the node's broker — the shared-memory ring (``transport='shm'``, the default when every rank is
    on this node) or a TCP broker served from rank 0's process (``'tcp'``) — and broadcasts its address. Every rank
    spawns one actor process on its own device. Ranks agree every iteration on whether to go on, so all of them run
    the same DP steps. Before the timed window, ``idle_probe`` seconds of actor throughput are measured with the
    learners idle (CPU sharing vs. the persistent recurrence holding the CUs).

    Returns, on every rank, the node aggregate: ``steps_per_s`` (the reference's ``steps per s``, padded, summed
    over ranks), ``valid_steps_per_s``, ``actor_steps_per_s`` (sum), their per-rank lists, ``queue_dropped`` (ring
    drops during the window) and the per-rank stage times. ``report(opt) -> dict`` (tests) runs on every rank after
    the window; the results are returned in rank order under ``reports``.

    BASELINE config 5 (``league='pfsp'``, ``actor_precision='fp8'``, ``replay_gb`` > 0): the actors play a PFSP
    self-play league on the fp8 policy step and every learner trains from an on-HBM replay of ``replay_gb`` GB
    (learner/replay.py) instead of the iteration's fresh rollouts only.

    ``actor_procs`` > 1 splits each rank's ``games`` and ``threads`` over that many actor processes (each with its own
    interpreter, GIL and graphs on the rank's GPU): the actor loop's Python between its native parallel regions is
    serial per process."""
    import multiprocessing as mp
    import os
    import torch.distributed as tdist
    from ..parallel import dist as pdist
    from .optimizer import DotaOptimizer, OptimizerConfig
    say = progress or (lambda msg: logger.info(msg))

    world, rank = pdist.get_world_size(), pdist.get_rank()
    local_world = int(os.environ.get('LOCAL_WORLD_SIZE', world))
    # (the recurrence keeps its default 2 s hand-off deadline beside the actor process: the multi-second stalls of
    # round 5's config-5 loops came from the actor's HIGH-PRIORITY step streams — a league's opponent policies keep them
    # busy and the persistent team kernel lost its CUs for seconds; with default-priority actor streams the e2e,
    # config-5 and config-4 loops run clean at 2 s, profiles/r5_replay_timeout.md)
    if transport == 'auto':
        from .. import native
        transport = 'shm' if (local_world == world and native.AVAILABLE) else 'tcp'
    dev = torch.device(device)
    coll_dev = dev if (dev.type == 'cuda' and pdist.is_distributed() and tdist.get_backend() == 'nccl') else 'cpu'

    owner = None                    # rank 0's ShmBroker (creator) or TcpBrokerServer
    addr = None
    if rank == 0:
        if transport == 'shm':
            from ..transport.shm import ShmBroker, ring_capacity_for, shm_free_bytes
            name = f'dca_e2e_{os.getpid()}_{int(time.time() * 1e3) % 10 ** 9}'
            want = ring_bytes * world
            free = shm_free_bytes()
            # a small /dev/shm (container default 64 MB, or a node with little RAM): the ring takes at most half of
            # it and leaves the broker's headroom (one rule with ShmBroker's own check); too small fails here, clearly
            cap = ring_capacity_for(want, free)
            if cap < want:
                say(f'e2e: /dev/shm has {free >> 20} MiB free: experience ring clamped to {cap >> 20} MiB')
            owner = ShmBroker(name, capacity=cap, create=True, drop_oldest=True)
            addr = f'shm://{name}'
        else:
            from ..transport.broker import TcpBrokerServer
            host = os.environ.get('MASTER_ADDR', '127.0.0.1') if world > 1 else '127.0.0.1'
            owner = TcpBrokerServer(host, 0, maxsize=64 * world, drop_oldest=True).start()
            addr = f'tcp://{owner.host}:{owner.port}'
    if pdist.is_distributed():
        box = [addr]
        tdist.broadcast_object_list(box, 0)
        addr = box[0]
    broker = owner if (rank == 0 and transport == 'shm') else open_node_broker(addr, drop_oldest=True)

    tmp = log_dir or tempfile.mkdtemp(prefix='dca_e2e_')
    ctx = mp.get_context('spawn')
    stop, failed = ctx.Event(), ctx.Event()
    K = max(1, int(actor_procs))
    readies = [ctx.Event() for _ in range(K)]
    counters = [ctx.Value('q', 0) for _ in range(K)]

    class _Sum:                     # the actor processes' step counters as one (the probes read ``.value``)
        @property
        def value(self):
            return sum(c.value for c in counters)
    steps = _Sum()
    procs = []
    proc = opt = None
    rows, wall, actor_steps, idle, gpu_busy = [], 0.0, 0, float('nan'), float('nan')
    err = None

    def dropped_total():
        return int(owner.ring.dropped()) if transport == 'shm' and rank == 0 else \
            (int(owner.broker.n_dropped) if rank == 0 else 0)
    try:
        # the actor starts first (interpreter + engine + graph capture overlap the learner's construction) and
        # waits for rank 0's model version 0
        # DCA_E2E_ACTOR_HW_QUEUES: hardware queues of the actor process only (HIP's GPU_MAX_HW_QUEUES, read by the
        # spawned interpreter at its runtime init) — fewer queues beside the learner's persistent recurrence (A/B)
        hwq = os.environ.get('DCA_E2E_ACTOR_HW_QUEUES')
        saved_hwq = os.environ.get('GPU_MAX_HW_QUEUES')
        if hwq and 1 <= int(hwq) <= 32:
            os.environ['GPU_MAX_HW_QUEUES'] = str(int(hwq))
        try:
            feeder = os.environ.get('DCA_E2E_FEEDER') == '1'
            for k in range(K):
                g_k = games // K + (1 if k < games % K else 0)
                t_k = max(1, threads // K)
                if feeder:
                    proc = ctx.Process(target=_feeder_process_main, name=f'e2e-feeder-{rank}-{k}', daemon=True,
                                       args=(addr, model, seq_len, stop, readies[k], counters[k], failed,
                                             11 + 7919 * rank + 104729 * k))
                    proc.start()
                    procs.append(proc)
                    continue
                proc = ctx.Process(target=_actor_process_main, name=f'e2e-actor-{rank}-{k}', daemon=True,
                                   args=(addr, model, g_k, t_k, seq_len, rollout_size, max_dota_time, str(device),
                                         11 + 7919 * rank + 104729 * k, stop, readies[k], counters[k], failed,
                                         f'a{rank}' if K == 1 else f'a{rank}_{k}', league, latest_weights_prob,
                                         actor_precision))
                proc.start()
                procs.append(proc)
        finally:
            if hwq:
                if saved_hwq is None:
                    os.environ.pop('GPU_MAX_HW_QUEUES', None)
                else:
                    os.environ['GPU_MAX_HW_QUEUES'] = saved_hwq
        cfg = OptimizerConfig(log_dir=tmp, epochs=epochs, seq_per_epoch=seq_per_epoch, batch_size=batch_size,
                              seq_len=seq_len, model=model, precision=precision, device=str(device),
                              backend=backend, checkpoint_keep=2, run_local=True, xp_timeout=120.0,
                              histogram_freq=10 ** 9, async_checkpoint=dev.type == 'cuda',
                              prefetch_rollouts=prefetch, record_consumed=record_consumed, pack_sequences=pack,
                              replay_gb=replay_gb, replay_prefill=replay_prefill, old_logp=old_logp,
                              advantages=advantages)
        opt = DotaOptimizer(cfg, broker, checkpoint=rank == 0)     # rank 0 publishes model version 0
        say(f'e2e: learner ready ({transport} broker {addr}); waiting for the actor process')
        t_ready = time.time() + 900
        if not all(r.wait(timeout=max(1.0, t_ready - time.time())) for r in readies) or failed.is_set():
            raise RuntimeError('e2e actor process failed to start')
        if pdist.is_distributed():
            tdist.barrier()
        say('e2e: actor ready')

        def agree(cont: bool) -> bool:
            if not pdist.is_distributed():
                return cont
            t = torch.tensor([1 if cont else 0], dtype=torch.int32, device=coll_dev)
            tdist.all_reduce(t, op=tdist.ReduceOp.MIN)
            return bool(t.item())
        if idle_probe > 0:
            s0, t0 = steps.value, time.perf_counter()
            time.sleep(idle_probe)
            idle = (steps.value - s0) / (time.perf_counter() - t0)
            say(f'e2e: idle-learner actor probe {idle:.0f} player-steps/s')
            if dev.type == 'cuda':
                gpu_busy = _gpu_busy_probe(opt, steps, idle_probe, batch_size, seq_len, agree)
                say(f'e2e: busy-GPU actor probe {gpu_busy:.0f} player-steps/s')

        def check():
            for p in procs:
                if failed.is_set() or not p.is_alive():
                    return RuntimeError(f'e2e actor process died (exit code {p.exitcode})')
            return None

        d0 = dropped_total()
        say('e2e: learner loop')
        probe = None
        if os.environ.get('DCA_GIL_PROBE') == '1':
            from ..utils.gilprobe import GilProbe
            probe = GilProbe()
        try:
            s0 = opt.ingest_stats()
            rows, wall, (actor_steps, _) = _learner_loop(opt, duration, warmup_iterations, max_iterations,
                                                         counters=lambda: (steps.value, 0), check=check, agree=agree)
            s1 = opt.ingest_stats()
            ingest_diag = {k: s1[k] - s0[k] for k in s1}
            if probe is not None:
                import sys
                print(probe.report(), file=sys.stderr, flush=True)
        finally:
            opt.close()
            opt.flush_checkpoints()
        queue_dropped = dropped_total() - d0
        extra = report(opt) if report is not None else None
    except BaseException as e:
        err = e
        raise
    finally:
        stop.set()
        for p in procs:
            p.join(timeout=120)
            if p.is_alive():
                p.kill()
                p.join(timeout=10)
                if err is None:
                    err = RuntimeError('e2e actor process did not exit')
            elif p.exitcode != 0 and err is None:
                err = RuntimeError(f'e2e actor process exited with status {p.exitcode}')
        if broker is not owner and hasattr(broker, 'close'):
            broker.close()
        if pdist.is_distributed() and err is None:
            tdist.barrier()             # every rank's actor is done with the broker before rank 0 removes it
        if owner is not None:
            if transport == 'shm':
                owner.close(unlink=True)
            else:
                owner.stop()
        if log_dir is None:
            shutil.rmtree(tmp, ignore_errors=True)
    if err is not None:
        raise err
    mine = _summary(rows, wall, actor_steps, queue_dropped, games, dict(seq_per_epoch=seq_per_epoch, seq_len=seq_len))
    mine['actor_idle_steps_per_s'] = idle
    mine['ingest_decode'] = ingest_diag          # decode threads over the window (claims, waits, decode seconds)
    mine['actor_gpu_busy_steps_per_s'] = gpu_busy
    mine['learner_metrics'] = {k: a / max(n, 1) for k, (a, n) in getattr(_learner_loop, 'metrics', {}).items()}
    mine['report'] = extra
    per_rank = [mine]
    if pdist.is_distributed():
        per_rank = [None] * world
        tdist.all_gather_object(per_rank, mine)
    out = dict(per_rank[0])
    for k in ('steps_per_s', 'valid_steps_per_s', 'actor_steps_per_s', 'actor_idle_steps_per_s',
              'actor_gpu_busy_steps_per_s'):
        out[k] = float(sum(r[k] for r in per_rank))
        out[k + '_per_rank'] = [r[k] for r in per_rank]
    out['queue_dropped'] = int(per_rank[0]['queue_dropped'])
    # competing consumers on one queue: how evenly the node's rollouts reached the ranks (max / min per rank)
    cons = [int(r.get('rollouts_consumed', 0)) for r in per_rank]
    out['rollouts_consumed_per_rank'] = cons
    out['consumption_skew'] = (max(cons) / max(1, min(cons))) if cons else float('nan')
    out['learner_gpu_ms_per_step_per_rank'] = [r.get('learner_gpu_ms_per_step') for r in per_rank]
    reports = [r.pop('report') for r in per_rank]
    out.pop('report', None)
    if report is not None:
        out['reports'] = reports
    out['iterations'] = int(per_rank[0]['iterations'])
    out['games'] = games * world
    out['ranks'] = world
    out['config'] = dict(batch_size=batch_size, seq_len=seq_len, seq_per_epoch=seq_per_epoch, epochs=epochs,
                         rollout_size=rollout_size, max_dota_time=max_dota_time, precision=precision,
                         prefetch_rollouts=prefetch, games_per_rank=games, pack_sequences=pack,
                         actor=(f'one process per rank over the node {transport} broker' if K == 1 else
                                f'{K} processes per rank over the node {transport} broker'), learners=world,
                         league=league, latest_weights_prob=latest_weights_prob, actor_precision=actor_precision,
                         replay_gb=replay_gb,
                         # what was allocated (≤ replay_gb: the learner keeps the replay within the free HBM)
                         replay_gb_allocated=(opt.replay.nbytes / 1e9 if opt is not None and opt.replay is not None
                                              else 0.),
                         replay_sequences=(len(opt.replay) if opt is not None and opt.replay is not None else 0),
                         replay_capacity=(opt.replay.capacity if opt is not None and opt.replay is not None else 0),
                         replay_fill=(opt.replay.fill_fraction if opt is not None and opt.replay is not None else 0.),
                         replay_prefill=replay_prefill,
                         # PPO advantages (in-step V-trace / per-iteration policy_old forward / actor GAE — whatever
                         # they cost is inside every rate above) and the PPO ratio's denominator
                         advantages=advantages, old_logp=old_logp)
    return out


def _gpu_busy_probe(opt, steps, seconds: float, batch_size: int, seq_len: int, agree) -> float:
    """Actor player-steps/s while this rank's learner runs back-to-back training steps on synthetic on-device data
    and NO host work (no ingest, decode, publish): against the idle-learner rate and the full-loop rate it separates
    GPU contention (the persistent recurrence holds every CU for ≈1.7-2 ms per launch) from CPU sharing. The
    learner's weights and optimizer state are restored afterwards."""
    from .synthetic import DeviceReplay
    lrn = opt.learner
    if getattr(lrn, 'backend', None) != 'fused':
        return float('nan')
    cfg = opt.policy_cfg
    rep = DeviceReplay(2 * batch_size, seq_len, cfg.layout, cfg.hidden if cfg.rnn == 'lstm' else None, opt.device,
                       seed=5, vtrace=bool(getattr(lrn.cfg, 'vtrace', False)))
    saved = [t.clone() for t in (lrn.flat.flat, lrn.opt.exp_avg, lrn.opt.exp_avg_sq, lrn.opt.steps)]
    n_steps = lrn.n_steps
    lrn.train_step_replay(rep.buf, batch_size)
    torch.cuda.synchronize(opt.device)
    s0, t0 = steps.value, time.perf_counter()
    for _ in range(400):
        lrn.train_step_replay(rep.buf, batch_size)
        torch.cuda.synchronize(opt.device)
        if not agree(time.perf_counter() - t0 < seconds):  # DP ranks stop on the same step (same all-reduces)
            break
    rate = (steps.value - s0) / (time.perf_counter() - t0)
    for dst, src in zip((lrn.flat.flat, lrn.opt.exp_avg, lrn.opt.exp_avg_sq, lrn.opt.steps), saved):
        dst.copy_(src)
    lrn.n_steps = n_steps
    lrn.check_error()
    torch.cuda.synchronize(opt.device)
    return rate


def measure_e2e_procs(**kw) -> Dict[str, float]:
    """One-GPU form of :func:`measure_e2e_node` (the actor in a process of its own over the shm broker)."""
    return measure_e2e_node(**kw)
