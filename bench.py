#!/usr/bin/env python3
"""Headline benchmark: PPO optimizer samples/s (whole node), 1v1-mid LSTM-512 policy, synthetic data.

Metric (BASELINE.json): "PPO optimizer samples/sec (whole node) + actor steps/sec, 1v1-mid LSTM policy". A *sample*
is one timestep of one sequence consumed by an optimizer step — the reference's ``steps per s``
(optimizer.py:485-486: n_steps = sequences × seq_len). The baseline is the reference's published ~1000 steps/s
(README.md:35).

One timed *step* = one synchronous data-parallel PPO minibatch update on every rank: on-device minibatch gather from
the HBM replay pool → forward (entity encoder, LSTM over seq_len, heads) → PPO clipped-surrogate + value + entropy
loss → backward → RCCL all-reduce of the flat gradient → fused clip + Adam. Per-GPU work is fixed (weak scaling):
each rank trains on ``--batch-size`` sequences of ``--seq-len`` steps.

    python bench.py                                   # 1 GPU
    python bench.py --gpus 8                          # 8 rank processes started by bench.py itself
    python -m torch.distributed.run --nproc-per-node 8 ... bench.py --gpus 8

Rank 0 prints ONE JSON line. The actor and end-to-end numbers are measured *outside* the timed learner region, on
EVERY rank (one actor runtime per GPU), and reported as node aggregates (sums over ranks) with per-rank lists:

* ``actor.steps_per_s`` — player-steps/s of the whole self-play runtime (actor/vec.py), ``actor.policy_step_per_s``
  the batched GPU policy step alone (raw unit records staged and featurized on the GPU, the runtime's path;
  ``policy_step_host_features_per_s``: fed host features instead), copy → kernels → copy one step at a time;
  ``actor.policy_step_fp8_per_s`` the same step on the e4m3 MFMA kernel (BASELINE config 5, actor/batched.py
  Fp8ActorPolicy, 16-byte raw records) and ``actor.fp8_vs_bf16_policy_step`` their ratio;
* ``e2e`` — the reference's node topology run for real (learner/e2e.py ``measure_e2e_node``): one experience queue
  per node fed by one actor process per GPU, WORLD_SIZE learner ranks consuming disjoint rollouts (DDP over RCCL),
  rank 0 alone publishing the model. ``e2e.steps_per_s`` is the reference's own metric (optimizer.py:485-486, padded
  sequence steps incl. the wait for experience) summed over ranks; ``vs_baseline_e2e`` compares THAT with the
  reference's ≈1000 steps/s, the like-for-like node-level comparison (``vs_baseline`` is the compute-only learner);
* ``model_5v5_exact`` — the 5v5 policy at IEEE fp32 (BASELINE config 4 at the reference precision) on the fused
  kernels (the attention block's exact-fp32 twins); ``model_5v5`` is the same step with bf16x3 operands;
* ``learner_vtrace`` — the headline step with the in-step V-trace (the node loop's default advantages, learner
  /engine.py); the node loop's learner runs this step;
* ``bptt350_learner`` — truncated BPTT: each sequence trained as ``seq_len / 350`` chains of 350 steps from
  actor-stored (h, c) (32 sequences of 350 steps per step, at the headline's precision; not the headline);
* ``learner_b16`` / ``learner_b32`` — the same learner at 16 / 32 sequences per GPU per step (the exact recurrence
  packs 2 / 4 rows per XCD chain; the reference's ``--batch-size`` is free, optimizer.py:776; not the headline);
* ``league_replay`` — BASELINE config 5 through the same node loop: PFSP self-play league (80 % of games on the
  latest weights), the fp8 actor policy step, and learners sampling every minibatch from an on-HBM replay of
  ``--league-replay-gb`` GB per GPU (``config.replay_capacity`` sequences).
* ``e2e_5v5`` — BASELINE config 4 end to end: the same node loop on the 5v5 entity-attention model (5v5 self-play
  actors, 10 players per game; the learner at the headline precision — fp32-exact by default).

Knobs for rehearsing the multi-rank path on one GPU: ``DCA_DIST_BACKEND=gloo`` and ``DCA_SHARED_GPU=1`` (every rank
on cuda:0).
"""
from __future__ import annotations

import argparse
import hashlib
import json
import os
import sys
import time

import torch
import torch.distributed as dist

BASELINE_STEPS_PER_S = 1000.0   # reference README.md:35 (one optimizer)


def parse():
    ap = argparse.ArgumentParser()
    from dotaclient_amd.presets import add_preset_arg
    add_preset_arg(ap)
    ap.add_argument('--gpus', type=int, default=int(os.environ.get('WORLD_SIZE', 1)))
    ap.add_argument('--steps', type=int, default=20)
    ap.add_argument('--warmup', type=int, default=5)
    ap.add_argument('--batch-size', type=int, default=8, help='sequences per GPU per step (reference deploy: 8)')
    ap.add_argument('--seq-len', type=int, default=1400, help='steps per sequence (reference deploy: 1400)')
    ap.add_argument('--model', default='lstm512')
    ap.add_argument('--backend', default='auto', choices=['auto', 'fused', 'torch'])
    ap.add_argument('--algo', default='ppo', choices=['ppo', 'vpg'])
    ap.add_argument('--precision', default='fp32-exact', choices=['fp32-exact', 'fp32', 'bf16'],
                    help="fp32-exact = IEEE fp32 products everywhere, the reference's training precision (headline); "
                         'fp32 = fp32 activations with bf16x3-split MFMA operands (~2^-16 per product); bf16 = the '
                         'torch backend under bf16 autocast (no kernel path)')
    ap.add_argument('--vtrace-extra', type=int, default=1,
                    help='also time the headline step with the in-step V-trace (extra field learner_vtrace)')
    ap.add_argument('--bf16x3-extra', type=int, default=1,
                    help='also time the bf16x3-operand fp32 learner (extra field fp32_bf16x3_learner, not the headline)')
    ap.add_argument('--model-5v5-extra', type=int, default=1,
                    help='also time the 5v5 entity-attention policy (BASELINE config 4) at the same B, S with bf16x3 '
                         'operands (extra field model_5v5; model_5v5_exact is the fp32-exact number)')
    ap.add_argument('--model-5v5-exact-extra', type=int, default=1,
                    help='also time the 5v5 policy at fp32-exact on the fused kernels (extra field model_5v5_exact)')
    ap.add_argument('--bptt350-extra', type=int, default=1,
                    help='also time truncated BPTT: each sequence as seq_len/350 chains of 350 steps from stored '
                         '(h, c) (extra field bptt350_learner, headline precision; not the headline)')
    ap.add_argument('--big-batch-extra', type=int, default=1,
                    help='also time 16 and 32 sequences per GPU per step (extra fields learner_b16 / learner_b32)')
    ap.add_argument('--replay', type=int, default=0, help='sequences in the on-HBM replay pool (0 = 4x batch)')
    ap.add_argument('--graph', type=int, default=-1, help='capture the step in a hipGraph (-1 = auto)')
    ap.add_argument('--actor', type=int, default=1, help='also measure actor steps/s (untimed region)')
    ap.add_argument('--actor-games', type=int, default=2048, help='concurrent 1v1 games of the actor runtime')
    ap.add_argument('--actor-threads', type=int, default=0,
                    help='host threads of the native actor runtime per GPU (0 = from this rank\'s CPU share: '
                         'parallel/placement.py Placement.actor_threads, in [1, 14])')
    ap.add_argument('--pin', type=int, default=1,
                    help='pin this rank (learner threads + its actor process) to its GPU-local CPU share')
    ap.add_argument('--e2e', type=float, default=20.0,
                    help='seconds of the end-to-end actors→queue→learners loop on every rank (0 = off)')
    # node-loop actor shape (scripts/e2e_ab.py on one MI355X, 15 s each, after the round-4 host-loop fixes: 2048 games
    # × 14 threads 1.04 M steps/s (0.89 M valid), × 12 threads 0.91 M, 1024 × 12 0.84 M — same box, same minute; then
    # 4096 / 3072 / 2048 / 3072 games × 14: 1.11 / 1.08 / 0.94 / 1.00 M, weight age 5.0 / 4.4 / 3.3 / 4.0 versions —
    # bigger policy steps hold up better beside the learner's recurrence; 3072 trades a version of policy lag for it)
    ap.add_argument('--e2e-games', type=int, default=3072)
    ap.add_argument('--e2e-threads', type=int, default=0,
                    help='actor host threads of the node loop (0 = from the CPU share, in [1, 14])')
    ap.add_argument('--e2e-actor-precision', default='fp32', choices=['bf16', 'fp32', 'fp8'],
                    help='policy step of the node loop\'s actors: fp32 = the reference actor\'s precision (IEEE fp32 '
                         'products, F32ActorPolicy; the credited e2e number); bf16 / fp8 as extras (--e2e-extra)')
    ap.add_argument('--e2e-extra', type=float, default=10.0,
                    help='seconds of the same node loop with the bf16 actor policy step (extra field e2e_bf16; 0 = off)')
    ap.add_argument('--e2e-advantages', default='vtrace-step', choices=['vtrace-step', 'vtrace-iteration', 'gae'],
                    help="PPO advantages of the node loops' stale experience: V-trace inside every learner step from "
                         "the step's own values (default), the per-iteration policy_old forward (reference "
                         "optimizer.py:279, 474) + V-trace, or GAE from the actor's values")
    ap.add_argument('--e2e-old-logp', default='actor', choices=['learner', 'actor'],
                    help="the PPO ratio's denominator: the actor's behaviour log-prob, or the learner's policy_old "
                         "(needs --e2e-advantages vtrace-iteration)")
    ap.add_argument('--e2e-actor-procs', type=int, default=1,
                    help='actor processes per rank in the node loop (games and threads split over them)')
    ap.add_argument('--e2e-mode', default='process', choices=['process', 'thread'],
                    help='e2e actors as one spawned process per rank over the node broker (deploy split) or as a '
                         'thread (1 GPU only)')
    ap.add_argument('--e2e-probe', type=float, default=3.0,
                    help='seconds of each actor probe before the e2e window (learner idle / GPU-only learner)')
    ap.add_argument('--e2e-pack', type=int, default=1,
                    help='pack whole episodes into the learner sequences (episode-start resets in the recurrence) '
                         'instead of padding every rollout to seq_len (the reference layout: --e2e-pack 0)')
    ap.add_argument('--league-replay-extra', type=float, default=15.0,
                    help='seconds of the BASELINE config-5 node loop (extra field league_replay, 0 = off): PFSP '
                         'self-play league on the fp8 actor policy step, learners sampling an on-HBM replay of '
                         '--league-replay-gb GB per GPU')
    ap.add_argument('--league-replay-gb', type=float, default=100.0)
    ap.add_argument('--league-replay-prefill', type=int, default=1,
                    help='fill the replay ring to capacity from the first ingest (copies of the fresh sequences, '
                         'version -1) so every timed minibatch gathers from the whole pool; 0 = fills from the '
                         'actors only (league_replay.config.replay_fill reports the fraction either way)')
    ap.add_argument('--e2e-5v5-extra', type=float, default=-1.0,
                    help='seconds of the node loop on the 5v5 entity-attention model (extra field e2e_5v5, BASELINE '
                         'config 4 end to end: 5v5 self-play actors, 10 players per game; 0 = off; default: 15 s on '
                         'a one-GPU run, off on multi-GPU scaling runs)')
    ap.add_argument('--e2e-transport', default='auto', choices=['auto', 'shm', 'tcp'],
                    help='node experience queue: shared-memory ring (auto on one node) or a TCP broker on rank 0')
    from dotaclient_amd.presets import parse_with_preset
    return parse_with_preset(ap, 'bench')


def progress(msg: str):
    """Phase markers on stderr (one line each, flushed) so a long multi-rank run shows where it is."""
    print(f'[bench r{os.environ.get("RANK", "0")} {time.strftime("%H:%M:%S")}] {msg}', file=sys.stderr, flush=True)


def _free_port() -> int:
    import socket
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    port = s.getsockname()[1]
    s.close()
    return port


def launch_ranks(n: int) -> int:
    """``python bench.py --gpus N`` without a launcher: start N fresh rank processes of this script (one per GPU,
    env:// rendezvous on 127.0.0.1), forward rank 0's stdout (the JSON line) and every rank's stderr, and return the
    first non-zero exit status (the other ranks are then stopped by PID). The caller has touched no GPU: the parent
    only parses arguments, and a HIP-initialised parent must never exec or fork a GPU program."""
    import signal
    import subprocess
    port = os.environ.get('MASTER_PORT') or str(_free_port())
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK='0', NODE_RANK='0', MASTER_ADDR=os.environ.get('MASTER_ADDR', '127.0.0.1'),
                   MASTER_PORT=port, DCA_BENCH_LAUNCHED='1')
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env,
                                      stdout=None if r == 0 else sys.stderr.fileno()))
    progress(f'launched {n} ranks: pids {[p.pid for p in procs]} (master 127.0.0.1:{port})')
    status = 0
    live = list(procs)
    kill_at = None
    while live:
        if kill_at is not None and time.time() > kill_at:
            for q in live:
                q.kill()
            kill_at = float('inf')
        for p in list(live):
            rc = p.poll()
            if rc is None:
                continue
            live.remove(p)
            if rc != 0 and status == 0:
                status = rc if rc > 0 else 128 - rc
                progress(f'rank pid {p.pid} exited with {rc}: stopping the other ranks')
                for q in live:
                    q.send_signal(signal.SIGTERM)
                kill_at = time.time() + 30.0
        time.sleep(0.2)
    return status


def main():
    args = parse()
    env_world = os.environ.get('WORLD_SIZE')
    if env_world is None and args.gpus > 1:
        # self-launch BEFORE anything touches the GPU (no torch.cuda call has been made in this process)
        sys.exit(launch_ranks(args.gpus))
    if env_world is not None and int(env_world) != args.gpus:
        print(f'bench.py: --gpus {args.gpus} but WORLD_SIZE={env_world} (launcher and flag disagree)', file=sys.stderr)
        sys.exit(2)
    world = int(os.environ.get('WORLD_SIZE', '1'))
    rank = int(os.environ.get('RANK', '0'))
    local = int(os.environ.get('LOCAL_RANK', '0'))
    use_cuda = torch.cuda.is_available()
    shared = os.environ.get('DCA_SHARED_GPU') == '1'          # rehearsal: every rank on GPU 0
    # the recurrence's hand-off deadline stays at its default 2 s (DCA_TEAM_PATIENT unset): round 5's multi-second
    # device stalls had a cause in this code — the league's high-priority actor streams preempting the persistent
    # recurrence, fixed (profiles/r5_replay_timeout.md) — so a stall now fails the section loudly instead of deflating
    # its number; every node-loop section reports its slowest in-loop learner step (learner_gpu_ms_per_step_max)
    if shared:
        # (rehearsal only: every rank's processes time-slice one device, so a rank's recurrence can be switched out
        # for longer than the 2 s hand-off deadline — measured: a two-rank shared run failing with a backward hand-off
        # timeout — the 60 s deadline applies; the driver's one-rank-per-GPU runs keep 2 s)
        os.environ.setdefault('DCA_TEAM_PATIENT', '1')
    device = torch.device(f'cuda:{0 if shared else local}' if use_cuda else 'cpu')
    if use_cuda:
        torch.cuda.set_device(device)
    # host placement before any worker thread / actor process starts (they inherit the mask)
    from dotaclient_amd.parallel.placement import for_this_rank
    place = for_this_rank(pin=bool(args.pin))
    if not args.actor_threads:
        args.actor_threads = place.actor_threads()
    if not args.e2e_threads:
        args.e2e_threads = place.actor_threads()
    host = dict(place.describe(), actor_threads=args.actor_threads, e2e_threads=args.e2e_threads)
    if world > 1:
        from dotaclient_amd.parallel.dist import init_distribution
        init_distribution(backend=os.environ.get('DCA_DIST_BACKEND') or None, device=device)

    from dotaclient_amd.learner.engine import Learner, LossConfig
    from dotaclient_amd.learner.synthetic import DeviceReplay
    from dotaclient_amd.models.policy import Policy, get_config

    cfg = get_config(args.model)
    trace = os.environ.get('DCA_BENCH_TRACE') == '1'

    def run(precision, cfg=cfg, B=None, S=None, backend=None, steps=None, warmup=None, vtrace=False):
        """Build a learner of this precision and time ``args.steps`` DP PPO steps (``B`` sequences of ``S`` steps,
        default the command line's) after ``args.warmup``; returns (elapsed s (max over ranks), loss_first,
        loss_last, learner, policy)."""
        B = B or args.batch_size
        S = S or args.seq_len
        n_steps = steps or args.steps
        n_warm = args.warmup if warmup is None else warmup
        torch.manual_seed(7 + rank)
        policy = Policy(cfg)
        backend = backend or args.backend
        if backend == 'auto':
            backend = 'fused' if use_cuda else 'torch'
        lc = LossConfig(algo=args.algo, vtrace=True) if vtrace else LossConfig(algo=args.algo)
        learner = Learner(policy, lc, device=device, backend=backend, precision=precision)
        learner.dp.timing = world > 1       # per-step all-reduce timing events (DataParallel.comm_stats)
        if args.graph == 1 or (args.graph == -1 and learner.backend == 'fused'):
            learner.enable_graph(warmup=1)
        n_pool = args.replay or 4 * B
        replay = DeviceReplay(n_pool, S, cfg.layout, cfg.hidden if cfg.rnn == 'lstm' else None, device,
                              seed=1000 * rank, vtrace=vtrace)

        def step():
            t = time.perf_counter()
            # on-device minibatch gather from the HBM replay pool (part of the captured step on the fused path)
            out = learner.train_step_replay(replay.buf, B)
            if trace:
                torch.cuda.synchronize()
                print(f'[bench] {precision} step {learner.n_steps} {1e3 * (time.perf_counter() - t):.2f} ms loss '
                      f'{float(out["loss"]):.5f} gnorm {float(out["grad_norm"]):.5f} '
                      f'params_finite {bool(torch.isfinite(learner.flat.flat).all())} '
                      f'grad_finite {bool(torch.isfinite(learner.flat.grad).all())} '
                      f'err {int(learner.model.err.item()) if learner.backend == "fused" else 0}',
                      file=sys.stderr, flush=True)
            return out

        m = None
        for _ in range(n_warm):
            m = step()
        if use_cuda:
            torch.cuda.synchronize()
        loss_first = float(m['loss']) if m is not None else float('nan')
        if world > 1:
            dist.barrier()
        if use_cuda:
            torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(n_steps):
            m = step()
        if use_cuda:
            torch.cuda.synchronize()
        if world > 1:
            dist.barrier()
        elapsed = time.perf_counter() - t0
        if world > 1:
            t = torch.tensor([elapsed], device=device, dtype=torch.float64)
            dist.all_reduce(t, op=dist.ReduceOp.MAX)
            elapsed = float(t.item())
        loss_last = float(m['loss'])
        learner.check_error()       # a persistent-kernel timeout would invalidate the measurement
        return elapsed, loss_first, loss_last, learner, policy

    progress(f'learner {args.precision}: world {world}, device {device}')
    elapsed, loss_val, final_loss, learner, policy = run(args.precision)
    progress(f'learner {args.precision} done: {elapsed / args.steps * 1e3:.3f} ms/step')
    backend = learner.backend
    # per-rank all-reduce wall time, the share of the early buckets' all-reduce hidden behind the step's second
    # compute phase, the exposed comm time, the bucket layout (the first 8-GPU driver run must be diagnosable)
    comm = learner.dp.comm_stats() if world > 1 else None
    if comm is not None:
        comm['dist_backend'] = dist.get_backend()
        comm['rank'] = rank
    step_mode = {'hipgraph': learner.graph is not None, 'dp_split_overlap': bool(getattr(learner, '_split', False)),
                 'dist_backend': dist.get_backend() if world > 1 else None}
    # DP replicas must hold bit-identical weights after the timed steps (checked across ranks below)
    weights_sha = hashlib.sha256(learner.flat.flat.detach().cpu().numpy().tobytes()).hexdigest()[:16]
    samples = args.batch_size * args.seq_len * world * args.steps
    value = samples / elapsed
    ms_per_step = elapsed / args.steps * 1e3
    vtr = None
    if args.vtrace_extra and args.algo == 'ppo' and use_cuda:
        # the same step with the in-step V-trace (the node loop's default advantages: every minibatch's advantages and
        # value targets recomputed from the step's own values / log-probs against the behaviour log-prob)
        learner = None
        try:
            ev, lv0, lv1, _, _ = run(args.precision, vtrace=True)
            progress(f'learner {args.precision} + in-step V-trace done: {ev / args.steps * 1e3:.3f} ms/step')
            vtr = {'precision': args.precision, 'advantages': 'vtrace-step', 'value': samples / ev,
                   'ms_per_step': ev / args.steps * 1e3, 'loss_first': lv0, 'loss_last': lv1}
        except Exception as e:
            vtr = {'error': repr(e)}
    bf16x3 = None
    if args.bf16x3_extra and args.precision == 'fp32-exact' and use_cuda:
        learner = None
        try:
            e3, l30, l31, _, _ = run('fp32')
            progress(f'learner fp32 (bf16x3 operands) done: {e3 / args.steps * 1e3:.3f} ms/step')
            bf16x3 = {'precision': 'fp32 activations / bf16x3-split MFMA operands (~2^-16 relative per product)',
                      'value': samples / e3, 'ms_per_step': e3 / args.steps * 1e3, 'loss_first': l30,
                      'loss_last': l31}
        except Exception as e:
            bf16x3 = {'error': repr(e)}

    model_5v5 = None
    if args.model_5v5_extra and use_cuda and not cfg.entity_attention:
        # BASELINE config 4: the 5v5 policy (64 unit slots, pre-LN entity self-attention) through the same fused
        # learner step, same B, S, precision and DP layout
        learner = None
        p5 = 'fp32' if args.precision == 'fp32-exact' else args.precision
        try:
            e5, l50, l51, _, _ = run(p5, get_config('5v5'))
            progress(f'learner 5v5 done: {e5 / args.steps * 1e3:.3f} ms/step')
            model_5v5 = {'model': '5v5', 'precision': p5 + (' (bf16x3 operands)' if p5 == 'fp32' else ''),
                         'value': samples / e5,
                         'ms_per_step': e5 / args.steps * 1e3, 'loss_first': l50, 'loss_last': l51}
        except Exception as e:
            model_5v5 = {'error': repr(e)}

    model_5v5_exact = None
    if args.model_5v5_exact_extra and use_cuda and not cfg.entity_attention:
        # the 5v5 policy at the reference's precision on the fused kernels: the IEEE-fp32 twins of the attention block
        # (ops/csrc/attn_block.hip EX), the exact encoder / recurrence / heads kernels, exact split-K ∂W GEMMs
        learner = None
        try:
            e5x, l0, l1, _, _ = run('fp32-exact', get_config('5v5'))
            progress(f'learner 5v5 fp32-exact done: {e5x / args.steps * 1e3:.3f} ms/step')
            model_5v5_exact = {'model': '5v5', 'precision': 'fp32-exact (IEEE fp32 products, hand-written kernels)',
                               'value': samples / e5x, 'ms_per_step': e5x / args.steps * 1e3, 'loss_first': l0,
                               'loss_last': l1}
        except Exception as e:
            model_5v5_exact = {'error': repr(e)}

    bptt = None
    if (args.bptt350_extra and use_cuda and cfg.rnn == 'lstm' and not cfg.entity_attention
            and args.seq_len % 350 == 0 and args.seq_len > 350):
        # truncated BPTT (SURVEY §5 long-context row): every seq_len-step sequence trained as seq_len/350
        # independent 350-step chains that start from the (h, c) the actor stored every 350 steps (replay h0 / c0),
        # 4x fewer serial recurrence steps; 32 chains per step run as 8 XCD chains of 4 rows (exact VALU recurrence)
        learner = None
        k = args.seq_len // 350
        try:
            eb, lb0, lb1, _, _ = run(args.precision, B=args.batch_size * k, S=350)
            progress(f'learner bptt350 done: {eb / args.steps * 1e3:.3f} ms/step')
            bptt = {'precision': args.precision, 'chains_per_sequence': k,
                    'batch': args.batch_size * k, 'seq_len': 350, 'value': samples / eb,
                    'ms_per_step': eb / args.steps * 1e3, 'loss_first': lb0, 'loss_last': lb1}
        except Exception as e:
            bptt = {'error': repr(e)}

    big = {}
    if args.big_batch_extra and use_cuda and cfg.rnn == 'lstm' and not cfg.entity_attention:
        # the same learner at 16 / 32 sequences per GPU (2 / 4 rows per XCD chain of the exact recurrence): the
        # recurrence is latency-bound, so samples per step grow faster than its time
        learner = None
        for bb in (16, 32):
            try:
                ebb, l0, l1, _, _ = run(args.precision, B=bb)
                progress(f'learner B={bb} done: {ebb / args.steps * 1e3:.3f} ms/step')
                big[f'learner_b{bb}'] = {'precision': args.precision, 'batch': bb, 'seq_len': args.seq_len,
                                         'value': bb * args.seq_len * world * args.steps / ebb,
                                         'ms_per_step': ebb / args.steps * 1e3, 'loss_first': l0, 'loss_last': l1}
            except Exception as e:
                big[f'learner_b{bb}'] = {'error': repr(e)}

    def gather(x):
        """Every rank's value of ``x`` on every rank (rank order)."""
        if world == 1:
            return [x]
        out = [None] * world
        dist.all_gather_object(out, x)
        return out

    actor = None
    if args.actor and use_cuda:
        # one actor runtime per GPU, all ranks at once (node aggregate = sum): actor.steps_per_s is the whole
        # self-play runtime (actor/vec.py: native engine + featurize + reward + trajectory/rollout encoding on host
        # threads, one hipGraph policy step for every player) in player-steps/s; actor.policy_step_per_s is the
        # batched GPU policy step alone (observations pre-staged)
        mine = {}
        if world > 1:
            dist.barrier()
        try:
            from dotaclient_amd.actor.vec import measure_vec_actor
            rt = measure_vec_actor(policy, device, n_games=args.actor_games, threads=args.actor_threads)
            mine.update(steps_per_s=rt['steps_per_s'], runtime=rt)
        except Exception as e:  # the learner metric stands on its own
            mine['runtime_error'] = repr(e)
        if not cfg.entity_attention:
            if world > 1:
                dist.barrier()
            try:
                # the same runtime with the IEEE-fp32 policy step (the reference actor's precision: log-probs within
                # 1e-5 of the torch fp32 policy, PPO ratio 1 ± 1e-7 at weight age 0)
                rt = measure_vec_actor(policy, device, n_games=args.actor_games, threads=args.actor_threads,
                                       precision='fp32')
                mine.update(steps_per_s_fp32=rt['steps_per_s'])
            except Exception as e:
                mine['runtime_fp32_error'] = repr(e)
        if world > 1:
            dist.barrier()
        try:
            # the same runtime on the reference actor's wire path: every observation a serialised CMsgBotWorldState
            # decoded + featurized natively, every team's orders an Actions protobuf (agent.py:564-637, 805-825)
            rt = measure_vec_actor(policy, device, n_games=args.actor_games, threads=args.actor_threads, wire=True)
            mine.update(protobuf_runtime_steps_per_s=rt['steps_per_s'], protobuf_runtime=rt)
        except Exception as e:
            mine['protobuf_runtime_error'] = repr(e)
        if world > 1:
            dist.barrier()
        try:
            from dotaclient_amd.actor.batched import measure_actor_throughput
            mb = measure_actor_throughput(policy, device, n_games=args.actor_games, threads=args.actor_threads)
            mine['policy_step_per_s'] = mb['gpu_steps_per_s']
            mine['policy_step_protobuf_featurize_per_s'] = mb['steps_per_s']
            # the same step fed host features (40 B fp32 + an 8 B handle per unit slot) instead of raw unit records
            # (32 B) featurized on the GPU (ops/csrc/featurize.hip) — the pre-round-6 staging
            mh = measure_actor_throughput(policy, device, n_games=args.actor_games, threads=args.actor_threads,
                                          raw=False)
            mine['policy_step_host_features_per_s'] = mh['gpu_steps_per_s']
            mine['policy_step_host_features_protobuf_featurize_per_s'] = mh['steps_per_s']
        except Exception as e:
            mine['policy_step_error'] = repr(e)
        try:
            # BASELINE config 5: the same step with the pre-RNN layer, LSTM step and heads on the hand-written e4m3
            # MFMA kernel (ops/csrc/actor_fp8.hip; per-channel weight / per-row activation scales) and fp16 / int32
            # observation staging
            mb = measure_actor_throughput(policy, device, n_games=args.actor_games, threads=args.actor_threads,
                                          precision='fp8')
            mine['policy_step_fp8_per_s'] = mb['gpu_steps_per_s']
            mine['policy_step_fp8_protobuf_featurize_per_s'] = mb['steps_per_s']
            if mine.get('policy_step_per_s'):
                mine['fp8_vs_bf16_policy_step'] = mb['gpu_steps_per_s'] / mine['policy_step_per_s']
        except Exception as e:
            mine['policy_step_fp8_error'] = repr(e)
        if not cfg.entity_attention:
            try:
                # the reference actor's precision: the IEEE-fp32 policy step (ops/csrc/actor_core.hip MODE 0,
                # v_mfma_f32_16x16x4_f32, no vendor GEMM)
                mb = measure_actor_throughput(policy, device, n_games=args.actor_games, threads=args.actor_threads,
                                              precision='fp32')
                mine['policy_step_fp32_per_s'] = mb['gpu_steps_per_s']
                mine['policy_step_fp32_protobuf_featurize_per_s'] = mb['steps_per_s']
            except Exception as e:
                mine['policy_step_fp32_error'] = repr(e)
        ranks = gather(mine)
        progress('actor measurements done')
        actor = dict(ranks[0])
        for k in ('steps_per_s', 'steps_per_s_fp32', 'protobuf_runtime_steps_per_s', 'policy_step_per_s',
                  'policy_step_host_features_per_s', 'policy_step_host_features_protobuf_featurize_per_s',
                  'policy_step_protobuf_featurize_per_s', 'policy_step_fp8_per_s',
                  'policy_step_fp8_protobuf_featurize_per_s', 'policy_step_fp32_per_s',
                  'policy_step_fp32_protobuf_featurize_per_s'):
            vals = [r.get(k) for r in ranks]
            if all(v is not None for v in vals):
                actor[k] = float(sum(vals))
                actor[k + '_per_rank'] = vals
        actor['ranks'] = world

    e2e = None
    if args.e2e > 0 and use_cuda and (args.e2e_mode == 'process' or world == 1):
        # the reference's own metric ('steps per s' incl. the wait for experience, optimizer.py:485-486) from the
        # real node loop: actor process per GPU → ONE node queue → WORLD_SIZE DotaOptimizer ranks (deploy shape
        # 8×1400, 16 seq/iteration, DDP) → rank 0 publishes the model → actors
        learner = None
        try:
            from dotaclient_amd.learner.e2e import measure_e2e, measure_e2e_node
            kw = dict(model=args.model, device=device, duration=args.e2e, games=args.e2e_games,
                      threads=args.e2e_threads, seq_len=args.seq_len, precision=args.precision,
                      pack=bool(args.e2e_pack), old_logp=args.e2e_old_logp, advantages=args.e2e_advantages)
            progress('e2e start')
            if args.e2e_mode == 'process':
                e2e = measure_e2e_node(transport=args.e2e_transport, progress=progress, idle_probe=args.e2e_probe,
                                       actor_procs=args.e2e_actor_procs, actor_precision=args.e2e_actor_precision,
                                       **kw)
            else:
                e2e = measure_e2e(**kw)
        except Exception as e:
            e2e = {'error': repr(e)}
        progress(f'e2e done: {e2e.get("error", "ok")}')
        errs = gather('error' in e2e)
        if any(errs) and 'error' not in e2e:
            e2e = {'error': f'failed on rank(s) {[i for i, x in enumerate(errs) if x]}'}

    e2e_bf16 = None
    if (args.e2e > 0 and args.e2e_extra > 0 and use_cuda and args.e2e_mode == 'process'
            and args.e2e_actor_precision != 'bf16'):
        # the same node loop with the bf16 actor policy step (extra; the credited e2e runs the reference precision)
        try:
            from dotaclient_amd.learner.e2e import measure_e2e_node
            progress('e2e-bf16 start')
            e2e_bf16 = measure_e2e_node(
                model=args.model, device=device, duration=args.e2e_extra, games=args.e2e_games,
                threads=args.e2e_threads, seq_len=args.seq_len, precision=args.precision, pack=bool(args.e2e_pack),
                transport=args.e2e_transport, progress=progress, idle_probe=0.0, actor_precision='bf16',
                old_logp=args.e2e_old_logp, advantages=args.e2e_advantages)
        except Exception as e:
            e2e_bf16 = {'error': repr(e)}
        progress(f'e2e-bf16 done: {e2e_bf16.get("error", "ok")}')
        errs = gather('error' in e2e_bf16)
        if any(errs) and 'error' not in e2e_bf16:
            e2e_bf16 = {'error': f'failed on rank(s) {[i for i, x in enumerate(errs) if x]}'}

    league_replay = None
    if args.league_replay_extra > 0 and use_cuda and args.e2e_mode == 'process' and cfg.rnn == 'lstm':
        # BASELINE config 5 (presets.py league-replay): the same node loop with a PFSP league of past versions
        # (80 % of games on the latest weights), the fp8 actor policy step (actor/batched.py Fp8ActorPolicy) and an
        # on-HBM replay of --league-replay-gb GB per learner (learner/replay.py) that every minibatch is sampled from
        try:
            from dotaclient_amd.learner.e2e import measure_e2e_node
            progress('league-replay start')
            league_replay = measure_e2e_node(
                model=args.model, device=device, duration=args.league_replay_extra, games=args.e2e_games,
                threads=args.e2e_threads, seq_len=args.seq_len, precision=args.precision, pack=bool(args.e2e_pack),
                transport=args.e2e_transport, progress=progress, idle_probe=0.0, league='pfsp',
                latest_weights_prob=0.8, actor_precision='fp8', replay_gb=args.league_replay_gb,
                replay_prefill=bool(args.league_replay_prefill), old_logp=args.e2e_old_logp, advantages=args.e2e_advantages)
        except Exception as e:
            league_replay = {'error': repr(e)}
        progress(f'league-replay done: {league_replay.get("error", "ok")}')
        errs = gather('error' in league_replay)
        if any(errs) and 'error' not in league_replay:
            league_replay = {'error': f'failed on rank(s) {[i for i, x in enumerate(errs) if x]}'}

    e2e_5v5 = None
    if args.e2e_5v5_extra < 0:
        args.e2e_5v5_extra = 15.0 if world == 1 else 0.0
    if args.e2e_5v5_extra > 0 and use_cuda and args.e2e_mode == 'process' and args.model != '5v5':
        # BASELINE config 4 end to end: the same node loop on the 5v5 model (entity attention, the learner at the
        # headline precision), 5v5 self-play games on the VecActor (e2e_games / 5 games, 10 player slots each)
        try:
            from dotaclient_amd.learner.e2e import measure_e2e_node
            progress('e2e-5v5 start')
            e2e_5v5 = measure_e2e_node(
                model='5v5', device=device, duration=args.e2e_5v5_extra, games=max(1, args.e2e_games // 5),
                threads=args.e2e_threads, seq_len=args.seq_len, precision=args.precision, pack=bool(args.e2e_pack),
                transport=args.e2e_transport, progress=progress, idle_probe=0.0,
                actor_precision=args.e2e_actor_precision, old_logp=args.e2e_old_logp, advantages=args.e2e_advantages)
        except Exception as e:
            e2e_5v5 = {'error': repr(e)}
        progress(f'e2e-5v5 done: {e2e_5v5.get("error", "ok")}')
        errs = gather('error' in e2e_5v5)
        if any(errs) and 'error' not in e2e_5v5:
            e2e_5v5 = {'error': f'failed on rank(s) {[i for i, x in enumerate(errs) if x]}'}

    shas = gather(weights_sha)
    hosts = gather(host)
    comms = gather(comm)
    if rank == 0:
        out = {
            'metric': 'PPO optimizer samples/sec (whole node) + actor steps/sec, 1v1-mid LSTM policy',
            'value': value,
            'unit': 'samples/s',
            'n_gpus': world,
            'steps': args.steps,
            'warmup': args.warmup,
            'ms_per_step': ms_per_step,
            'higher_is_better': True,
            'scaling': 'weak',
            'vs_baseline': value / BASELINE_STEPS_PER_S,
            'vs_baseline_e2e': (e2e['steps_per_s'] / BASELINE_STEPS_PER_S
                                if e2e and 'steps_per_s' in e2e else None),
            'e2e_layout': ('packed: whole episodes packed into the seq_len sequences with episode-start resets '
                           '(--e2e-pack 1; steps_per_s counts padded steps, valid_steps_per_s real ones)'
                           if args.e2e_pack else 'reference layout: every rollout padded to seq_len (--e2e-pack 0)'),
            'dtype': {'fp32-exact': 'fp32', 'fp32': 'fp32 (bf16x3 MFMA operands)'}.get(args.precision, args.precision),
            'precision_note': {
                'fp32-exact': 'IEEE fp32 end to end like the reference (torch fp32 nn.Linear + Adam): every GEMM product '
                              'an fp32 fma on v_mfma_f32_16x16x4_f32 or fp32 VALU in hand-written kernels, fp32 '
                              'activations, gradients, accumulation and optimizer; no vendor GEMM',
                'fp32': 'fp32 activations / gradients / optimizer, GEMM operands bf16x3-split (~2^-16 relative per '
                        'product)',
            }.get(args.precision, 'bf16 GEMM operands and saved activations, fp32 accumulation / recurrence / '
                                  'optimizer'),
            'data': 'synthetic (on-HBM replay of synthetic 1v1-mid experience, random-init weights)',
            'config': {'model': f'{args.model} ({cfg.rnn}-{cfg.hidden}, '
                                f'{"5v5 entity-attention" if cfg.entity_attention else "1v1-mid entity"} encoder, '
                                f'{cfg.layout.max_units} units)',
                       'global_batch': args.batch_size * world, 'seq_len': args.seq_len,
                       'parallelism': f'dp{world}', 'algo': args.algo, 'backend': backend, 'step': step_mode},
            'loss_first': loss_val, 'loss_last': final_loss,
            'fp32_bf16x3_learner': bf16x3,
            'model_5v5': model_5v5,
            'model_5v5_exact': model_5v5_exact,
            'bptt350_learner': bptt,
            'learner_vtrace': vtr,
            'learner_b16': big.get('learner_b16'),
            'learner_b32': big.get('learner_b32'),
            'dp_replicas_identical': len(set(shas)) == 1,
            'dp_comm': ({'dist_backend': step_mode['dist_backend'], 'per_rank': comms,
                         'allreduce_ms_max': max((c or {}).get('allreduce_ms', 0.0) for c in comms),
                         'exposed_ms_max': max((c or {}).get('exposed_ms', 0.0) for c in comms)}
                        if world > 1 else None),
            'weights_sha16_per_rank': shas,
            'actor': actor,
            'e2e': e2e,
            'e2e_bf16': e2e_bf16,
            'league_replay': league_replay,
            'e2e_5v5': e2e_5v5,
            'host_placement': hosts,
        }
        print(json.dumps(out), flush=True)
    if world > 1:
        dist.barrier()
        dist.destroy_process_group()


if __name__ == '__main__':
    main()
