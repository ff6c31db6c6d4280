"""Actor entrypoint (reference ``agent.py`` CLI, agent.py:952-973).

Reference-compatible flags: ``--ip --port --rollout-size --max-dota-time -l/--log --model --use-latest-weights-prob
--validation --log-dir``. Additional: ``--broker`` (inproc | tcp://host:port | shm://name; default tcp://ip:port),
``--env`` (synthetic | grpc://host:port, reference: the dotaservice sidecar on 127.0.0.1:13337), ``--games`` (games
driven in lockstep with one batched policy step), ``--device``, ``--model-preset``, ``--wire`` (dcx1 | pickle).

    python -m dotaclient_amd.cli.agent --ip 127.0.0.1 --port 5672 --env synthetic --games 64 --device cuda
"""
from __future__ import annotations

import argparse
import logging
import random
import sys
import time

import torch

logger = logging.getLogger('dotaclient_amd.agent')


def str2bool(v):
    return str(v).lower() in ('1', 'true', 'yes', 'y', 't')


def build_parser():
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    from ..presets import add_preset_arg
    add_preset_arg(ap)
    ap.add_argument('--ip', type=str, default='127.0.0.1', help='broker ip')
    ap.add_argument('--port', type=int, default=5672, help='broker port')
    ap.add_argument('--broker', type=str, default=None, help='broker url (overrides --ip/--port)')
    ap.add_argument('--rollout-size', type=int, default=int(1e6), help='size of each rollout (steps)')
    ap.add_argument('--max-dota-time', type=int, default=600, help='maximum in-game time before restarting')
    ap.add_argument('-l', '--log', dest='log_level', default='INFO',
                    choices=['DEBUG', 'INFO', 'WARNING', 'ERROR', 'CRITICAL'])
    ap.add_argument('--model', type=str, default=None,
                    help='initial model: a state_dict file or a store URL (<url>#<key>, gs://bucket/path.pt)')
    ap.add_argument('--artifact-url', type=str, default=None,
                    help='validation: mirror the tensorboard events file here (reference: GCS)')
    ap.add_argument('--use-latest-weights-prob', type=float, default=1.0)
    # reference: type=bool (any non-empty string is True, quirk §2.9); we parse booleans properly
    ap.add_argument('--validation', type=str2bool, default=False)
    ap.add_argument('--log-dir', type=str, default='')
    ap.add_argument('--env', type=str, default='synthetic', help='synthetic | grpc://host:port')
    ap.add_argument('--games', type=int, default=1, help='games driven concurrently (batched policy step)')
    ap.add_argument('--n-games', type=int, default=10_000_000, help='total games to play (reference N_GAMES)')
    ap.add_argument('--device', type=str, default='cpu')
    ap.add_argument('--model-preset', type=str, default='lstm512')
    ap.add_argument('--wire', type=str, default='dcx1', choices=['dcx1', 'pickle'])
    ap.add_argument('--seed', type=int, default=None)
    ap.add_argument('--hidden-stride', type=int, default=256, help='store LSTM state every N steps')
    ap.add_argument('--runtime', type=str, default='auto', choices=['auto', 'vec', 'service'],
                    help='vec: native vectorised self-play (actor/vec.py, synthetic env only); service: the '
                         'protobuf Actor over DotaService games; auto: vec for synthetic self-play')
    ap.add_argument('--threads', type=int, default=8, help='host threads of the vec runtime')
    ap.add_argument('--actor-precision', type=str, default='bf16', choices=['bf16', 'fp32', 'fp8'],
                    help='vec runtime policy step: bf16, fp32 (IEEE fp32, the reference actor\'s precision; 1v1) or '
                         'fp8 (e4m3 MFMA kernel; 1v1 LSTM-512 policies)')
    ap.add_argument('--league', type=str, default='oldest', choices=['oldest', 'uniform', 'recent', 'pfsp'],
                    help='opponent sampling over the weight history when not playing the latest weights')
    return ap


def make_services(env: str, n: int, seed: int):
    if env == 'synthetic':
        from ..env import SyntheticDotaService
        return [SyntheticDotaService(seed=seed + i) for i in range(n)]
    if env.startswith('grpc://'):
        from ..env.service import DotaServiceClient
        host, port = env[7:].rsplit(':', 1)
        return [DotaServiceClient(host, int(port)) for _ in range(n)]
    raise ValueError(env)


def main(argv=None):
    from ..presets import parse_with_preset
    args = parse_with_preset(build_parser(), 'agent', argv)
    logging.basicConfig(format='%(asctime)s %(levelname)-8s %(message)s', level=args.log_level)
    from ..actor.game import Actor
    from ..actor.gpu_runner import GpuRunner, gpu_runner_supported
    from ..actor.runner import PolicyRunner, RunnerCache
    from ..actor.weights import WeightStore
    from ..env import get_1v1_bot_vs_default_config, get_1v1_selfplay_config
    from ..models.policy import get_config
    from ..transport.broker import make_broker
    from ..utils.metrics import MetricsWriter

    seed = args.seed if args.seed is not None else random.randrange(1 << 30)
    rng = random.Random(seed)
    cfg = get_config(args.model_preset)
    broker = make_broker(args.broker or f'tcp://{args.ip}:{args.port}')
    ws = WeightStore(cfg, device='cpu')
    if args.model:
        from ..utils.artifacts import resolve_model_path
        ws.load_file(resolve_model_path(args.model))
    broker.subscribe_model(ws.add_bytes)
    logger.info('waiting for the first model...')
    while not ws.wait_ready(timeout=5.0):
        logger.info('still waiting for weights')
    device = args.device
    if device.startswith('cuda') and not torch.cuda.is_available():
        device = 'cpu'

    def make_runner(policy):
        seed_r = rng.randrange(1 << 30)
        if device.startswith('cuda') and gpu_runner_supported(policy):
            # graph-captured batched GPU step; players' LSTM state lives in device slots
            return GpuRunner(policy.to(device), device=device, seed=seed_r, capacity=max(8, 2 * args.games),
                             )
        return PolicyRunner(policy, device=device, seed=seed_r)
    runner_for = RunnerCache(make_runner, latest_policy=ws.latest_policy)
    metrics = MetricsWriter(args.log_dir) if (args.validation and args.log_dir) else None
    uploader = None
    if metrics is not None and args.artifact_url:
        import os
        from ..utils.artifacts import Uploader, mirror_events, open_store
        uploader = Uploader(open_store(args.artifact_url))
        metrics.on_flush.append(mirror_events(uploader, os.path.basename(os.path.normpath(args.log_dir))))
    config_fn = (lambda: get_1v1_bot_vs_default_config(rng=rng)) if args.validation else get_1v1_selfplay_config
    from ..actor.league import League
    league = None if args.league == 'oldest' else League(ws, mode=args.league, rng=rng)
    runtime = args.runtime
    if runtime == 'auto':
        from .. import native
        runtime = 'vec' if (args.env == 'synthetic' and not args.validation and native.AVAILABLE) else 'service'
    if runtime == 'vec':
        if args.env != 'synthetic' or args.validation:
            raise SystemExit('--runtime vec drives the synthetic engine in self-play only')
        return _run_vec(args, ws, broker, league, device, seed, cfg)
    actor = Actor(make_services(args.env, args.games, seed), ws, runner_for,
                  None if args.validation else broker.publish_experience, config_fn,
                  rollout_size=args.rollout_size, max_dota_time=args.max_dota_time,
                  latest_weights_prob=args.use_latest_weights_prob, validation=args.validation, layout=cfg.layout,
                  hidden_size=cfg.hidden if cfg.rnn == 'lstm' else None, hidden_stride=args.hidden_stride,
                  wire=args.wire, metrics=metrics, rng=rng, league=league)
    t0 = time.time()
    last = 0
    try:
        while actor.games_finished < args.n_games:
            actor.step()
            if time.time() - t0 > 30:
                logger.info('actor steps/s: %.1f, games finished: %d, rollouts: %d',
                            (actor.steps_taken - last) / (time.time() - t0), actor.games_finished, actor.rollouts_sent)
                t0, last = time.time(), actor.steps_taken
    except Exception:   # reference: any exception ends the agent; the supervisor restarts it (agent.py:896-900)
        logger.exception('actor failed')
        return 1
    finally:
        if uploader is not None:
            uploader.flush()
    return 0


def _run_vec(args, ws, broker, league, device, seed, cfg):
    from ..actor.vec import VecActor
    va = VecActor(ws, args.games, broker.publish_experience, device=device,
                  mode='5v5' if cfg.layout.counts[0] > 1 else '1v1', seed=seed, rollout_size=args.rollout_size,
                  max_dota_time=args.max_dota_time, latest_weights_prob=args.use_latest_weights_prob,
                  hidden_stride=args.hidden_stride, threads=args.threads, league=league, stagger=True,
                  precision=args.actor_precision)
    try:
        va.run(n_games=args.n_games)
    except Exception:
        logger.exception('actor failed')
        return 1
    finally:
        va.close()
    return 0


if __name__ == '__main__':
    sys.exit(main())
