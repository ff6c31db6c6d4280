"""Learner entrypoint (reference ``optimizer.py`` CLI, optimizer.py:769-809).

Reference-compatible flags: ``--log-dir --ip --port --epochs --seq-per-epoch --batch-size --seq-len --learning-rate
--entropy-coef --vf-coef --pretrained-model --mq-prefetch-count -l/--log --run-local``. Additional: ``--broker``,
``--algo`` (ppo | vpg), ``--model-preset``, ``--iterations``, ``--device``, ``--backend`` (fused | torch),
``--precision`` (fp32-exact | fp32 | bf16), ``--pack-sequences``,
``--gamma --gae-lambda --clip-eps --max-grad-norm --compat-value-bug --checkpoint-keep``.

Data parallel: launch one process per GPU with ``torch.distributed.run`` (RCCL over xGMI); every rank consumes
disjoint rollouts from the shared queue, rank 0 checkpoints and publishes (optimizer.py:718-762):

    python -m torch.distributed.run --nproc-per-node 8 --master-addr 127.0.0.1 -m dotaclient_amd.cli.optimizer ...
"""
from __future__ import annotations

import argparse
import logging
import sys

logger = logging.getLogger('dotaclient_amd.optimizer')


def str2bool(v):
    return str(v).lower() in ('1', 'true', 'yes', 'y', 't')


def build_parser():
    from ..learner.optimizer import default_log_dir
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    from ..presets import add_preset_arg
    add_preset_arg(ap)
    ap.add_argument('--log-dir', type=str, default=default_log_dir())
    ap.add_argument('--ip', type=str, default='127.0.0.1')
    ap.add_argument('--port', type=int, default=5672)
    ap.add_argument('--broker', type=str, default=None)
    ap.add_argument('--epochs', type=int, default=4)
    ap.add_argument('--seq-per-epoch', type=int, default=16)
    ap.add_argument('--batch-size', type=int, default=4)
    ap.add_argument('--seq-len', type=int, default=256)
    ap.add_argument('--learning-rate', type=float, default=1e-4)
    ap.add_argument('--entropy-coef', type=float, default=0.01)
    ap.add_argument('--vf-coef', type=float, default=0.5)
    ap.add_argument('--pretrained-model', type=str, default=None)
    ap.add_argument('--mq-prefetch-count', type=int, default=4)
    ap.add_argument('-l', '--log', dest='log_level', default='INFO',
                    choices=['DEBUG', 'INFO', 'WARNING', 'ERROR', 'CRITICAL'])
    ap.add_argument('--run-local', type=str2bool, default=None,
                    help='disable the artifact store (default: on when --artifact-url is not given)')
    ap.add_argument('--artifact-url', type=str, default=None,
                    help='mirror checkpoints + events here (dir, file://, or an fsspec URL such as gs://bucket)')
    ap.add_argument('--algo', type=str, default='ppo', choices=['ppo', 'vpg'])
    ap.add_argument('--model-preset', type=str, default='lstm512')
    ap.add_argument('--iterations', type=int, default=10000)
    ap.add_argument('--device', type=str, default='auto')
    ap.add_argument('--backend', type=str, default='auto', choices=['auto', 'fused', 'torch'])
    ap.add_argument('--graph', type=int, default=1, help='capture the fused train step in a hipGraph')
    ap.add_argument('--async-checkpoint', type=int, default=1,
                    help='publish the model first, write checkpoint files on a background thread')
    ap.add_argument('--precision', type=str, default='fp32-exact', choices=['fp32-exact', 'fp32', 'bf16'],
                    help='fp32-exact = the reference training precision (IEEE fp32 products on f32 MFMA / VALU); '
                         'fp32 = fp32 activations with bf16x3-split MFMA operands; bf16 = bf16 GEMM operands '
                         '(the 5v5 entity-attention policy runs fp32 or bf16)')
    ap.add_argument('--pack-sequences', type=str2bool, default=False,
                    help='pack whole episodes into the seq_len sequences with episode-start resets instead of '
                         'padding every rollout (non-reference layout; GPU device ingest)')
    ap.add_argument('--advantages', type=str, default='vtrace-step',
                    choices=['vtrace-step', 'vtrace-iteration', 'gae'],
                    help='PPO advantages of stale / replayed experience: V-trace inside every learner step (default), '
                         'the per-iteration policy_old forward + V-trace, or GAE from the actor values')
    ap.add_argument('--old-logp', type=str, default='actor', choices=['actor', 'learner'],
                    help="PPO ratio denominator: the actor's behaviour log-prob or the learner's policy_old")
    ap.add_argument('--gamma', type=float, default=0.98)
    ap.add_argument('--gae-lambda', type=float, default=0.95)
    ap.add_argument('--clip-eps', type=float, default=0.1)
    ap.add_argument('--max-grad-norm', type=float, default=0.5)
    ap.add_argument('--compat-value-bug', type=str2bool, default=False)
    ap.add_argument('--checkpoint-keep', type=int, default=0)
    ap.add_argument('--replay-gb', type=float, default=0.0, help='on-HBM replay buffer budget in GB (0 = off)')
    ap.add_argument('--replay-capacity', type=int, default=0, help='replay capacity in sequences (overrides GB)')
    ap.add_argument('--replay-recent', type=int, default=0, help='sample from the newest N sequences (0 = all)')
    ap.add_argument('--prefetch-rollouts', type=int, default=0,
                    help='decode up to N experience messages ahead on a background thread (0 = inline)')
    ap.add_argument('--allow-pickle-experience', type=str2bool, default=False,
                    help='also accept reference agents\' pickled experience (restricted unpickler: arrays only)')
    return ap


def main(argv=None):
    from ..presets import parse_with_preset
    args = parse_with_preset(build_parser(), 'optimizer', argv)
    logging.basicConfig(format='%(asctime)s %(levelname)-8s %(message)s', level=args.log_level)
    import torch
    from ..learner.optimizer import DotaOptimizer, OptimizerConfig
    from ..parallel import dist as pdist
    from ..transport.broker import make_broker
    device = args.device
    if device == 'auto':
        device = f'cuda:{pdist.local_rank()}' if torch.cuda.is_available() else 'cpu'
    if device.startswith('cuda'):
        torch.cuda.set_device(torch.device(device))
    pdist.init_distribution(device=device)
    cfg = OptimizerConfig(log_dir=args.log_dir, epochs=args.epochs, seq_per_epoch=args.seq_per_epoch,
                          batch_size=args.batch_size, seq_len=args.seq_len, learning_rate=args.learning_rate,
                          entropy_coef=args.entropy_coef, vf_coef=args.vf_coef, pretrained_model=args.pretrained_model,
                          mq_prefetch_count=args.mq_prefetch_count,
                          run_local=(args.artifact_url is None) if args.run_local is None else args.run_local,
                          artifact_url=args.artifact_url,
                          iterations=args.iterations, algo=args.algo, model=args.model_preset, gamma=args.gamma,
                          gae_lambda=args.gae_lambda, clip_eps=args.clip_eps, max_grad_norm=args.max_grad_norm,
                          advantages=args.advantages, old_logp=args.old_logp,
                          compat_value_bug=args.compat_value_bug, device=device, backend=args.backend,
                          precision=args.precision, graph=bool(args.graph), async_checkpoint=bool(args.async_checkpoint),
                          checkpoint_keep=args.checkpoint_keep, replay_gb=args.replay_gb,
                          replay_capacity=args.replay_capacity, replay_recent=args.replay_recent,
                          allow_pickle_experience=args.allow_pickle_experience,
                          prefetch_rollouts=args.prefetch_rollouts, pack_sequences=args.pack_sequences)
    broker = make_broker(args.broker or f'tcp://{args.ip}:{args.port}')
    try:
        DotaOptimizer(cfg, broker).run()
    except KeyboardInterrupt:
        pass
    finally:
        pdist.destroy()
    return 0


if __name__ == '__main__':
    sys.exit(main())
