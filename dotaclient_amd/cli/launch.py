"""Single-node job launcher: broker + learner rank(s) + actor processes (+ optional validation actor).

The reference deploys this as k8s objects (ks-app/components/{rmq,optimizer,agent,agent-val}.jsonnet); this launcher
runs the same topology on one machine (and is what ``deploy/`` manifests call per pod):

    python -m dotaclient_amd.cli.launch --actors 4 --games-per-actor 16 --optimizers 1 --log-dir runs/exp1

Children are supervised: an actor that exits is restarted (the reference relies on k8s restarting agent pods,
agent.py:896-900); the learner is restarted with resume-from-checkpoint (``restartPolicy: OnFailure``,
optimizer.jsonnet:82). Ctrl-C / SIGTERM stops the whole job.
"""
from __future__ import annotations

import argparse
import logging
import os
import signal
import subprocess
import sys
import time

logger = logging.getLogger('dotaclient_amd.launch')


def build_parser():
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    from ..presets import add_preset_arg
    add_preset_arg(ap)
    ap.add_argument('--port', type=int, default=5672)
    ap.add_argument('--actors', type=int, default=2)
    ap.add_argument('--games-per-actor', type=int, default=4)
    ap.add_argument('--optimizers', type=int, default=1, help='learner ranks (one per GPU)')
    ap.add_argument('--validation', type=int, default=0, help='number of validation actors')
    ap.add_argument('--log-dir', type=str, default='runs/local')
    ap.add_argument('--model-preset', type=str, default='lstm512')
    ap.add_argument('--actor-device', type=str, default='cpu')
    ap.add_argument('--max-restarts', type=int, default=5)
    ap.add_argument('--duration', type=float, default=0.0, help='stop after N seconds (0 = run forever)')
    ap.add_argument('optimizer_args', nargs=argparse.REMAINDER, help='extra args after -- go to the optimizer')
    return ap


class Supervisor:
    """Restart-on-exit process supervisor (the reference relies on k8s for this: agent pods are restarted when
    agent.py returns, agent.py:896-900; the optimizer Job has ``restartPolicy: OnFailure``)."""

    def __init__(self, specs, max_restarts: int = 5, env=None):
        self.specs = dict(specs)
        self.max_restarts = max_restarts
        self.env = env
        self.procs = {}
        self.restarts = {k: 0 for k in self.specs}
        self.failed = None

    def start(self):
        for k, cmd in self.specs.items():
            self.procs[k] = subprocess.Popen(cmd, env=self.env)
        return self

    def poll(self) -> bool:
        """Restart exited children; False once a child exhausted its restart budget."""
        for k, p in list(self.procs.items()):
            code = p.poll()
            if code is None:
                continue
            if self.restarts[k] >= self.max_restarts:
                logger.error('%s exited with %s; restart budget exhausted', k, code)
                self.failed = (k, code)
                return False
            self.restarts[k] += 1
            logger.warning('%s exited with %s; restarting (%d/%d)', k, code, self.restarts[k], self.max_restarts)
            self.procs[k] = subprocess.Popen(self.specs[k], env=self.env)
        return True

    def stop(self, timeout: float = 20.0):
        for p in self.procs.values():
            if p.poll() is None:
                p.terminate()
        for p in self.procs.values():
            try:
                p.wait(timeout=timeout)
            except subprocess.TimeoutExpired:
                p.kill()


def main(argv=None):
    from ..presets import parse_with_preset
    args = parse_with_preset(build_parser(), 'launch', argv)
    logging.basicConfig(format='%(asctime)s %(levelname)-8s %(message)s', level='INFO')
    from ..transport.broker import TcpBrokerServer
    srv = TcpBrokerServer('127.0.0.1', args.port).start()
    logger.info('broker on 127.0.0.1:%d', srv.port)
    py = sys.executable
    extra = [a for a in args.optimizer_args if a != '--']
    specs = {}
    if args.optimizers > 1:
        specs['optimizer'] = [py, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={args.optimizers}',
                              '--master-addr', '127.0.0.1', '-m', 'dotaclient_amd.cli.optimizer']
    else:
        specs['optimizer'] = [py, '-m', 'dotaclient_amd.cli.optimizer']
    pre = ['--preset', args.preset] if args.preset else []
    specs['optimizer'] += (pre + ['--port', str(srv.port), '--log-dir', args.log_dir, '--model-preset',
                                  args.model_preset] + extra)
    for i in range(args.actors):
        dev = args.actor_device
        if dev == 'cuda' and args.optimizers > 1:
            dev = f'cuda:{i % args.optimizers}'          # one actor process per GPU next to its learner rank
        specs[f'actor{i}'] = [py, '-m', 'dotaclient_amd.cli.agent'] + pre + [
            '--port', str(srv.port), '--games', str(args.games_per_actor), '--device', dev, '--model-preset',
            args.model_preset, '--seed', str(1000 + i)]
    for i in range(args.validation):
        specs[f'val{i}'] = [py, '-m', 'dotaclient_amd.cli.agent', '--port', str(srv.port), '--validation', 'true',
                            '--log-dir', os.path.join(args.log_dir, 'val'), '--model-preset', args.model_preset]
    sup = Supervisor(specs, args.max_restarts).start()
    stop = {'flag': False}

    def handler(*_):
        stop['flag'] = True
    signal.signal(signal.SIGINT, handler)
    signal.signal(signal.SIGTERM, handler)
    t0 = time.time()
    rc = 0
    try:
        while not stop['flag']:
            if args.duration and time.time() - t0 > args.duration:
                break
            if not sup.poll():
                rc = sup.failed[1] or 1
                break
            time.sleep(1.0)
    finally:
        sup.stop()
        srv.stop()
    return rc


if __name__ == '__main__':
    sys.exit(main())
