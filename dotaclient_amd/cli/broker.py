"""Experience/model broker server — the RabbitMQ deployment's replacement (reference rmq.jsonnet, rabbitmq.conf,
enabled_plugins: an ``experience`` work queue consumed by learners + a ``model`` fanout with recent-history replay,
SURVEY §2.2 D5/D8).

    python -m dotaclient_amd.cli.broker --host 0.0.0.0 --port 5672 [--max-queue 4096 --drop-oldest true]

Actors (``cli.agent --broker tcp://host:5672``) publish rollouts; learner ranks (``cli.optimizer``) consume them and
publish versioned weights, which late-joining actors receive immediately (the recent-history exchange).
"""
from __future__ import annotations

import argparse
import logging
import signal
import sys
import threading

logger = logging.getLogger('dotaclient_amd.broker')


def str2bool(v):
    return str(v).lower() in ('1', 'true', 'yes', 'y', 't')


def main(argv=None):
    ap = argparse.ArgumentParser(formatter_class=argparse.ArgumentDefaultsHelpFormatter)
    ap.add_argument('--host', type=str, default='0.0.0.0')
    ap.add_argument('--port', type=int, default=5672)
    ap.add_argument('--max-queue', type=int, default=0, help='experience queue bound (0 = unbounded)')
    ap.add_argument('--drop-oldest', type=str2bool, default=False,
                    help='when full, drop the oldest rollout instead of blocking publishers')
    ap.add_argument('-l', '--log', dest='log_level', default='INFO')
    args = ap.parse_args(argv)
    logging.basicConfig(format='%(asctime)s %(levelname)-8s %(message)s', level=args.log_level)
    from ..transport.broker import TcpBrokerServer
    srv = TcpBrokerServer(args.host, args.port, maxsize=args.max_queue, drop_oldest=args.drop_oldest).start()
    logger.info('broker listening on %s:%d', args.host, srv.port)
    done = threading.Event()
    signal.signal(signal.SIGINT, lambda *_: done.set())
    signal.signal(signal.SIGTERM, lambda *_: done.set())
    done.wait()
    srv.stop()
    return 0


if __name__ == '__main__':
    sys.exit(main())
