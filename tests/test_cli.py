"""CLI entrypoints: graph export (reference write_graph.py), standalone broker server, agent/optimizer parsers."""
import json
import os
import signal
import socket
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def test_write_graph_exports_torchscript_and_dot(tmp_path):
    from dotaclient_amd.cli import write_graph
    out = tmp_path / 'g'
    assert write_graph.main(['--model-preset', 'compat', '--out', str(out)]) == 0
    s = json.loads((out / 'summary.json').read_text())
    assert s['params'] == 434966                    # reference Policy size
    assert abs(s['flops_per_step'] - 2.09e6) < 0.02e6
    assert (out / 'graph.dot').read_text().startswith('digraph')
    import torch
    m = torch.jit.load(str(out / 'policy.pt'))
    outs = m(torch.zeros(2, 1, 3), torch.zeros(2, 1, 40, 10), torch.zeros(1, 2, 256), torch.zeros(1, 2, 256))
    assert len(outs) == 5


def _free_port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_broker_server_process_roundtrip():
    from dotaclient_amd.transport.broker import TcpBroker
    port = _free_port()
    env = dict(os.environ, PYTHONPATH=ROOT)
    proc = subprocess.Popen([sys.executable, '-m', 'dotaclient_amd.cli.broker', '--host', '127.0.0.1', '--port',
                             str(port)], env=env, cwd=ROOT)
    try:
        cli = TcpBroker('127.0.0.1', port, max_retries=60, retry_delay=0.25)
        cli.publish_experience(b'rollout-1')
        cli.publish_model(b'weights', 7)
        assert cli.consume_experience(timeout=5) == b'rollout-1'
        assert cli.latest_model() == (7, b'weights')
        cli.close()
    finally:
        proc.send_signal(signal.SIGTERM)
        proc.wait(timeout=20)
    assert proc.returncode == 0


def test_agent_and_optimizer_parsers_keep_reference_flags():
    from dotaclient_amd.cli import agent, optimizer
    a = agent.build_parser().parse_args(['--ip', '1.2.3.4', '--port', '1', '--rollout-size', '100',
                                         '--max-dota-time', '300', '-l', 'DEBUG', '--model', 'm.pt',
                                         '--use-latest-weights-prob', '0.8', '--validation', '1', '--log-dir', 'x'])
    assert (a.ip, a.rollout_size, a.use_latest_weights_prob, a.validation) == ('1.2.3.4', 100, 0.8, True)
    o = optimizer.build_parser().parse_args(['--epochs', '1', '--seq-per-epoch', '16', '--batch-size', '8',
                                             '--seq-len', '1400', '--learning-rate', '1e-4', '--entropy-coef', '0',
                                             '--vf-coef', '0.5', '--pretrained-model', 'p.pt',
                                             '--mq-prefetch-count', '2', '--run-local', 'false'])
    assert (o.batch_size, o.seq_len, o.run_local) == (8, 1400, False)
