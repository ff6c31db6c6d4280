"""bench.py's multi-rank path on the MI355X at the deploy shape: two ranks launched by
torch.distributed.run share cuda:0 (DCA_SHARED_GPU=1) and talk gloo (DCA_DIST_BACKEND=gloo; RCCL refuses two ranks
on one device). lstm512, batch 8 × seq 1400, fused backend with the graph-captured split step (recurrence/heads
buckets all-reduced between the two graph replays), every rank's actor runtime, and the node e2e loop (one actor
process per rank → one shared-memory queue → two learner ranks, rank 0 publishing)."""
import json
import os
import socket
import subprocess
import sys

import pytest
import torch

pytestmark = pytest.mark.gpu
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


def test_bench_two_ranks_on_one_gpu_deploy_shape():
    if not torch.cuda.is_available():
        pytest.skip('no GPU')
    env = dict(os.environ, PYTHONPATH=ROOT, DCA_SHARED_GPU='1', DCA_DIST_BACKEND='gloo', OMP_NUM_THREADS='4')
    cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', '--nproc-per-node=2',
           '--master-addr', '127.0.0.1', '--master-port', str(_port()), 'bench.py', '--gpus', '2', '--steps', '3',
           '--warmup', '2', '--bf16x3-extra', '0', '--actor-games', '256', '--actor-threads', '4', '--e2e', '6',
           '--e2e-games', '128', '--e2e-probe', '1']
    # the ranks' progress goes to a file under gpurun_out/ as it happens (a long run stays visibly alive)
    os.makedirs(os.path.join(ROOT, 'gpurun_out'), exist_ok=True)
    log = os.path.join(ROOT, 'gpurun_out', 'bench_2rank_shared_gpu.err')
    with open(log, 'w') as err:
        out = subprocess.run(cmd, cwd=ROOT, env=env, stdout=subprocess.PIPE, stderr=err, text=True, timeout=600)
    assert out.returncode == 0, open(log).read()[-4000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout[-4000:]
    r = json.loads(lines[0])
    assert r['n_gpus'] == 2 and r['config']['parallelism'] == 'dp2'
    assert r['config']['global_batch'] == 16 and r['config']['seq_len'] == 1400
    assert r['config']['backend'] == 'fused' and r['config']['model'].startswith('lstm512')
    step = r['config']['step']
    assert step['hipgraph'] and step['dp_split_overlap'] and step['dist_backend'] == 'gloo'
    assert r['dp_replicas_identical'] is True
    a = r['actor']
    assert a['ranks'] == 2 and len(a['steps_per_s_per_rank']) == 2 and a['steps_per_s'] > 0
    e = r['e2e']
    assert 'error' not in e, e
    assert e['ranks'] == 2 and e['steps_per_s'] > 0 and len(e['steps_per_s_per_rank']) == 2
    assert e['iterations'] >= 1 and e['queue_dropped'] >= 0
