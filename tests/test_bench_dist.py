"""bench.py contract on the multi-process path (gloo on CPU, world_size 2 and 4): one JSON line from rank 0 with the
whole-job aggregate, weak-scaling fields and the BASELINE metric name."""
import json
import os
import socket
import subprocess
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _port():
    s = socket.socket()
    s.bind(('127.0.0.1', 0))
    p = s.getsockname()[1]
    s.close()
    return p


@pytest.mark.parametrize('world', [1, 2, 4])
def test_bench_json_contract_cpu(world):
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='2', CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='')
    args = ['bench.py', '--gpus', str(world), '--steps', '2', '--warmup', '1', '--batch-size', '2', '--seq-len', '16',
            '--model', 'lstm128', '--actor', '0']
    if world > 1:
        cmd = [sys.executable, '-m', 'torch.distributed.run', '--nnodes=1', f'--nproc-per-node={world}',
               '--master-addr', '127.0.0.1', '--master-port', str(_port())] + args
    else:
        cmd = [sys.executable] + args
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r['metric'] == 'PPO optimizer samples/sec (whole node) + actor steps/sec, 1v1-mid LSTM policy'
    assert r['n_gpus'] == world and r['steps'] == 2 and r['warmup'] == 1 and r['scaling'] == 'weak'
    assert r['higher_is_better'] is True and r['config']['parallelism'] == f'dp{world}'
    assert r['config']['global_batch'] == 2 * world and r['config']['seq_len'] == 16
    assert abs(r['value'] - 2 * world * 16 * 2 / (r['ms_per_step'] * 2 / 1e3)) / r['value'] < 1e-6
    assert r['vs_baseline'] == pytest.approx(r['value'] / 1000.0)
    assert r['dp_replicas_identical'] is True and len(r['weights_sha16_per_rank']) == world
    # every rank reports the host placement it ran with (CPU share, GPU-local NUMA node, derived thread counts)
    hp = r['host_placement']
    assert len(hp) == world and all(h['n_cpus'] >= 1 and h['actor_threads'] >= 1 and h['e2e_threads'] >= 1
                                    for h in hp)
    assert [h['local_rank'] for h in hp] == list(range(world))
    # per-rank all-reduce timing of the timed steps (DataParallel.comm_stats): the first multi-GPU driver run reports
    # where its step time went
    dc = r['dp_comm']
    if world == 1:
        assert dc is None
        return
    assert dc['dist_backend'] == 'gloo' and len(dc['per_rank']) == world
    for i, c in enumerate(dc['per_rank']):
        assert c['rank'] == i and c['dist_backend'] == 'gloo' and c['steps'] >= 1
        assert c['allreduce_ms'] > 0 and 0.0 <= c['overlap_frac'] <= 1.0 and c['exposed_ms'] >= 0
        assert len(c['bucket_mb']) == c['buckets'] >= 1
    assert dc['allreduce_ms_max'] == max(c['allreduce_ms'] for c in dc['per_rank'])


def test_bench_self_launches_ranks_for_gpus_flag():
    """``python bench.py --gpus 2`` with no launcher: bench.py starts the 2 rank processes itself (the driver's
    scaling run must never silently measure one GPU)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='2', CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='',
               DCA_DIST_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'LOCAL_WORLD_SIZE', 'MASTER_PORT'):
        env.pop(k, None)
    cmd = [sys.executable, 'bench.py', '--gpus', '2', '--steps', '2', '--warmup', '1', '--batch-size', '2',
           '--seq-len', '16', '--model', 'lstm128', '--actor', '0']
    out = subprocess.run(cmd, cwd=ROOT, env=env, capture_output=True, text=True, timeout=600)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [ln for ln in out.stdout.splitlines() if ln.startswith('{')]
    assert len(lines) == 1, out.stdout
    r = json.loads(lines[0])
    assert r['n_gpus'] == 2 and r['config']['parallelism'] == 'dp2' and r['config']['global_batch'] == 4
    assert r['dp_replicas_identical'] is True and len(r['weights_sha16_per_rank']) == 2
    assert [h['local_rank'] for h in r['host_placement']] == [0, 1]
    assert 'launched 2 ranks' in out.stderr


def test_bench_rejects_world_size_flag_mismatch():
    env = dict(os.environ, PYTHONPATH=ROOT, CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='', WORLD_SIZE='1',
               RANK='0', LOCAL_RANK='0')
    out = subprocess.run([sys.executable, 'bench.py', '--gpus', '4', '--steps', '1'], cwd=ROOT, env=env,
                         capture_output=True, text=True, timeout=300)
    assert out.returncode == 2 and 'WORLD_SIZE=1' in out.stderr


def test_bench_launcher_fails_when_a_rank_fails():
    """A failing rank makes the self-launched bench exit non-zero (and stops the others)."""
    env = dict(os.environ, PYTHONPATH=ROOT, OMP_NUM_THREADS='2', CUDA_VISIBLE_DEVICES='', HIP_VISIBLE_DEVICES='',
               DCA_DIST_BACKEND='gloo')
    for k in ('WORLD_SIZE', 'RANK', 'LOCAL_RANK', 'LOCAL_WORLD_SIZE', 'MASTER_PORT'):
        env.pop(k, None)
    out = subprocess.run([sys.executable, 'bench.py', '--gpus', '2', '--steps', '1', '--model', 'no-such-model',
                          '--actor', '0'], cwd=ROOT, env=env, capture_output=True, text=True, timeout=300)
    assert out.returncode != 0
