"""Deployment manifests render to valid YAML with the reference's job parameters (ks-app params.libsonnet)."""
import os
import sys

import yaml

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, 'deploy'))


def test_render_single_node(tmp_path):
    import render
    assert render.main(['--out', str(tmp_path)]) == 0
    docs = {n: list(yaml.safe_load_all((tmp_path / n).read_text())) for n in os.listdir(tmp_path)}
    assert set(docs) == {'broker.yaml', 'agent.yaml', 'agent-val.yaml', 'learner.yaml'}
    agent = docs['agent.yaml'][0]
    assert agent['spec']['replicas'] == 22
    args = agent['spec']['template']['spec']['containers'][0]['args']
    assert args[args.index('--rollout-size') + 1] == '9999'
    learner = docs['learner.yaml'][0]['spec']['template']['spec']['containers'][0]
    assert learner['resources']['limits']['amd.com/gpu'] == 8
    assert '--nproc-per-node' in learner['command']
    assert learner['args'][learner['args'].index('--seq-len') + 1] == '1400'


def test_render_multinode_gpu_actors_and_sidecar(tmp_path):
    import render
    render.main(['--out', str(tmp_path), '--set', 'learner_nodes=4', '--set', 'gpu_agents=2',
                 '--set', 'dotaservice_image=ds:0.3.8'])
    names = set(os.listdir(tmp_path))
    assert 'learner-multinode.yaml' in names and 'learner.yaml' not in names and 'agent-gpu.yaml' in names
    pj = yaml.safe_load((tmp_path / 'learner-multinode.yaml').read_text())
    assert pj['spec']['pytorchReplicaSpecs']['Worker']['replicas'] == 3
    agent = yaml.safe_load((tmp_path / 'agent.yaml').read_text())
    assert [c['name'] for c in agent['spec']['template']['spec']['containers']] == ['agent', 'dotaservice']
