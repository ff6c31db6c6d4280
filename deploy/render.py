#!/usr/bin/env python3
"""Render the Kubernetes manifests in deploy/templates from deploy/params.yaml (the ksonnet app's role,
reference ks-app/). ``{{key}}`` is replaced by the parameter; ``#if key`` … ``#endif`` blocks are kept only when
the parameter is truthy. ``learner-multinode.yaml`` replaces ``learner.yaml`` when learner_nodes > 1, and
``agent-gpu.yaml`` is emitted only when gpu_agents > 0.

    python deploy/render.py --out build/ --set jobname=exp2 --set agents=40
"""
import argparse
import os
import re
import sys

import yaml

HERE = os.path.dirname(os.path.abspath(__file__))


def load_params(path, overrides):
    with open(path) as f:
        p = yaml.safe_load(f)
    for kv in overrides:
        k, v = kv.split('=', 1)
        p[k] = yaml.safe_load(v) if v else ''
    p['learner_workers'] = max(0, int(p.get('learner_nodes', 1)) - 1)
    return p


def render(text, params):
    out, keep = [], [True]
    for line in text.splitlines():
        s = line.strip()
        if s.startswith('#if '):
            keep.append(keep[-1] and bool(params.get(s[4:].strip())))
            continue
        if s == '#endif':
            keep.pop()
            continue
        if keep[-1]:
            out.append(line)

    def sub(m):
        k = m.group(1)
        if k not in params:
            raise KeyError(f'template parameter {k!r} missing from params')
        return str(params[k])
    return re.sub(r'\{\{(\w+)\}\}', sub, '\n'.join(out) + '\n')


def manifests(params):
    names = ['broker.yaml', 'agent.yaml', 'agent-val.yaml']
    names.append('learner-multinode.yaml' if int(params['learner_nodes']) > 1 else 'learner.yaml')
    if int(params.get('gpu_agents', 0)) > 0:
        names.append('agent-gpu.yaml')
    out = {}
    for n in names:
        with open(os.path.join(HERE, 'templates', n)) as f:
            out[n] = render(f.read(), params)
    return out


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--params', default=os.path.join(HERE, 'params.yaml'))
    ap.add_argument('--out', default='build')
    ap.add_argument('--set', action='append', default=[])
    args = ap.parse_args(argv)
    params = load_params(args.params, args.set)
    os.makedirs(args.out, exist_ok=True)
    for name, text in manifests(params).items():
        list(yaml.safe_load_all(text))            # validate
        with open(os.path.join(args.out, name), 'w') as f:
            f.write(text)
        print(os.path.join(args.out, name))
    return 0


if __name__ == '__main__':
    sys.exit(main())
