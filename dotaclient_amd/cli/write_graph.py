"""Export the policy graph (the reference's ``write_graph.py``, which is broken: it imports jax and calls Policy
with the wrong signature — write_graph.py:1-22).

    python -m dotaclient_amd.cli.write_graph --model-preset lstm512 --out runs/graph

Writes into ``--out``:
  * ``policy.pt``        TorchScript trace of one batched policy step ``(env, units, h, c) → (logits…, value, h, c)``
  * ``graph.txt``        the torch.fx graph (one op per line) and a parameter table
  * ``graph.dot``        Graphviz rendering of the fx graph (``dot -Tpng graph.dot``)
  * ``summary.json``     parameter count, per-step FLOPs, layout
"""
from __future__ import annotations

import argparse
import json
import os
import sys

import torch


class _Step(torch.nn.Module):
    """Single-step policy with explicit recurrent state (what the actor runs)."""

    def __init__(self, policy):
        super().__init__()
        self.policy = policy

    def forward(self, env, units, h, c):
        hidden = (h, c) if self.policy.is_recurrent else None
        logits, value, hn = self.policy.forward_packed(env, units, hidden)
        out = [logits[k] for k in sorted(logits)] + [value]
        if hn is not None:
            out += [hn[0], hn[1]]
        return tuple(out)


def step_flops(cfg) -> int:
    U = cfg.layout.max_units
    f = 2 * (3 * cfg.env_dim + U * 10 * 128 + U * 128 * cfg.unit_dim)
    f += 2 * (cfg.env_dim + 6 * cfg.unit_dim) * cfg.pre_rnn_dim
    f += 2 * 4 * cfg.hidden * (cfg.pre_rnn_dim + cfg.hidden) if cfg.rnn == 'lstm' else 2 * cfg.pre_rnn_dim * cfg.hidden
    f += 2 * cfg.hidden * (128 + 3 + 9 + 9 + 1) + 2 * U * 128
    return int(f)


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--model-preset', type=str, default='lstm512')
    ap.add_argument('--out', type=str, default='graph')
    ap.add_argument('--batch', type=int, default=2)
    args = ap.parse_args(argv)
    from ..models.policy import Policy, get_config
    cfg = get_config(args.model_preset)
    pol = Policy(cfg).eval()
    os.makedirs(args.out, exist_ok=True)
    n, U, H = args.batch, cfg.layout.max_units, cfg.hidden
    ex = (torch.zeros(n, 1, 3), torch.zeros(n, 1, U, 10), torch.zeros(1, n, H), torch.zeros(1, n, H))
    step = _Step(pol).eval()
    with torch.no_grad():
        traced = torch.jit.trace(step, ex, check_trace=False)
    traced.save(os.path.join(args.out, 'policy.pt'))
    import torch.fx as fx

    class _Leaf(fx.Tracer):
        def is_leaf_module(self, m, qn):
            return isinstance(m, (torch.nn.LSTM, torch.nn.Linear)) or super().is_leaf_module(m, qn)

    graph = _Leaf().trace(step)
    lines = [f'{nd.op:14s} {nd.name:40s} {str(nd.target)[:60]:60s} args={nd.args}' for nd in graph.nodes]
    params = [(k, tuple(v.shape), v.numel()) for k, v in pol.state_dict().items()]
    with open(os.path.join(args.out, 'graph.txt'), 'w') as f:
        f.write('\n'.join(lines) + '\n\n# parameters\n')
        f.writelines(f'{k:40s} {str(s):20s} {c}\n' for k, s, c in params)
    with open(os.path.join(args.out, 'graph.dot'), 'w') as f:
        f.write('digraph policy {\n  rankdir=TB; node [shape=box, fontsize=10];\n')
        for nd in graph.nodes:
            label = nd.name if nd.op in ('placeholder', 'output') else f'{nd.name}\\n{str(nd.target)[:40]}'
            f.write(f'  "{nd.name}" [label="{label}"];\n')
            for a in nd.all_input_nodes:
                f.write(f'  "{a.name}" -> "{nd.name}";\n')
        f.write('}\n')
    summary = {'preset': args.model_preset, 'params': sum(c for _, _, c in params),
               'flops_per_step': step_flops(cfg), 'units': U, 'hidden': H, 'rnn': cfg.rnn,
               'nodes': len(lines)}
    with open(os.path.join(args.out, 'summary.json'), 'w') as f:
        json.dump(summary, f, indent=1)
    print(json.dumps(summary))
    return 0


if __name__ == '__main__':
    sys.exit(main())
