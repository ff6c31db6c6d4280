#!/usr/bin/env python3
"""Actor precision vs the learner's IEEE-fp32 policy: the PPO ratio bias at weight age 0 and the head-distribution KL
of the fp32 / bf16 / fp8 actor policy steps against torch fp32.

The reference trains PPO-style on log-probs its fp32 actor recorded (agent.py:641-660; the ratio sketch at
optimizer.py:632-639 against policy_old). Here the learner's ``logp_old`` is the actor's recorded log-prob, so an
actor at lower precision than the learner biases the ratio exp(logp_learner − logp_actor) away from 1 even at weight
age 0. For every actor precision this plays ``--steps`` recurrent steps of ``--slots`` player slots on synthetic
world states (the same observations and carried LSTM state for every precision) and compares with the torch fp32
policy at the same weights:

* ``dlogp_max`` / ``dlogp_mean``: |log-prob of the sampled action, actor − torch fp32|;
* ``ratio_bias``: mean |exp(torch − actor) − 1| (the PPO ratio at weight age 0), ``clipfrac_0.1`` / ``_0.2``: the
  fraction of samples whose ratio leaves [1 − ε, 1 + ε] (reference e_clip 0.1, optimizer.py:239);
* ``kl_<head>``: mean KL(torch fp32 ‖ actor) of the enum / x / y head distributions (from the actor's head logits);
* ``value_max``: |V actor − V torch|.

    python scripts/actor_precision_check.py [--model ckpt.pt] --out profiles/r5_actor_precision.jsonl
"""
import argparse
import json
import os
import sys

import numpy as np
import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))


def main(argv=None):
    ap = argparse.ArgumentParser()
    ap.add_argument('--preset', default='lstm512')
    ap.add_argument('--model', default=None, help='state_dict checkpoint (model_%%09d.pt); default: random init')
    ap.add_argument('--slots', type=int, default=2048)
    ap.add_argument('--steps', type=int, default=6)
    ap.add_argument('--precisions', default='fp32,bf16,fp8')
    ap.add_argument('--label', default='')
    ap.add_argument('--out', default='gpurun_out/actor_precision.jsonl')
    a = ap.parse_args(argv)
    from dotaclient_amd.actor.batched import F32ActorPolicy, Fp8ActorPolicy, GpuActorPolicy, _synthetic_states
    from dotaclient_amd.features.featurizer import featurize
    from dotaclient_amd.models.policy import Policy, batched_action_masks, get_config, masked_log_softmax
    from dotaclient_amd.protos import pb
    from dotaclient_amd.utils.checkpoint import load_model_file

    torch.backends.cuda.matmul.allow_tf32 = False
    torch.manual_seed(3)
    cfg = get_config(a.preset)
    pol = Policy(cfg)
    if a.model:
        pol.load_state_dict(load_model_file(a.model), strict=True)
    pol = pol.cuda().eval()
    n, lay = a.slots, cfg.layout
    states = _synthetic_states(512)
    obs = []
    for step in range(a.steps):
        feats = []
        for i in range(n):
            j = (i * 7 + step * 131) % len(states)      # even entries are Radiant's view, odd ones Dire's
            ws = pb.CMsgBotWorldState.FromString(states[j])
            team = 2 if j % 2 == 0 else 3
            feats.append(featurize(ws, 0 if team == 2 else 5, team, lay))
        obs.append((np.stack([f.env for f in feats]).astype(np.float32),
                    np.stack([f.units for f in feats]).astype(np.float32),
                    np.stack([f.handles for f in feats]).astype(np.int64)))
    classes = {'fp32': F32ActorPolicy, 'bf16': GpuActorPolicy, 'fp8': Fp8ActorPolicy}
    heads = (('enum', 0, 3), ('x', 3, 9), ('y', 12, 9))
    rows = []
    for prec in a.precisions.split(','):
        gp = classes[prec](pol, n, device='cuda', seed=5)
        hidden = pol.initial_hidden(n, device='cuda')
        acc = {k: [] for k in ('dlogp', 'ratio', 'dv')}
        kl = {k: [] for k, _, _ in heads}
        for env, units, handles in obs:
            out = gp.step(env, units, handles)
            z = gp.z.float().clone()
            with torch.no_grad():
                e = torch.as_tensor(env, device='cuda')[:, None]
                u = torch.as_tensor(units, device='cuda')[:, None]
                logits, value, hidden = pol.forward_packed(e, u, hidden)
                valid = batched_action_masks(torch.as_tensor(handles, device='cuda'))
                lps = {k: masked_log_softmax(logits[k][:, 0].reshape(n, -1).float(), valid[:, o:o + w], dim=-1)
                       for k, o, w in heads + (('target_unit', 21, lay.max_units),)}
                for k, o, w in heads:
                    la = masked_log_softmax(z[:, 128 + o:128 + o + w], valid[:, o:o + w], dim=-1)
                    p = lps[k].exp()
                    d = torch.where(p > 0, p * (lps[k] - la), torch.zeros_like(p))
                    kl[k].append(d.sum(-1))
            idx = torch.as_tensor(out['idx'], device='cuda').long()
            r = torch.arange(n, device='cuda')
            enum, x, y, t = idx.unbind(1)
            mv, att = enum == 1, enum == 2
            ref = lps['enum'][r, enum] + mv * (lps['x'][r, x] + lps['y'][r, y]) + torch.where(
                att, lps['target_unit'][r, t], 0.)
            got = torch.as_tensor(out['logp'], device='cuda')
            acc['dlogp'].append((got - ref).abs())
            acc['ratio'].append(torch.exp(ref - got))
            acc['dv'].append((torch.as_tensor(out['value'], device='cuda') - value[:, 0, 0].float()).abs())
        d = torch.cat(acc['dlogp'])
        ratio = torch.cat(acc['ratio'])
        row = {'precision': prec, 'preset': a.preset, 'weights': a.model or 'random-init', 'label': a.label,
               'samples': int(d.numel()), 'dlogp_max': float(d.max()), 'dlogp_mean': float(d.mean()),
               'ratio_bias': float((ratio - 1).abs().mean()), 'ratio_max_dev': float((ratio - 1).abs().max()),
               'clipfrac_0.1': float(((ratio - 1).abs() > 0.1).float().mean()),
               'clipfrac_0.2': float(((ratio - 1).abs() > 0.2).float().mean()),
               'value_max': float(torch.cat(acc['dv']).max())}
        for k in kl:
            row[f'kl_{k}'] = float(torch.cat(kl[k]).mean())
        rows.append(row)
        print(json.dumps(row), flush=True)
        del gp
    os.makedirs(os.path.dirname(os.path.abspath(a.out)), exist_ok=True)
    with open(a.out, 'a') as fh:
        for row in rows:
            fh.write(json.dumps(row) + '\n')


if __name__ == '__main__':
    main()
