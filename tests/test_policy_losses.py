"""Reference policy (compat) parity, action helpers, and the dense losses vs the reference's masked_select formula
(optimizer.py:602-672)."""
import importlib.util
import os

import numpy as np
import pytest
import torch

from dotaclient_amd.learner.losses import ppo_loss, split_heads, vpg_loss
from dotaclient_amd.learner.synthetic import make_batch
from dotaclient_amd.models.policy import Policy, batched_action_masks, get_config, masked_log_softmax
from dotaclient_amd.constants import LAYOUT_1V1

REF = '/root/reference/policy.py'


def _ref_policy_module():
    if not os.path.exists(REF):
        pytest.skip('reference checkout not mounted')
    spec = importlib.util.spec_from_file_location('ref_policy', REF)
    m = importlib.util.module_from_spec(spec)
    spec.loader.exec_module(m)
    return m


def _inputs(B=2, S=3, seed=0):
    g = torch.Generator().manual_seed(seed)
    counts = LAYOUT_1V1.counts
    keys = ['allied_heroes', 'enemy_heroes', 'allied_nonheroes', 'enemy_nonheroes', 'allied_towers', 'enemy_towers']
    d = {'env': torch.randn(B, S, 3, generator=g)}
    for k, c in zip(keys, counts):
        d[k] = torch.randn(B, S, c, 10, generator=g)
    return d


def test_compat_policy_matches_reference_exactly():
    ref = _ref_policy_module()
    r = ref.Policy()
    m = Policy('compat')
    assert sorted(r.state_dict()) == sorted(m.state_dict())
    m.load_state_dict(r.state_dict(), strict=True)
    inp = _inputs()
    a, va, _ = r(**inp, hidden=None)
    b, vb, _ = m(**inp, hidden=None)
    for k in a:
        torch.testing.assert_close(a[k], b[k], rtol=0, atol=0)
    torch.testing.assert_close(va, vb, rtol=0, atol=0)
    mask = torch.rand(2, 3, 40) > 0.4
    mask[..., 5] = True
    torch.testing.assert_close(ref.Policy.masked_softmax(a['target_unit'], mask)[mask],
                               m.masked_softmax(a['target_unit'], mask)[mask])


def test_fixed_policy_differs_only_in_enemy_tower_pool():
    p = Policy(get_config('compat'))
    q = Policy(get_config('compat'))
    q.config.compat_bugs = False
    q.load_state_dict(p.state_dict())
    inp = _inputs()
    a, _, _ = p(**inp)
    inp2 = dict(inp)
    inp2['enemy_towers'] = inp['enemy_towers'] * 3.0   # compat ignores enemy towers in the pool
    a2, _, _ = p(**inp2)
    torch.testing.assert_close(a['enum'], a2['enum'])
    b, _, _ = q(**inp)
    b2, _, _ = q(**inp2)
    assert not torch.allclose(b['enum'], b2['enum'])


@pytest.mark.parametrize('preset', ['lstm128', 'lstm512', '5v5'])
def test_presets_forward_and_hidden(preset):
    cfg = get_config(preset)
    p = Policy(cfg)
    B, S, U = 2, 5, cfg.layout.max_units
    env, units = torch.randn(B, S, 3), torch.randn(B, S, U, 10)
    logits, v, h = p.forward_packed(env, units)
    assert logits['target_unit'].shape == (B, S, U) and v.shape == (B, S, 1)
    # running the sequence in two halves with the carried state = one pass
    l1, _, h1 = p.forward_packed(env[:, :2], units[:, :2])
    l2, _, _ = p.forward_packed(env[:, 2:], units[:, 2:], h1)
    torch.testing.assert_close(torch.cat([l1['enum'], l2['enum']], 1), logits['enum'], rtol=1e-5, atol=1e-5)


def test_masked_log_softmax_stable_equals_reference_formula():
    x = torch.randn(4, 7, 40) * 3
    m = torch.rand(4, 7, 40) > 0.5
    m[0, 0] = False        # empty row stays finite
    a = masked_log_softmax(x, m, stable=True)
    b = masked_log_softmax(x, m, stable=False)
    assert torch.isfinite(a).all()
    torch.testing.assert_close(a[m], b[m], rtol=1e-5, atol=1e-5)
    big = torch.full((1, 3), 1000.0)
    assert torch.isfinite(masked_log_softmax(big, torch.ones(1, 3, dtype=torch.bool))).all()


def test_action_masks_and_helpers():
    p = Policy('compat')
    handles = torch.full((40,), -1)
    handles[0] = 7                         # self only → no attack
    m = p.action_masks(handles)
    assert m['enum'][0, 0, 2] == 0 and m['target_unit'].sum() == 0
    handles[3] = 9
    m = p.action_masks(handles)
    assert m['enum'][0, 0, 2] == 1 and m['target_unit'][0, 0, 3] == 1 and m['target_unit'][0, 0, 0] == 0
    bm = batched_action_masks(torch.stack([handles, torch.full((40,), -1)]))
    assert bm[0, 2] and not bm[1, 2] and bm.shape == (2, 61)
    sel = p.flatten_selections({'enum': 1, 'x': 3, 'y': 4})
    assert sel['x'][3] == 1 and sel['target_unit'].sum() == 0
    flat = torch.cat([sel[k] for k in ['enum', 'x', 'y', 'target_unit']]).unsqueeze(0)
    hm = p.flat_actions_to_headmask(flat)
    assert hm[0, :21].all() and not hm[0, 21:].any()
    logits = {k: torch.randn(1, 1, n) for k, n in p.ACTION_OUTPUT_COUNTS.items()}
    a = p.select_actions(logits, p.action_masks(handles))
    assert int(a['enum']) in (0, 1, 2)


def _reference_vpg(logits, values, actions, masks, norm_ret, returns, ent_coef, vf_coef):
    """Literal re-statement of optimizer.py:602-672 (masked_select form)."""
    advantage = values - returns[-1]
    policy_loss, entropies = {}, {}
    for key in logits:
        exp = torch.exp(logits[key])
        me = exp.clone()
        me[~masks[key].bool()] = 0.
        lp = logits[key] - torch.log(me.sum(2, keepdim=True))
        hl = -lp * norm_ret.unsqueeze(-1)
        sel = torch.masked_select(hl, actions[key].bool())
        policy_loss[key] = sel
        n = sel.size(0)
        lps = torch.masked_select(lp, masks[key].bool())
        entropies[key] = torch.zeros([]) if n == 0 else -(torch.exp(lps) * lps).sum() / n
    pl = torch.cat(list(policy_loss.values())).mean()
    ent = torch.stack(list(entropies.values())).sum()
    el = -ent_coef * ent if ent_coef > 0 else torch.tensor(0.)
    al = vf_coef * advantage.pow(2).mean() if vf_coef > 0 else torch.tensor(0.)
    return pl + el + al


def test_vpg_loss_matches_reference_formula_including_value_bug():
    torch.manual_seed(0)
    b = make_batch(3, 20, LAYOUT_1V1, None, pad_frac=0.0, seed=5)
    counts = LAYOUT_1V1.action_counts()
    logits = {k: torch.randn(3, 20, n, requires_grad=True) for k, n in counts.items()}
    values = torch.randn(3, 20, 1, requires_grad=True)
    actions, masks = split_heads(b['actions'], counts), split_heads(b['masks'], counts)
    ref = _reference_vpg(logits, values, actions, masks, b['norm_ret'], b['ret'], 0.01, 0.5)
    ours, _ = vpg_loss(logits, values, actions, masks, b['norm_ret'], b['ret'], 0.01, 0.5, compat_value_bug=True,
                       stable=False)
    torch.testing.assert_close(ours, ref, rtol=1e-5, atol=1e-6)
    g1 = torch.autograd.grad(ref, list(logits.values()) + [values])
    g2 = torch.autograd.grad(ours, list(logits.values()) + [values])
    for a, c in zip(g1, g2):
        torch.testing.assert_close(a, c, rtol=1e-4, atol=1e-6)


def test_ppo_loss_against_manual():
    torch.manual_seed(1)
    b = make_batch(2, 16, LAYOUT_1V1, None, pad_frac=0.3, seed=2)
    counts = LAYOUT_1V1.action_counts()
    logits = {k: torch.randn(2, 16, n) for k, n in counts.items()}
    values = torch.randn(2, 16, 1)
    actions, masks = split_heads(b['actions'], counts), split_heads(b['masks'], counts)
    loss, m = ppo_loss(logits, values, actions, masks, b['adv'], b['ret'], b['logp_old'], 0.1, 0.0, 1.0)
    logp = sum((masked_log_softmax(logits[k], masks[k]) * actions[k]).sum(-1) for k in counts)
    valid = b['actions'].sum(-1) > 0
    r = torch.exp(logp - b['logp_old'])
    s = torch.minimum(r * b['adv'], r.clamp(0.9, 1.1) * b['adv'])[valid]
    vl = ((values.squeeze(-1) - b['ret']) ** 2)[valid].mean()
    torch.testing.assert_close(loss, -s.mean() + vl, rtol=1e-5, atol=1e-6)
    assert 0.0 <= float(m['clipfrac']) <= 1.0
