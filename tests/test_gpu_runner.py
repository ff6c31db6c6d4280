"""Stateful (device-slot) policy runners in the Actor game loop (actor/gpu_runner.py).

CPU: the Actor's stateful-runner protocol (``step_players`` / ``release`` / ``need_hidden``) is checked with a
host double that wraps the stateless PolicyRunner — the experience it produces must be bit-identical to the
stateless path. GPU: GpuRunner's slot state (subset steps, fresh slots, release/reuse, capacity growth) against
the torch policy carried step by step, and whole games through the Actor.
"""
import random

import numpy as np
import pytest
import torch

from dotaclient_amd.actor.runner import PolicyRunner, RunnerCache
from dotaclient_amd.models.policy import Policy, batched_action_masks, get_config, masked_log_softmax


class _HostSlotRunner:
    """Stateful runner protocol implemented over the stateless PolicyRunner (test double)."""
    stateful = True

    def __init__(self, policy, seed):
        self.inner = PolicyRunner(policy, seed=seed)
        self.H = policy.config.hidden
        self.state = {}
        self.released = []

    def step_players(self, env, units, handles, keys, need_hidden=None):
        z = np.zeros(self.H, np.float32)
        hs = [self.state.get(k, (z, z)) for k in keys]
        out, nh = self.inner.step(env, units, handles, (np.stack([h for h, _ in hs]), np.stack([c for _, c in hs])))
        prev = {j: hs[j] for j in range(len(keys)) if need_hidden is not None and need_hidden[j]}
        for j, k in enumerate(keys):
            self.state[k] = (nh[0][j], nh[1][j])
        return out, prev

    def release(self, key):
        self.state.pop(key)
        self.released.append(key)


def _play(stateful: bool, n_games=4):
    from dotaclient_amd.actor.game import Actor
    from dotaclient_amd.actor.weights import WeightStore
    from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config
    from dotaclient_amd.transport.codec import decode
    torch.manual_seed(0)
    ws = WeightStore('lstm128')
    ws.add(0, Policy('lstm128').state_dict())
    runners = {}
    mk = (lambda p: _HostSlotRunner(p, 0)) if stateful else (lambda p: PolicyRunner(p, seed=0))
    sent = []
    actor = Actor([SyntheticDotaService(seed=s) for s in range(2)], ws,
                  lambda p: runners.setdefault(id(p), mk(p)), sent.append, get_1v1_selfplay_config,
                  rollout_size=16, max_dota_time=12, hidden_size=128, hidden_stride=5, rng=random.Random(1))
    while actor.games_finished < n_games:
        actor.step()
    return [decode(b) for b in sent], runners


def test_actor_stateful_runner_protocol_matches_stateless():
    a, _ = _play(False)
    b, runners = _play(True)
    assert len(a) == len(b) > 4
    for ra, rb in zip(a, b):
        assert (ra.player_id, ra.team_id) == (rb.player_id, rb.team_id)
        np.testing.assert_array_equal(ra.actions, rb.actions)
        np.testing.assert_array_equal(ra.logp, rb.logp)
        assert ra.hiddens is not None and rb.hiddens is not None
        np.testing.assert_array_equal(ra.hiddens, rb.hiddens)
    r = next(iter(runners.values()))
    assert len(r.released) >= 8            # 4 finished games × 2 players, slots handed back


def test_runner_cache_shares_runners_by_version():
    made = []
    latest = Policy('compat')
    cache = RunnerCache(lambda p: made.append(p) or len(made), latest_policy=latest, max_snapshots=2)
    assert cache(latest) == cache(latest) == 1
    snaps = []
    for v in (3, 3, 4, 5, 3):
        p = Policy('compat')
        p.weight_version = v
        snaps.append(cache(p))
    assert snaps[0] == snaps[1] == 2          # two objects of version 3 share one runner
    assert snaps[4] not in snaps[:2]           # version 3 was evicted (LRU of 2) and rebuilt
    assert len(cache.runners()) == 3


# ---------------------------------------------------------------------------------------------------------
def _ref_logp(pol, env, units, handles, hidden, out):
    n, U = handles.shape[0], pol.config.layout.max_units
    with torch.no_grad():
        logits, value, hn = pol.forward_packed(torch.as_tensor(env, device='cuda')[:, None],
                                               torch.as_tensor(units, device='cuda')[:, None], hidden)
        valid = batched_action_masks(torch.as_tensor(handles, device='cuda'))
        lps = {k: masked_log_softmax(logits[k][:, 0].reshape(n, -1).float(), valid[:, o:o + w], dim=-1)
               for k, o, w in (('enum', 0, 3), ('x', 3, 9), ('y', 12, 9), ('target_unit', 21, U))}
    r = torch.arange(n, device='cuda')
    e, x, y, t = (torch.as_tensor(v, device='cuda') for v in (out.enum, out.x, out.y, out.target))
    mv, att = e == 1, e == 2
    lp = lps['enum'][r, e] + mv * (lps['x'][r, x] + lps['y'][r, y]) + torch.where(att, lps['target_unit'][r, t], 0.)
    return lp, value[:, 0, 0].float(), hn


@pytest.mark.gpu
@pytest.mark.parametrize('preset', ['lstm128', 'lstm512'])
def test_gpu_runner_slot_state(gpu_ops, preset):
    """Alternating subsets (teams) share one graph; untouched slots keep their state; fresh and reused slots start
    from zero; capacity grows with the state carried over; need_hidden returns the pre-step state."""
    from dotaclient_amd.actor.gpu_runner import GpuRunner
    torch.manual_seed(11)
    cfg = get_config(preset)
    pol = Policy(cfg).cuda().eval()
    H, U = cfg.hidden, cfg.layout.max_units
    run = GpuRunner(pol, device='cuda', seed=3, capacity=4)
    rng = np.random.default_rng(0)
    state = {}

    def feats(n):
        env = rng.standard_normal((n, 3)).astype(np.float32)
        units = rng.standard_normal((n, U, 10)).astype(np.float32)
        handles = np.where(rng.random((n, U)) < 0.5, rng.integers(1, 999, (n, U)), -1).astype(np.int64)
        return env, units, handles

    teams = [['a0', 'a1', 'a2'], ['b0', 'b1', 'b2']]
    for step in range(6):
        for ti, keys in enumerate(teams):
            if step == 3 and ti == 0:
                run.release('a1')
                state.pop('a1')
                keys[1] = 'a9'                          # reuses a1's slot → must start from zero
            if step == 4 and ti == 1:
                keys.extend(['b3', 'b4', 'b5', 'b6'])   # 10 players > capacity 8 → growth
            env, units, handles = feats(len(keys))
            z = torch.zeros(len(keys), H, device='cuda')
            h0 = torch.stack([state[k][0] if k in state else z[0] for k in keys])
            c0 = torch.stack([state[k][1] if k in state else z[0] for k in keys])
            need = [True] * len(keys)
            out, prev = run.step_players(env, units, handles, keys, need)
            for j, k in enumerate(keys):
                torch.testing.assert_close(torch.as_tensor(prev[j][0], device='cuda'), h0[j], atol=2e-2, rtol=0)
            lp, v, hn = _ref_logp(pol, env, units, handles, (h0[None], c0[None]), out)
            assert (torch.as_tensor(out.logp, device='cuda') - lp).abs().max() < 5e-2, (step, ti)
            assert (torch.as_tensor(out.value, device='cuda') - v).abs().max() < 2e-2 + 2e-2 * v.abs().max()
            for j, k in enumerate(keys):
                state[k] = (hn[0][0, j], hn[1][0, j])
    assert run.capacity >= 10 and len(run) == 10


@pytest.mark.gpu
def test_gpu_runner_stateless_step_matches_policy(gpu_ops):
    from dotaclient_amd.actor.gpu_runner import GpuRunner
    torch.manual_seed(12)
    pol = Policy(get_config('lstm512')).cuda().eval()
    run = GpuRunner(pol, device='cuda', seed=4, capacity=8)
    U, H, n = pol.config.layout.max_units, pol.config.hidden, 5
    rng = np.random.default_rng(1)
    hidden = (np.zeros((n, H), np.float32), np.zeros((n, H), np.float32))
    for _ in range(3):
        env = rng.standard_normal((n, 3)).astype(np.float32)
        units = rng.standard_normal((n, U, 10)).astype(np.float32)
        handles = np.where(rng.random((n, U)) < 0.5, rng.integers(1, 999, (n, U)), -1).astype(np.int64)
        hd = tuple(torch.as_tensor(x, device='cuda')[None] for x in hidden)
        out, hidden = run.step(env, units, handles, hidden)
        lp, v, hn = _ref_logp(pol, env, units, handles, hd, out)
        assert (torch.as_tensor(out.logp, device='cuda') - lp).abs().max() < 5e-2
        torch.testing.assert_close(torch.as_tensor(hidden[0], device='cuda'), hn[0][0], atol=2e-2, rtol=0)
    assert len(run) == 0


@pytest.mark.gpu
@pytest.mark.parametrize('preset', ['compat', 'lstm512'])
def test_actor_plays_games_on_gpu_runner(gpu_ops, preset):
    from dotaclient_amd.actor.game import Actor
    from dotaclient_amd.actor.gpu_runner import GpuRunner
    from dotaclient_amd.actor.weights import WeightStore
    from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config
    from dotaclient_amd.transport.codec import decode
    cfg = get_config(preset)
    ws = WeightStore(preset)
    ws.add(0, Policy(cfg).state_dict())
    cache = RunnerCache(lambda p: GpuRunner(p.cuda(), device='cuda', seed=1, capacity=4),
                        latest_policy=ws.latest_policy)
    sent = []
    lstm = cfg.rnn == 'lstm'
    actor = Actor([SyntheticDotaService(seed=s) for s in range(3)], ws, cache, sent.append, get_1v1_selfplay_config, rollout_size=32, max_dota_time=15,
                  hidden_size=cfg.hidden if lstm else None, hidden_stride=8, rng=random.Random(2),
                  latest_weights_prob=0.5)
    while actor.games_finished < 5:
        actor.step()
    ws.add(1, Policy(cfg).state_dict())              # hot-swap: next step loads the new weights in place
    actor.step()
    assert cache.latest._version == 1
    rs = [decode(b) for b in sent]
    assert rs and all(np.isfinite(r.logp).all() and np.isfinite(r.values).all() for r in rs)
    assert all((r.logp <= 1e-5).all() for r in rs)
    if lstm:
        assert all(r.hiddens is not None and r.hiddens.shape[1:] == (2, cfg.hidden) for r in rs)
    live = sum(len(p) for s in actor.slots if s is not None for p in s.players.values())
    assert sum(len(r) for r in cache.runners()) <= live
