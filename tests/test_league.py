"""Opponent league (actor/league.py) and its use by the Actor (reference mini-league agent.py:760-765)."""
import random

import pytest
import torch

from dotaclient_amd.actor.league import League
from dotaclient_amd.actor.weights import WeightStore
from dotaclient_amd.models.policy import Policy


def _store(n, cfg='compat'):
    ws = WeightStore(cfg, maxlen=64)
    base = Policy(cfg).state_dict()
    for v in range(n):
        g = torch.Generator().manual_seed(v)
        ws.add(v, {k: t + 1e-3 * torch.randn(t.shape, generator=g) for k, t in base.items()})
    return ws


def test_oldest_mode_is_reference_behaviour():
    ws = _store(5)
    lg = League(ws, mode='oldest', rng=random.Random(0))
    assert all(lg.sample()[0] == 0 for _ in range(20))


def test_uniform_and_recent_distributions():
    ws = _store(4)
    lg = League(ws, mode='uniform', rng=random.Random(1))
    counts = [0] * 4
    for _ in range(8000):
        counts[lg.sample()[0]] += 1
    assert all(abs(c / 8000 - 0.25) < 0.03 for c in counts)
    lg = League(ws, mode='recent', decay=0.5, rng=random.Random(2))
    w = lg.weights()
    assert w == [0.125, 0.25, 0.5, 1.0]


def test_pfsp_prefers_opponents_the_learner_loses_to():
    ws = _store(3)
    lg = League(ws, mode='pfsp', rng=random.Random(3))
    for _ in range(20):
        lg.record(0, 1.0)      # learner always beats snapshot 0
        lg.record(2, 0.0)      # and always loses to snapshot 2
    w = lg.weights()
    assert w[2] > w[1] > w[0]
    assert lg.win_rate(0) > 0.9 and lg.win_rate(2) < 0.1


def test_policy_cache_reuses_snapshot_policies():
    ws = _store(3)
    lg = League(ws, mode='uniform', cache_size=2)
    a = lg.policy(ws.weights[0])
    assert lg.policy(ws.weights[0]) is a
    lg.policy(ws.weights[1])
    lg.policy(ws.weights[2])
    assert lg.policy(ws.weights[0]) is not a       # evicted (LRU of 2)
    torch.testing.assert_close(a.affine_env.bias, ws.weights[0][1]['affine_env.bias'])


def test_actor_plays_league_opponents_and_records_results():
    from dotaclient_amd.actor.game import Actor
    from dotaclient_amd.actor.runner import PolicyRunner
    from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config
    ws = _store(3, 'compat')
    lg = League(ws, mode='uniform', rng=random.Random(4))
    runners = {}
    sent = []
    actor = Actor([SyntheticDotaService(seed=s) for s in range(2)], ws,
                  lambda p: runners.setdefault(id(p), PolicyRunner(p, seed=0)), sent.append,
                  get_1v1_selfplay_config, max_dota_time=20, latest_weights_prob=0.0, rng=random.Random(5),
                  league=lg)
    while actor.games_finished < 4:
        actor.step()
    assert sum(lg.games.values()) >= 4
    assert set(lg.games) <= {0, 1, 2}
