"""VecActor orchestration (actor/vec.py) on CPU: the native VecEnv + TorchSlotPolicy (GpuActorPolicy's interface).

The decisive check is *replay consistency*: every published rollout is re-run through the eager policy from its
first stored LSTM state — the stored states at every ``hidden_stride`` step, the recorded ``values`` and the
``logp`` of the recorded actions under the recorded masks must all match what the actor had. That pins the slot
bookkeeping (resets, active masks, group pipelining, hidden snapshots, truncated rollouts) end to end.
"""
import numpy as np
import pytest
import torch

from dotaclient_amd import native
from dotaclient_amd.actor.weights import WeightStore
from dotaclient_amd.models.policy import Policy, get_config, masked_log_softmax
from dotaclient_amd.transport.codec import decode

pytestmark = pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')

HEADS = [('enum', 0, 3), ('x', 3, 9), ('y', 12, 9)]


def _store(cfg, versions=(0,), seed=0):
    ws = WeightStore(cfg, device='cpu')
    for v in versions:
        torch.manual_seed(seed + v)
        ws.add(v, {k: t.detach().clone() for k, t in Policy(cfg).state_dict().items()})
    return ws


def _replay(policy, r, stride):
    """Re-run a rollout; returns (hidden states at the stride points, values, logp of the recorded actions).
    (A GPU actor's rollouts carry raw unit records: featurized here by the kernel's numpy oracle.)"""
    r.ensure_units()
    U = r.units.shape[1]
    heads = HEADS + [('target_unit', 21, U)]
    h = (torch.from_numpy(r.hiddens[0, 0].copy())[None, None], torch.from_numpy(r.hiddens[0, 1].copy())[None, None])
    hs, vals, lps = [], [], []
    with torch.no_grad():
        for t in range(r.length):
            if t % stride == 0:
                hs.append(np.stack([h[0][0, 0].numpy(), h[1][0, 0].numpy()]))
            logits, value, h = policy.forward_packed(torch.from_numpy(r.env[t:t + 1].copy())[None],
                                                     torch.from_numpy(r.units[t:t + 1].copy())[None], h)
            vals.append(float(value[0, 0, 0]))
            lp = 0.0
            for k, o, w in heads:
                m = torch.from_numpy(r.masks[t, o:o + w].astype(bool))
                if not m.any():
                    continue
                a = int(np.argmax(r.actions[t, o:o + w]))
                lp += float(masked_log_softmax(logits[k].reshape(1, w).float(), m[None], dim=-1)[0, a])
            lps.append(lp)
    return np.stack(hs), np.array(vals, np.float32), np.array(lps, np.float32)


@pytest.mark.parametrize('groups', [1, 2])
def test_vec_actor_rollouts_replay_consistent(groups):
    from dotaclient_amd.actor.vec import VecActor
    cfg = get_config('lstm128')
    ws = _store(cfg)
    sent = []
    stride = 8
    va = VecActor(ws, 3, sent.append, device='cpu', seed=5, rollout_size=24, max_dota_time=25.0,
                  hidden_stride=stride, threads=2, groups=groups)
    while va.games_finished < 4:
        va.step()
    assert va.rollouts_sent == len(sent) > 0
    rs = [decode(b) for b in sent]
    pol = ws.policy_for(ws.latest_weights())
    per_player = {}
    for r in rs:
        assert r.hiddens.shape == (-(-r.length // stride), 2, 128)
        assert r.weight_version == 0 and r.hidden_stride == stride
        hs, vals, lps = _replay(pol, r, stride)
        np.testing.assert_allclose(hs, r.hiddens, atol=2e-5)
        np.testing.assert_allclose(vals, r.values, atol=2e-5)
        np.testing.assert_allclose(lps, r.logp, atol=5e-4)
        per_player.setdefault((r.game_id, r.team_id, r.player_id), []).append(r)
    for key, lst in per_player.items():
        assert lst[-1].done and not any(r.done for r in lst[:-1]), key
        assert not np.any(lst[0].hiddens[0]), key                  # a game starts from the zero state
        assert all(r.length == 24 for r in lst[:-1]), key
    assert va.steps_taken >= sum(r.length for r in rs)


def test_vec_actor_ring_sink_encodes_into_the_ring():
    """VecActor(ring_sink=ShmBroker): the engine's worker threads encode finished rollouts straight into reserved ring
    regions (native/vecenv.h dcx2_write, per-block CRC) — the same messages the publish path produces: they decode
    with a valid CRC-32C, replay-consistent, counted in rollouts_sent, none through ``publish``."""
    import uuid
    from dotaclient_amd.actor.vec import VecActor
    from dotaclient_amd.transport.shm import ShmBroker
    cfg = get_config('lstm128')
    ws = _store(cfg)
    b = ShmBroker(f'dca_sink_{uuid.uuid4().hex[:8]}', capacity=1 << 26, create=True, drop_oldest=True)
    try:
        sent = []
        stride = 8
        va = VecActor(ws, 3, sent.append, device='cpu', seed=5, rollout_size=24, max_dota_time=25.0,
                      hidden_stride=stride, threads=2, groups=2, ring_sink=b)
        while va.games_finished < 4:
            va.step()
        assert not sent and va.rollouts_sent > 0 and va.sink_lost == 0
        rs = []
        while True:
            got = b.consume_experience_checked(0.0)
            if got is None:
                break
            arr, ok = got
            assert ok is True
            rs.append(decode(arr.tobytes()))
        assert len(rs) == va.rollouts_sent
        pol = ws.policy_for(ws.latest_weights())
        for r in rs[:6]:
            hs, vals, lps = _replay(pol, r, stride)
            np.testing.assert_allclose(hs, r.hiddens, atol=2e-5)
            np.testing.assert_allclose(vals, r.values, atol=2e-5)
            np.testing.assert_allclose(lps, r.logp, atol=5e-4)
    finally:
        b.close(unlink=True)


def test_vec_actor_league_opponents_and_hot_swap():
    from dotaclient_amd.actor.league import League
    from dotaclient_amd.actor.vec import VecActor
    import random
    cfg = get_config('lstm128')
    ws = _store(cfg, versions=(0, 1, 2))
    league = League(ws, mode='uniform', rng=random.Random(0))
    sent = []
    va = VecActor(ws, 4, sent.append, device='cpu', seed=9, max_dota_time=15.0, hidden_stride=8, threads=2,
                  groups=2, latest_weights_prob=0.0, league=league, opponent_refresh=2)
    while va.games_finished < 6:
        va.step()
    # every game had an opponent team: exactly one (team, player) per game rolls out
    teams = {}
    for b in sent:
        r = decode(b)
        teams.setdefault(r.game_id, set()).add(r.team_id)
    assert teams and all(len(t) == 1 for t in teams.values())
    assert sum(g for _, g in league.stats().values()) == va.opp_games_finished == va.games_finished
    # the opponents played stored snapshots and never more than two at once per group
    assert all(len(g.opp) <= 2 for g in va.groups)
    # hot swap: a new latest version reaches the games started after it, which replay exactly under it
    torch.manual_seed(99)
    ws.add(7, {k: t.detach().clone() for k, t in Policy(cfg).state_dict().items()})
    n0 = va.games_finished
    while va.games_finished < n0 + 4:      # drain the games in flight at the swap
        va.step()
    sent.clear()
    while va.games_finished < n0 + 8:
        va.step()
    rs = [decode(b) for b in sent]
    assert rs and all(r.weight_version == 7 for r in rs)
    pol = ws.policy_for(ws.latest_weights())
    for r in rs:
        _, vals, lps = _replay(pol, r, 8)
        np.testing.assert_allclose(vals, r.values, atol=2e-5)
        np.testing.assert_allclose(lps, r.logp, atol=5e-4)


@pytest.mark.gpu
@pytest.mark.parametrize('preset,mode', [('lstm512', '1v1'), ('5v5', '5v5')])
def test_vec_actor_gpu_graph_policy_replay_consistent(preset, mode):
    """The hipGraph GpuActorPolicy path (bf16 GEMMs, fused LSTM cell + sampling kernels) with league opponents:
    rollouts replay under the fp32 eager policy within bf16 tolerance (slot/state mix-ups would be O(1))."""
    import random
    from dotaclient_amd.actor.batched import GpuActorPolicy
    from dotaclient_amd.actor.league import League
    from dotaclient_amd.actor.vec import VecActor
    cfg = get_config(preset)
    ws = _store(cfg, versions=(0, 1))
    sent = []
    va = VecActor(ws, 16 if mode == '1v1' else 4, sent.append, device='cuda', seed=3, rollout_size=32,
                  max_dota_time=20.0, mode=mode, hidden_stride=16, threads=4, groups=2, latest_weights_prob=0.5,
                  league=League(ws, mode='uniform', rng=random.Random(1)))
    assert all(isinstance(g.gp, GpuActorPolicy) for g in va.groups)
    while va.games_finished < (24 if mode == '1v1' else 6):
        va.step()
    va.close()
    assert va.opp_games_finished > 0
    pol = ws.policy_for(ws.latest_weights())
    rs = [decode(b) for b in sent]
    assert len(rs) > 16
    # GPU featurization: the rollouts carry raw unit records (features/raw.py), not host features
    assert all(r.units is None and r.units_raw is not None and r.hero is not None for r in rs)
    for r in rs[:60]:
        hs, vals, lps = _replay(pol, r, 16)
        np.testing.assert_allclose(hs, r.hiddens, atol=5e-2 if mode == '1v1' else 1e-1)
        np.testing.assert_allclose(vals, r.values, atol=5e-2)
        np.testing.assert_allclose(lps, r.logp, atol=1e-1)


def test_validation_vs_default_bot_5v5_cpu():
    """The reference's validation agent (agent.py:905-927) for the 5v5 policy: five controlled heroes against five
    default-bot heroes (native engine mode 3, sides alternating with the game serial), the reference's metrics."""
    from dotaclient_amd.actor.validate import evaluate_vs_default_bot
    from dotaclient_amd.models.policy import Policy, get_config
    torch.manual_seed(0)
    out = evaluate_vs_default_bot(Policy(get_config('5v5')), n_games=4, device='cpu', seed=3, max_dota_time=20.0,
                                  threads=2, timeout=300)
    assert out['games'] == 4
    assert 0.0 <= out['game/win_rate'] <= 1.0 and out['game/steps'] > 10
    assert 'game/rewards_sum' in out and 'game/rewards_lh' in out
