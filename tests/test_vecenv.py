"""Native vectorised runtime (native/vecenv.h) vs its python oracle.

* ``SimGame`` (the C++ engine) vs ``env/synthetic.py:SyntheticGame``: same seed, same random orders — every unit's
  position / hp / target and every featurized observation (both teams) and shaped reward bit-identical, step by step.
* ``VecEnv`` (engine + featurize + reward + canvas + trajectory recording + action decode + DCX1 rollouts) vs the
  reference-semantics python :class:`~dotaclient_amd.actor.game.Actor` driving ``SyntheticDotaService`` games: fed
  the same per-observation policy outputs, both publish identical rollouts (every array, byte for byte).
"""
import hashlib

import numpy as np
import pytest

from dotaclient_amd import native
from dotaclient_amd.constants import LAYOUT_1V1, MOVE_ENUMS
from dotaclient_amd.env.configs import get_1v1_selfplay_config
from dotaclient_amd.env.synthetic import SyntheticDotaService, SyntheticGame
from dotaclient_amd.features.actions import action_to_pb
from dotaclient_amd.features.featurizer import featurize, get_unit
from dotaclient_amd.features.reward import get_reward
from dotaclient_amd.protos import TEAM_DIRE, TEAM_RADIANT, pb
from dotaclient_amd.transport.codec import decode

pytestmark = pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')
N = native._native if native.AVAILABLE else None
COUNTS = list(LAYOUT_1V1.counts)
REWARD_KEYS = ['enemy', 'win', 'xp', 'hp', 'kills', 'death', 'lh', 'denies', 'tower_hp']


def _picks(cfg):
    return [(p.team_id, p.hero_id, p.control_mode) for p in cfg.hero_picks]


@pytest.mark.parametrize('seed', [3, 11, 2 ** 33 + 5])
def test_simgame_matches_python_engine_step_by_step(seed):
    cfg = get_1v1_selfplay_config()
    py = SyntheticGame(cfg, seed=seed)
    cc = N.SimGame(_picks(cfg), seed)
    rng = np.random.default_rng(seed)
    prev_ws = {t: py.world_state(t) for t in (TEAM_RADIANT, TEAM_DIRE)}
    for t in (TEAM_RADIANT, TEAM_DIRE):
        cc.reward(0 if t == TEAM_RADIANT else 5, t)        # prime the reward views
    for step in range(700):
        assert cc.dota_time == py.dota_time and cc.status == py.status, step
        got = cc.units()
        want = [(u.handle, u.unit_type, u.team_id, u.x, u.y, u.hp, u.alive, u.target) for u in py.units.values()]
        assert got == want, step
        acts = {}
        for team, pid in ((TEAM_RADIANT, 0), (TEAM_DIRE, 5)):
            ws = py.world_state(team)
            f = featurize(ws, pid, team, layout=LAYOUT_1V1, hero_unit=get_unit(ws, pid))
            env, units, handles = cc.featurize(team, pid, COUNTS)
            np.testing.assert_array_equal(env, f.env)
            np.testing.assert_array_equal(units, f.units)
            np.testing.assert_array_equal(handles, f.handles)
            r = get_reward(prev_ws[team], ws, pid)
            np.testing.assert_array_equal(cc.reward(pid, team), [r[k] for k in REWARD_KEYS])
            prev_ws[team] = ws
            hero = get_unit(ws, pid)
            e = int(rng.integers(3))
            valid = np.flatnonzero(f.handles >= 0)
            if e == 2 and len(valid) == 0:
                e = 1
            d = {'enum': e, 'x': int(rng.integers(9)), 'y': int(rng.integers(9))}
            if e == 2:
                d['target_unit'] = int(rng.choice(valid))
            a = action_to_pb(d, hero.location, f.handles, player_id=pid)
            acts[team] = [a]
        orders = []
        for team in (TEAM_RADIANT, TEAM_DIRE):
            a = acts[team][0]
            typ = {0: 0, 2: 1, 4: 2}.get(a.actionType, 0) if False else (
                1 if a.HasField('moveDirectly') else (2 if a.HasField('attackTarget') else 0))
            orders.append((a.player, typ, a.moveDirectly.location.x, a.moveDirectly.location.y,
                           a.attackTarget.target if typ == 2 else -1))
        py.step(acts)
        cc.step(orders)
        if py.status != 0:
            break


def _policy_out(env, units, handles, A, U):
    """A deterministic 'policy': indices and behaviour data as a hash of the observation (identical inputs →
    identical outputs on both runtimes)."""
    h = hashlib.sha256(env.tobytes() + units.tobytes() + handles.tobytes()).digest()
    e = h[0] % 3
    valid = np.flatnonzero(handles >= 0)
    if e == 2 and len(valid) == 0:
        e = 1
    x, y = h[1] % 9, h[2] % 9
    tgt = int(valid[h[3] % len(valid)]) if e == 2 else 0
    idx = np.array([e, x, y, tgt], np.int32)
    act = np.zeros(A, np.uint8)
    msk = np.zeros(A, np.uint8)
    act[e] = 1
    msk[:3] = 1
    if e == 1:
        act[3 + x] = 1
        act[12 + y] = 1
        msk[3:21] = 1
    elif e == 2:
        act[21 + tgt] = 1
        msk[21:21 + U] = 1
    logp = np.float32(-(h[4] / 64.0))
    value = np.float32((h[5] - 128) / 100.0)
    return idx, act, msk, logp, value


class _Out:
    def __init__(self, rows):
        self.idx = np.stack([r[0] for r in rows])
        self.actions = np.stack([r[1] for r in rows])
        self.masks = np.stack([r[2] for r in rows])
        self.logp = np.array([r[3] for r in rows], np.float32)
        self.value = np.array([r[4] for r in rows], np.float32)

    def action_dict(self, j):
        e, x, y, t = (int(v) for v in self.idx[j])
        d = {'enum': e}
        if e == 1:
            d.update(x=x, y=y)
        elif e == 2:
            d['target_unit'] = t
        return d


class _Runner:
    stateful = False

    def step(self, env, units, handles, hidden):
        U = units.shape[1]
        return _Out([_policy_out(env[i], units[i], handles[i], 21 + U, U) for i in range(len(env))]), None


class _Policy:
    is_recurrent = False
    weight_version = 7


class _Store:
    latest_policy = _Policy()


@pytest.mark.parametrize('seed,rollout_size', [(17, 10 ** 9), (4, 50), (23, 10 ** 9)])
def test_vecenv_rollouts_equal_python_actor(seed, rollout_size):
    """One game on each runtime (the python Actor's service seeded like VecEnv's first game: seed·1000003 + 1)."""
    from dotaclient_amd.actor.game import Actor
    max_t = 140.0
    sent = []
    actor = Actor([SyntheticDotaService(seed=seed * 1000003 + 1)], _Store(), lambda pol: _Runner(), sent.append,
                  get_1v1_selfplay_config, rollout_size=rollout_size, max_dota_time=max_t, layout=LAYOUT_1V1)
    while actor.games_finished < 1:
        actor.step()
    want = {}
    for b in sent:
        r = decode(b)
        want.setdefault((r.team_id, r.player_id), []).append(r)

    ve = N.VecEnv(1, mode=0, seed=seed, max_dota_time=max_t, rollout_size=rollout_size, counts=COUNTS, threads=2)
    S, U = ve.slots, sum(COUNTS)
    env = np.zeros((S, 3), np.float32)
    units = np.zeros((S, U, 10), np.float32)
    handles = np.zeros((S, U), np.int64)
    active = np.zeros(S, np.uint8)
    got = {}
    while ve.games_finished < 1:
        ve.begin_step()
        ve.observe(env, units, handles, active)
        o = _Out([_policy_out(env[i], units[i], handles[i], 21 + U, U) for i in range(S)])
        ve.act(o.idx, o.actions, o.masks, o.logp, o.value, None, None, handles, 7)
        for b in ve.pop_rollouts():
            r = decode(b)
            got.setdefault((r.team_id, r.player_id), []).append(r)
    assert set(got) == set(want) == {(2, 0), (3, 5)}
    for key in want:
        assert len(got[key]) == len(want[key]), key
        for rw, rg in zip(want[key], got[key]):
            for k in ('env', 'units', 'actions', 'masks', 'rewards', 'logp', 'values', 'canvas'):
                np.testing.assert_array_equal(getattr(rg, k), getattr(rw, k), err_msg=f'{key} {k}')
            assert (rg.done, rg.weight_version, rg.bootstrap_value) == (rw.done, rw.weight_version, rw.bootstrap_value)


@pytest.mark.parametrize('seed', [5, 29])
def test_actor_native_featurize_rollouts_identical(seed):
    """The protobuf Actor with the native batched featurizer (one C++ call per team-turn) publishes exactly the
    rollouts of the python-featurizer Actor."""
    from dotaclient_amd.actor.game import Actor
    out = {}
    for nat in (False, True):
        sent = []
        actor = Actor([SyntheticDotaService(seed=seed + i) for i in range(3)], _Store(), lambda pol: _Runner(),
                      sent.append, get_1v1_selfplay_config, rollout_size=40, max_dota_time=60.0, layout=LAYOUT_1V1,
                      native_featurize=nat)
        while actor.games_finished < 3:
            actor.step()
        out[nat] = [decode(b) for b in sent]
    assert len(out[True]) == len(out[False]) > 0
    for a, b in zip(out[False], out[True]):
        for k in ('env', 'units', 'actions', 'masks', 'rewards', 'logp', 'values', 'canvas'):
            np.testing.assert_array_equal(getattr(a, k), getattr(b, k), err_msg=k)


@pytest.mark.parametrize('seed', [3, 2 ** 33 + 5])
def test_simgame_world_bytes_equal_python_protobuf(seed):
    """The engine's serialised CMsgBotWorldState (the observation the reference actor receives from
    DotaService.observe, agent.py:805-810) is byte-identical to python protobuf's SerializeToString of the oracle's
    world_state, for both teams' views (fog included), every step."""
    cfg = get_1v1_selfplay_config()
    py = SyntheticGame(cfg, seed=seed)
    cc = N.SimGame(_picks(cfg), seed)
    rng = np.random.default_rng(seed)
    for step in range(400):
        for team in (TEAM_RADIANT, TEAM_DIRE):
            want = py.world_state(team).SerializeToString()
            got = cc.world_bytes(team)
            assert got == want, (step, team)
        acts, orders = {}, []
        for team, pid in ((TEAM_RADIANT, 0), (TEAM_DIRE, 5)):
            hero = get_unit(py.world_state(team), pid)
            mx, my = hero.location.x + 68.75 * int(rng.integers(-4, 5)), hero.location.y + 68.75 * int(rng.integers(-4, 5))
            a = pb.CMsgBotWorldState.Action(actionType=pb.CMsgBotWorldState.Action.DOTA_UNIT_ORDER_MOVE_DIRECTLY,
                                            player=pid)
            a.moveDirectly.location.x, a.moveDirectly.location.y = mx, my
            acts[team] = [a]
            orders.append((pid, 1, a.moveDirectly.location.x, a.moveDirectly.location.y, -1))
        py.step(acts)
        cc.step(orders)
        if py.status != 0:
            break


@pytest.mark.parametrize('mode', ['1v1', '5v5'])
def test_vecenv_wire_observations_identical(mode):
    """VecEnv(wire=True) — observations serialised to protobuf and featurized by the wire decoder, the reference
    actor's path — yields exactly the struct path's observations and rollouts."""
    from dotaclient_amd.constants import LAYOUT_5V5
    lay = LAYOUT_1V1 if mode == '1v1' else LAYOUT_5V5
    m = 0 if mode == '1v1' else 1
    envs = [N.VecEnv(6, mode=m, seed=9, max_dota_time=40.0, counts=list(lay.counts), threads=2, wire=w,
                     rollout_size=37) for w in (False, True)]
    S, U = envs[0].slots, lay.max_units
    rng = np.random.default_rng(0)
    out = []
    for ve in envs:
        out.append([])
        r = np.random.default_rng(0)
        for step in range(120):
            ve.begin_step()
            env = np.zeros((S, 3), np.float32)
            units = np.zeros((S, U, 10), np.float32)
            handles = np.zeros((S, U), np.int64)
            active = np.zeros(S, np.uint8)
            ve.observe(env, units, handles, active)
            out[-1].append((env.copy(), units.copy(), handles.copy(), active.copy()))
            idx = np.zeros((S, 4), np.int32)
            idx[:, 0] = r.integers(0, 3, S)                   # none / move / attack (orders via Actions protobufs)
            idx[:, 1] = r.integers(0, 9, S)
            idx[:, 2] = r.integers(0, 9, S)
            idx[:, 3] = r.integers(0, U, S)
            A = 21 + U
            ve.act(idx, np.zeros((S, A), np.uint8), np.zeros((S, A), np.uint8), np.zeros(S, np.float32),
                   np.zeros(S, np.float32), None, None, handles, 0)
            out[-1].append(tuple(sorted(ve.pop_rollouts())))      # (pool threads emit in any order)
    assert envs[1].wire_bytes > 0 and envs[0].wire_bytes == 0
    for a, b in zip(out[0], out[1]):
        for x, y in zip(a, b):
            if isinstance(x, np.ndarray):
                np.testing.assert_array_equal(x, y)
            else:
                assert x == y
    del rng
