"""Synthetic DotaService + featurizer + reward + action decoding against hand-built protobufs
(reference agent.py:118-158, 456-709)."""
import math

import numpy as np
import pytest

from dotaclient_amd.constants import LAYOUT_1V1, LAYOUT_5V5, MOVE_ENUMS, TEAM_DIRE, TEAM_RADIANT
from dotaclient_amd.env import SyntheticDotaService, get_1v1_bot_vs_default_config, get_1v1_selfplay_config
from dotaclient_amd.features.actions import action_to_pb
from dotaclient_amd.features.featurizer import featurize, unit_matrix, unit_separation
from dotaclient_amd.features.reward import end_state_reward, get_reward, pack_rewards
from dotaclient_amd.protos import ActionType, Status, UnitType, pb


def _ws(dota_time=10.0):
    ws = pb.CMsgBotWorldState(dota_time=dota_time)
    ws.players.add(player_id=0, team_id=TEAM_RADIANT, kills=0, deaths=0)
    ws.players.add(player_id=5, team_id=TEAM_DIRE, kills=0, deaths=0)

    def unit(**kw):
        loc = kw.pop('loc', (0.0, 0.0, 0.0))
        u = ws.units.add(**kw)
        u.location.x, u.location.y, u.location.z = loc
        return u
    me = unit(handle=1, unit_type=UnitType.HERO, team_id=TEAM_RADIANT, player_id=0, is_alive=True, health=500,
              health_max=600, level=2, xp_needed_to_level=100, attack_range=500, facing=90.0, loc=(100., 200., 256.),
              last_hits=3, denies=1)
    unit(handle=2, unit_type=UnitType.HERO, team_id=TEAM_DIRE, player_id=5, is_alive=True, health=600, health_max=600,
         level=1, attack_range=500, attack_target_handle=1, loc=(400., 200., 256.))
    unit(handle=3, unit_type=UnitType.LANE_CREEP, team_id=TEAM_RADIANT, is_alive=True, health=200, health_max=550,
         loc=(150., 200., 256.))
    unit(handle=4, unit_type=UnitType.LANE_CREEP, team_id=TEAM_RADIANT, is_alive=True, health=500, health_max=550,
         loc=(160., 200., 256.))
    unit(handle=5, unit_type=UnitType.LANE_CREEP, team_id=TEAM_DIRE, is_alive=False, health=0, health_max=550)
    t = unit(handle=6, unit_type=UnitType.TOWER, team_id=TEAM_DIRE, name='npc_dota_badguys_tower1_mid', is_alive=True,
             health=1800, health_max=1800, anim_activity=1500, loc=(524., 652., 256.))
    unit(handle=7, unit_type=UnitType.TOWER, team_id=TEAM_RADIANT, name='npc_dota_goodguys_tower1_mid',
         is_alive=True, health=1800, health_max=1800, loc=(-1544., -1408., 256.))
    unit(handle=8, unit_type=UnitType.TOWER, team_id=TEAM_RADIANT, name='npc_dota_goodguys_tower2_mid',
         is_alive=True, health=1800, health_max=1800)
    ws.units[1].incoming_tracking_projectiles.add(caster_handle=1, is_attack=True)
    return ws, me


def test_unit_matrix_features_and_handles():
    ws, me = _ws()
    sep = unit_separation(ws, TEAM_RADIANT)
    assert len(sep.allied_heroes) == 1 and len(sep.enemy_heroes) == 1 and len(sep.allied_creep) == 2
    assert len(sep.allied_towers) == 1 and len(sep.enemy_towers) == 1   # tier-2 ignored (agent.py:479)
    m, h = unit_matrix(sep.enemy_heroes, me, max_units=5)
    d = 300.0
    expect = [0.0, 400 / 7000, 200 / 7000, 0.0, d / 7000 - 0.5, 0.0, 1.0, 0.5, 0.5, 0.5]
    np.testing.assert_allclose(m[0], expect, atol=1e-6)
    assert h[0] == 2 and (h[1:] == -1).all()
    m, h = unit_matrix(sep.allied_creep, me, max_units=16)
    assert h[0] == 3            # low-hp allied creep is deniable
    assert h[1] == -1           # > 50 % hp: not deniable
    _, h = unit_matrix(sep.enemy_towers, me, max_units=1)
    assert h[0] == -1           # idle enemy tower (anim 1500) is not attackable
    _, h = unit_matrix(sep.allied_towers, me, max_units=1)
    assert h[0] == -1           # own tower


def test_featurize_layout_env_and_self_slot():
    ws, me = _ws(dota_time=30.0)
    f = featurize(ws, player_id=0, team_id=TEAM_RADIANT)
    assert f.units.shape == (40, 10) and f.handles.shape == (40,)
    np.testing.assert_allclose(f.env, [30 / 1200, math.sin(math.pi), 0.2], atol=1e-6)
    assert f.handles[0] == -1                     # self: an ally above 50 % hp is "not deniable" (agent.py:555)
    assert f.units[6, 0] == pytest.approx(1 - 200 / 550)   # first allied non-hero = creep 3
    for k, v in f.inputs.items():
        assert v.shape[0] == (3 if k == 'env' else dict(zip(['allied_heroes', 'enemy_heroes', 'allied_nonheroes',
                                                             'enemy_nonheroes', 'allied_towers', 'enemy_towers'],
                                                            LAYOUT_1V1.counts))[k])


def test_reward_terms():
    a, _ = _ws()
    b, _ = _ws()
    me = b.units[0]
    me.health = 300
    me.last_hits = 5
    me.denies = 2
    me.xp_needed_to_level = 50
    b.players[0].kills = 1
    b.units[6 + 0].health = 1800
    tower = [u for u in b.units if u.name == 'npc_dota_goodguys_tower1_mid'][0]
    tower.health = 1700
    r = get_reward(a, b, player_id=0)
    hp_rel = 300 / 600
    assert r['hp'] == pytest.approx((hp_rel - 500 / 600) * (1 + (1 - hp_rel) ** 2) * 0.2)
    assert r['xp'] == pytest.approx(50 * 0.001)
    assert r['kills'] == pytest.approx(0.4) and r['death'] == 0
    assert r['lh'] == pytest.approx(0.2) and r['denies'] == pytest.approx(0.05)
    assert r['tower_hp'] == pytest.approx(-100 / 1900)
    assert end_state_reward(Status.RADIANT_WIN, TEAM_RADIANT) == 1.0
    assert end_state_reward(Status.RADIANT_WIN, TEAM_DIRE) == -1.0
    assert end_state_reward(None, TEAM_DIRE) == -0.25
    assert pack_rewards([r]).shape == (1, 9)


def test_action_to_pb():
    ws, me = _ws()
    handles = np.arange(40) + 100
    a = action_to_pb({'enum': 1, 'x': 0, 'y': 8}, me.location, handles, player_id=0)
    assert a.actionType == ActionType.DOTA_UNIT_ORDER_MOVE_DIRECTLY
    assert a.moveDirectly.location.x == pytest.approx(100 + MOVE_ENUMS[0])
    assert a.moveDirectly.location.y == pytest.approx(200 + MOVE_ENUMS[8])
    a = action_to_pb({'enum': 2, 'target_unit': 7}, me.location, handles)
    assert a.actionType == ActionType.DOTA_UNIT_ORDER_ATTACK_TARGET and a.attackTarget.target == 107
    assert a.attackTarget.once
    assert action_to_pb({'enum': 0}, me.location, handles).actionType == ActionType.DOTA_UNIT_ORDER_NONE


def test_synthetic_service_contract_and_determinism():
    def run(seed):
        svc = SyntheticDotaService(seed=seed)
        r = svc.reset_sync(get_1v1_selfplay_config())
        assert len(r.players) == 10
        times = []
        for _ in range(150):
            for team in (TEAM_RADIANT, TEAM_DIRE):
                o = svc.observe_sync(pb.ObserveConfig(team_id=team))
                times.append(o.world_state.dota_time)
                svc.act_sync(pb.Actions(actions=pb.CMsgBotWorldState.Actions(), team_id=team))
        return times, o.world_state.SerializeToString()
    t1, s1 = run(3)
    t2, s2 = run(3)
    assert t1 == t2 and s1 == s2
    assert t1[-1] > 60   # creeps spawned and the clock advanced 0.5 s per observation
    ws = pb.CMsgBotWorldState.FromString(s1)
    assert any(u.unit_type == UnitType.LANE_CREEP for u in ws.units)


def test_validation_config_has_default_bot():
    import random
    cfg = get_1v1_bot_vs_default_config(rng=random.Random(0))
    modes = sorted(p.control_mode for p in cfg.hero_picks if p.hero_id == 11)
    assert modes == [1, 2]   # DEFAULT + CONTROLLED


def test_5v5_layout_featurize():
    from dotaclient_amd.env import get_5v5_selfplay_config
    svc = SyntheticDotaService(seed=0)
    r = svc.reset_sync(get_5v5_selfplay_config())
    ws = r.world_state_radiant
    f = featurize(ws, player_id=0, team_id=TEAM_RADIANT, layout=LAYOUT_5V5)
    assert f.units.shape == (LAYOUT_5V5.max_units, 10)
