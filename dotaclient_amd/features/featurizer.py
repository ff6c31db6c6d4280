"""Observation featurizer: CMsgBotWorldState → fixed policy tensors (python reference implementation).

Behaviour matches the reference exactly:

* ``unit_separation`` — reference agent.py:456-493 (allied/enemy × hero/creep-hero/lane-creep/mid-tower)
* ``unit_matrix``     — reference agent.py:496-562 (10 features per unit, handle validity rules)
* ``featurize``       — reference agent.py:564-637 (env features, 6 unit blocks, unit_handles)

Besides the reference's 7-tensor dict, :func:`featurize_packed` returns the packed ``(U, 10)`` unit tensor in the
:class:`~dotaclient_amd.constants.UnitLayout` order the HIP kernels consume. The C++ featurizer
(``dotaclient_amd/native/featurizer.cpp``) implements the same function on the protobuf wire bytes and is tested
against this module.
"""
from __future__ import annotations

import math
from typing import Dict, NamedTuple, Tuple

import numpy as np

from ..constants import (LAYOUT_1V1, MAP_HALF_WIDTH, N_UNIT_FEATURES, OPPOSITE_TEAM, TEAM_DIRE, UNIT_KEYS,
                         UnitLayout)
from ..protos import UnitType

ANIM_TOWER_IDLE = 1500


def get_player(state, player_id):
    for player in state.players:
        if player.player_id == player_id:
            return player
    raise ValueError(f'hero {player_id} not found in state')


def get_unit(state, player_id):
    for unit in state.units:
        if unit.unit_type == UnitType.HERO and unit.player_id == player_id:
            return unit
    raise ValueError(f'unit {player_id} not found in state')


def get_mid_tower(state, team_id):
    for unit in state.units:
        if unit.unit_type == UnitType.TOWER and unit.team_id == team_id and 'tower1_mid' in unit.name:
            return unit
    raise ValueError('tower not found in state')


def is_unit_attacking_unit(unit_attacker, unit_target) -> float:
    """Direct attack or an incoming attack projectile (agent.py:250-259)."""
    if unit_attacker.attack_target_handle == unit_target.handle:
        return 1.0
    for projectile in unit_target.incoming_tracking_projectiles:
        if projectile.caster_handle == unit_attacker.handle and projectile.is_attack:
            return 1.0
    return 0.0


def is_invulnerable(unit) -> bool:
    """Modifier-based invulnerability check (agent.py:261-265; unused by the reference's featurizer)."""
    return any(mod.name == 'modifier_invulnerable' for mod in unit.modifiers)


class Separated(NamedTuple):
    allied_heroes: list
    enemy_heroes: list
    allied_nonheroes: list
    enemy_nonheroes: list
    allied_creep: list
    enemy_creep: list
    allied_towers: list
    enemy_towers: list


def unit_separation(state, team_id) -> Separated:
    """Single pass over the unit list (agent.py:456-493)."""
    ah, eh, anh, enh, ac, ec, at, et = [], [], [], [], [], [], [], []
    for unit in state.units:
        t = unit.unit_type
        if unit.team_id == team_id:
            if t == UnitType.HERO:
                ah.append(unit)
            elif t == UnitType.CREEP_HERO:
                anh.append(unit)
            elif t == UnitType.LANE_CREEP:
                ac.append(unit)
            elif t == UnitType.TOWER and unit.name[-5:] == '1_mid':
                at.append(unit)
        else:
            if t == UnitType.HERO:
                eh.append(unit)
            elif t == UnitType.CREEP_HERO:
                enh.append(unit)
            elif t == UnitType.LANE_CREEP:
                ec.append(unit)
            elif t == UnitType.TOWER and unit.name[-5:] == '1_mid':
                et.append(unit)
    return Separated(ah, eh, anh, enh, ac, ec, at, et)


def unit_matrix(unit_list, hero_unit, only_self: bool = False, max_units: int = 16
                ) -> Tuple[np.ndarray, np.ndarray]:
    """(max_units, 10) features + (max_units,) handles (−1 = not targetable) — agent.py:496-562."""
    handles = np.full([max_units], -1, dtype=np.int64)
    m = np.zeros([max_units, N_UNIT_FEATURES], dtype=np.float32)
    i = 0
    for unit in unit_list:
        if not unit.is_alive:
            continue
        if only_self and unit != hero_unit:
            continue
        if i >= max_units:
            break
        rel_hp = 1.0 - (unit.health / unit.health_max)
        loc_x = unit.location.x / MAP_HALF_WIDTH
        loc_y = unit.location.y / MAP_HALF_WIDTH
        loc_z = (unit.location.z / 512.) - 0.5
        dx = hero_unit.location.x - unit.location.x
        dy = hero_unit.location.y - unit.location.y
        distance = math.sqrt(dx ** 2 + dy ** 2)
        norm_distance = (distance / MAP_HALF_WIDTH) - 0.5
        facing_sin = math.sin(unit.facing * (2 * math.pi) / 360)
        facing_cos = math.cos(unit.facing * (2 * math.pi) / 360)
        in_attack_range = float(distance <= hero_unit.attack_range) - 0.5
        is_attacking_me = is_unit_attacking_unit(unit, hero_unit) - 0.5
        me_attacking_unit = is_unit_attacking_unit(hero_unit, unit) - 0.5
        m[i] = (rel_hp, loc_x, loc_y, loc_z, norm_distance, facing_sin, facing_cos, in_attack_range,
                is_attacking_me, me_attacking_unit)
        if unit.is_invulnerable or unit.is_attack_immune:
            handles[i] = -1
        elif (unit.team_id == OPPOSITE_TEAM.get(hero_unit.team_id) and unit.unit_type == UnitType.TOWER
              and unit.anim_activity == ANIM_TOWER_IDLE):
            handles[i] = -1   # idle enemy tower cannot be attacked through the bot API (agent.py:548-551)
        elif unit.team_id == hero_unit.team_id and unit.unit_type == UnitType.TOWER:
            handles[i] = -1   # own tower
        elif unit.team_id == hero_unit.team_id and (unit.health / unit.health_max) > 0.5:
            handles[i] = -1   # not deniable
        else:
            handles[i] = unit.handle
        i += 1
    return m, handles


class Featurized(NamedTuple):
    env: np.ndarray                 # (3,)
    units: np.ndarray               # (U, 10) packed in layout order
    handles: np.ndarray             # (U,) int64, -1 = invalid
    inputs: Dict[str, np.ndarray]   # reference 7-key dict (views into env/units)
    n_allied_creep: int             # for the creep-spawn sanity check (agent.py:621-627)


def env_features(dota_time: float, team_id: int) -> np.ndarray:
    """(dota_time/1200, sin(2π t/60), ±0.2 team) — agent.py:568-572."""
    return np.array([dota_time / 1200., math.sin(dota_time * (2. * math.pi) / 60),
                     -.2 if team_id == TEAM_DIRE else .2], dtype=np.float32)


def featurize(world_state, player_id: int, team_id: int, layout: UnitLayout = LAYOUT_1V1,
              hero_unit=None) -> Featurized:
    """Full observation → policy input (agent.py:564-637)."""
    if hero_unit is None:
        hero_unit = get_unit(world_state, player_id=player_id)
    env = env_features(world_state.dota_time, team_id)
    sep = unit_separation(world_state, hero_unit.team_id)
    counts = dict(zip(UNIT_KEYS, layout.counts))
    lists = {
        'allied_heroes': sep.allied_heroes,
        'enemy_heroes': sep.enemy_heroes,
        'allied_nonheroes': [*sep.allied_nonheroes, *sep.allied_creep],
        'enemy_nonheroes': [*sep.enemy_nonheroes, *sep.enemy_creep],
        'allied_towers': sep.allied_towers,
        'enemy_towers': sep.enemy_towers,
    }
    units = np.zeros([layout.max_units, N_UNIT_FEATURES], dtype=np.float32)
    handles = np.full([layout.max_units], -1, dtype=np.int64)
    inputs = {'env': env}
    for key, sl in layout.slices().items():
        ulist = lists[key]
        only_self = False
        if key == 'allied_heroes':
            if counts[key] == 1:
                only_self = True   # 1v1: "For now, ignore teammates" (agent.py:581-586)
            else:
                # 5v5: self first, then teammates.
                ulist = [hero_unit] + [u for u in ulist if u.player_id != player_id]
        m, h = unit_matrix(ulist, hero_unit, only_self=only_self, max_units=counts[key])
        units[sl] = m
        handles[sl] = h
        inputs[key] = units[sl]
    return Featurized(env=env, units=units, handles=handles, inputs=inputs, n_allied_creep=len(sep.allied_creep))
