"""Compact raw unit records: the observation form that crosses PCIe and the experience ring when featurization runs
on the GPU (``ops/csrc/featurize.hip``).

The reference featurizes every unit on the actor's CPU (agent.py:496-562; :func:`~.featurizer.unit_matrix`). Here the
host keeps only what needs the protobuf unit lists — which units fill which slot, the handle validity rules, the
attack / projectile cross-references and the health ratio — and writes one 8-word record per slot:

    w0 x, w1 y, w2 z, w3 facing   fp32 as observed
    w4 1 − health / health_max    the first feature (double, rounded once — it also decides the denial rule)
    w5 handle                     −1 = not targetable
    w6 flags                      bit 0 present, bit 1 attacks the hero, bit 2 the hero attacks it
    w7 0

plus a per-observation hero record (x, y, attack range, 0). Distance, normalised position / height, facing sin / cos
and the attack-range test are computed from these on the device (:func:`featurize_raw_np` is the numpy oracle of that
kernel and the host fallback for consumers without a GPU). Every value equals :func:`~.featurizer.featurize`'s.
"""
from __future__ import annotations

import math
from typing import Tuple

import numpy as np

from ..constants import LAYOUT_1V1, MAP_HALF_WIDTH, OPPOSITE_TEAM, UNIT_KEYS, UnitLayout
from ..protos import UnitType
from .featurizer import ANIM_TOWER_IDLE, env_features, get_unit, is_unit_attacking_unit, unit_separation

RAW_WORDS = 8
HERO_WORDS = 4
F_PRESENT, F_ATTACKS_ME, F_ME_ATTACKING = 1, 2, 4


def raw_unit_rows(unit_list, hero_unit, only_self: bool = False, max_units: int = 16) -> np.ndarray:
    """(max_units, 8) int32 raw records of one unit block — :func:`~.featurizer.unit_matrix`'s slot selection and
    handle rules, without the per-unit feature arithmetic."""
    out = np.zeros((max_units, RAW_WORDS), np.int32)
    f = out.view(np.float32)
    i = 0
    for unit in unit_list:
        if not unit.is_alive:
            continue
        if only_self and unit != hero_unit:
            continue
        if i >= max_units:
            break
        hp = unit.health / unit.health_max
        f[i, 0], f[i, 1], f[i, 2] = unit.location.x, unit.location.y, unit.location.z
        f[i, 3] = unit.facing
        f[i, 4] = 1.0 - hp
        if unit.is_invulnerable or unit.is_attack_immune:
            h = -1
        elif (unit.team_id == OPPOSITE_TEAM.get(hero_unit.team_id) and unit.unit_type == UnitType.TOWER
              and unit.anim_activity == ANIM_TOWER_IDLE):
            h = -1
        elif unit.team_id == hero_unit.team_id and unit.unit_type == UnitType.TOWER:
            h = -1
        elif unit.team_id == hero_unit.team_id and hp > 0.5:
            h = -1
        else:
            h = unit.handle
        out[i, 5] = h                      # (handles ≥ 2³¹ do not fit the record: numpy raises)
        out[i, 6] = (F_PRESENT | (F_ATTACKS_ME if is_unit_attacking_unit(unit, hero_unit) else 0)
                     | (F_ME_ATTACKING if is_unit_attacking_unit(hero_unit, unit) else 0))
        i += 1
    return out


def featurize_raw_obs(world_state, player_id: int, team_id: int, layout: UnitLayout = LAYOUT_1V1,
                      hero_unit=None) -> Tuple[np.ndarray, np.ndarray, np.ndarray]:
    """(env (3,), hero (4,), raw (U, 8)) of one observation — :func:`~.featurizer.featurize`'s slot layout."""
    if hero_unit is None:
        hero_unit = get_unit(world_state, player_id=player_id)
    env = env_features(world_state.dota_time, team_id)
    hero = np.array([hero_unit.location.x, hero_unit.location.y, hero_unit.attack_range, 0.0], np.float32)
    sep = unit_separation(world_state, hero_unit.team_id)
    counts = dict(zip(UNIT_KEYS, layout.counts))
    lists = {
        'allied_heroes': sep.allied_heroes, 'enemy_heroes': sep.enemy_heroes,
        'allied_nonheroes': [*sep.allied_nonheroes, *sep.allied_creep],
        'enemy_nonheroes': [*sep.enemy_nonheroes, *sep.enemy_creep],
        'allied_towers': sep.allied_towers, 'enemy_towers': sep.enemy_towers,
    }
    raw = np.zeros((layout.max_units, RAW_WORDS), np.int32)
    for key, sl in layout.slices().items():
        ulist = lists[key]
        only_self = False
        if key == 'allied_heroes':
            if counts[key] == 1:
                only_self = True
            else:
                ulist = [hero_unit] + [u for u in ulist if u.player_id != player_id]
        raw[sl] = raw_unit_rows(ulist, hero_unit, only_self=only_self, max_units=counts[key])
    return env, hero, raw


def featurize_raw_np(raw: np.ndarray, hero: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Numpy oracle of ``featurize_raw_kernel``: raw (…, U, 8) int32 + hero (…, 4) fp32 → units (…, U, 10) fp32,
    handles (…, U) int64. Float64 arithmetic in the host featurizer's order, one rounding per feature."""
    raw = np.asarray(raw)
    f = raw.view(np.float32).astype(np.float64)
    hero = np.asarray(hero, np.float32).astype(np.float64)[..., None, :]
    present = (raw[..., 6] & F_PRESENT) != 0
    x, y, z, facing = f[..., 0], f[..., 1], f[..., 2], f[..., 3]
    dx, dy = hero[..., 0] - x, hero[..., 1] - y
    dist = np.sqrt(dx * dx + dy * dy)
    ang = facing * (2.0 * math.pi) / 360.0
    units = np.stack([raw[..., 4].view(np.float32).astype(np.float64), x / MAP_HALF_WIDTH, y / MAP_HALF_WIDTH,
                      z / 512.0 - 0.5, dist / MAP_HALF_WIDTH - 0.5, np.sin(ang), np.cos(ang),
                      (dist <= hero[..., 2]).astype(np.float64) - 0.5,
                      ((raw[..., 6] & F_ATTACKS_ME) != 0).astype(np.float64) - 0.5,
                      ((raw[..., 6] & F_ME_ATTACKING) != 0).astype(np.float64) - 0.5], -1).astype(np.float32)
    units[~present] = 0.0
    handles = np.where(present, raw[..., 5].astype(np.int64), -1)
    return units, handles


# ---- the 16-byte record of the fp8 policy step (its features are fp16): x | y, z | facing, (1 − hp) | flags as
# binary16 pairs, then the handle (native/core.h raw_to_raw16, ops/csrc/featurize.hip featurize_raw16_kernel)
RAW16_WORDS = 4


def pack_raw16(raw: np.ndarray) -> np.ndarray:
    """(…, U, 8) int32 raw records → (…, U, 4) int32 16-byte records (float → binary16 round to nearest even; the
    native converter when built, this numpy form otherwise — equal, tests/test_gpu_featurize.py)."""
    raw = np.ascontiguousarray(raw, dtype=np.int32)
    try:
        from ..native import _native
        return _native.pack_raw16(raw)
    except (ImportError, AttributeError):
        pass
    return _pack_raw16_np(raw)


def _pack_raw16_np(raw: np.ndarray) -> np.ndarray:
    f16 = raw.view(np.float32)[..., :5].astype(np.float16).view(np.uint16).astype(np.uint32)
    out = np.empty(raw.shape[:-1] + (RAW16_WORDS,), np.uint32)
    out[..., 0] = f16[..., 0] | (f16[..., 1] << 16)
    out[..., 1] = f16[..., 2] | (f16[..., 3] << 16)
    out[..., 2] = f16[..., 4] | ((raw[..., 6].astype(np.uint32) & 0xFFFF) << 16)
    out[..., 3] = raw[..., 5].view(np.uint32)
    return out.view(np.int32)


def featurize_raw16_np(raw16: np.ndarray, hero: np.ndarray) -> Tuple[np.ndarray, np.ndarray]:
    """Numpy oracle of ``featurize_raw16_kernel`` (fp32 arithmetic, one fp16 rounding per feature): → units (…, U, 10)
    fp16, handles (…, U) int32."""
    w = np.asarray(raw16).view(np.uint32)
    half = lambda v: v.astype(np.uint16).view(np.float16).astype(np.float32)   # noqa: E731
    x, y = half(w[..., 0] & 0xFFFF), half(w[..., 0] >> 16)
    z, facing = half(w[..., 1] & 0xFFFF), half(w[..., 1] >> 16)
    rel, flags = half(w[..., 2] & 0xFFFF), (w[..., 2] >> 16).astype(np.int32)
    hero = np.asarray(hero, np.float32)[..., None, :]
    dx, dy = hero[..., 0] - x, hero[..., 1] - y
    dist = np.sqrt(dx * dx + dy * dy)
    ang = facing * np.float32(2.0 * 3.14159265358979) / np.float32(360.0)
    one, h = np.float32(1.0), np.float32(0.5)
    units = np.stack([rel, x / np.float32(7000.0), y / np.float32(7000.0), z / np.float32(512.0) - h,
                      dist / np.float32(7000.0) - h, np.sin(ang), np.cos(ang),
                      np.where(dist <= hero[..., 2], one, np.float32(0.0)) - h,
                      np.where(flags & F_ATTACKS_ME, one, np.float32(0.0)) - h,
                      np.where(flags & F_ME_ATTACKING, one, np.float32(0.0)) - h], -1).astype(np.float16)
    present = (flags & F_PRESENT) != 0
    units[~present] = 0
    handles = np.where(present, w[..., 3].view(np.int32), -1).astype(np.int32)
    return units, handles
