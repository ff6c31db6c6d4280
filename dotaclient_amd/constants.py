"""Game / action-space / reward constants shared by actor, learner and kernels.

Mirrors the reference's module constants so that experience records, checkpoints and metric tags are
interchangeable with dotaclient:

* action space and move grid — reference policy.py:38-49
* reward keys — reference policy.py:20
* observation timing — reference agent.py:50-54, policy.py:17
* XP table — reference agent.py:69-95
* featurizer scale — reference agent.py:55 (MAP_HALF_WIDTH)

The unit layout (how the 7 policy inputs are packed into one contiguous ``(.., U, 10)`` tensor for the
HIP kernels) is defined here too, since both the featurizer (C++ and python) and the kernels depend on it.
"""
from __future__ import annotations

import math
from dataclasses import dataclass
from typing import Dict, List, Tuple

import numpy as np

# --- timing (agent.py:50-53, policy.py:17) -------------------------------------------------------------
TICKS_PER_SECOND = 30
TICKS_PER_OBSERVATION = 15
HOST_TIMESCALE = 10
N_DELAY_ENUMS = 5
OBSERVATIONS_PER_SECOND = TICKS_PER_SECOND / TICKS_PER_OBSERVATION
MAX_AGE_WEIGHTSTORE = 64
N_GAMES = 10_000_000

# --- featurizer scales (agent.py:55, 537-542) -------------------------------------------------------------
MAP_HALF_WIDTH = 7000.0
N_UNIT_FEATURES = 10
N_ENV_FEATURES = 3

# --- move grid (policy.py:38-43) --------------------------------------------------------------------------
MAX_MOVE_SPEED = 550
MAX_MOVE_IN_OBS = (MAX_MOVE_SPEED / TICKS_PER_SECOND) * TICKS_PER_OBSERVATION  # 275 world units
N_MOVE_ENUMS = 9
MOVE_ENUMS = (np.arange(N_MOVE_ENUMS, dtype=np.float32) - int(N_MOVE_ENUMS / 2)) * (
    MAX_MOVE_IN_OBS / (N_MOVE_ENUMS - 1) * 2)

# --- rewards (policy.py:20) -------------------------------------------------------------------------------
REWARD_KEYS: List[str] = ['enemy', 'win', 'xp', 'hp', 'kills', 'death', 'lh', 'denies', 'tower_hp']

# XP needed to *reach* a level (agent.py:69-95).
XP_TO_REACH_LEVEL: Dict[int, int] = {
    1: 0, 2: 230, 3: 600, 4: 1080, 5: 1680, 6: 2300, 7: 2940, 8: 3600, 9: 4280, 10: 5080,
    11: 5900, 12: 6740, 13: 7640, 14: 8865, 15: 10115, 16: 11390, 17: 12690, 18: 14015,
    19: 15415, 20: 16905, 21: 18405, 22: 20155, 23: 22155, 24: 24405, 25: 26905,
}

# --- action heads (policy.py:44-49) -----------------------------------------------------------------------
OUTPUT_KEYS: List[str] = ['enum', 'x', 'y', 'target_unit']
INPUT_KEYS: List[str] = ['env', 'allied_heroes', 'enemy_heroes', 'allied_nonheroes', 'enemy_nonheroes',
                         'allied_towers', 'enemy_towers']
UNIT_KEYS: List[str] = INPUT_KEYS[1:]

ENUM_NONE, ENUM_MOVE, ENUM_ATTACK = 0, 1, 2
N_ENUMS = 3

# Team ids of the DotaService contract (TEAM_RADIANT=2, TEAM_DIRE=3 as in Valve's enum).
TEAM_RADIANT = 2
TEAM_DIRE = 3
OPPOSITE_TEAM = {TEAM_RADIANT: TEAM_DIRE, TEAM_DIRE: TEAM_RADIANT}


@dataclass(frozen=True)
class UnitLayout:
    """Number of unit slots per unit-type group, in the fixed order of ``UNIT_KEYS``.

    1v1-mid (reference agent.py:581-616): self hero 1, enemy heroes 5, allied/enemy non-heroes 16,
    allied/enemy mid towers 1  → MAX_UNITS = 40 (policy.py:45).
    5v5: all 5 allied heroes (self first), 5 enemy heroes, 24 non-heroes per side, 3 towers per side.
    """
    allied_heroes: int = 1
    enemy_heroes: int = 5
    allied_nonheroes: int = 16
    enemy_nonheroes: int = 16
    allied_towers: int = 1
    enemy_towers: int = 1

    @property
    def counts(self) -> Tuple[int, ...]:
        return (self.allied_heroes, self.enemy_heroes, self.allied_nonheroes, self.enemy_nonheroes,
                self.allied_towers, self.enemy_towers)

    @property
    def max_units(self) -> int:
        return sum(self.counts)

    @property
    def offsets(self) -> Tuple[int, ...]:
        out, acc = [], 0
        for c in self.counts:
            out.append(acc)
            acc += c
        return tuple(out)

    def slices(self) -> Dict[str, slice]:
        return {k: slice(o, o + c) for k, o, c in zip(UNIT_KEYS, self.offsets, self.counts)}

    def action_counts(self) -> Dict[str, int]:
        return {'enum': N_ENUMS, 'x': N_MOVE_ENUMS, 'y': N_MOVE_ENUMS, 'target_unit': self.max_units}

    def head_offsets(self) -> Dict[str, Tuple[int, int]]:
        """(start, width) of each head inside the flat ``enum|x|y|target_unit`` vector (policy.py:197-203)."""
        out, acc = {}, 0
        for k, n in self.action_counts().items():
            out[k] = (acc, n)
            acc += n
        return out

    @property
    def flat_action_width(self) -> int:
        return sum(self.action_counts().values())


LAYOUT_1V1 = UnitLayout()
LAYOUT_5V5 = UnitLayout(allied_heroes=5, enemy_heroes=5, allied_nonheroes=24, enemy_nonheroes=24,
                        allied_towers=3, enemy_towers=3)
MAX_UNITS = LAYOUT_1V1.max_units  # 40, policy.py:45
ACTION_OUTPUT_COUNTS = LAYOUT_1V1.action_counts()

# numerically-safe epsilon (policy.py:15, optimizer.py:39)
EPS = float(np.finfo(np.float32).eps)


def get_total_xp(level: int, xp_needed_to_level: int) -> int:
    """Total XP from level and the XP still needed (agent.py:110-115)."""
    if level >= 25:
        return XP_TO_REACH_LEVEL[25]
    xp_required_for_next = XP_TO_REACH_LEVEL[level + 1] - XP_TO_REACH_LEVEL[level]
    return XP_TO_REACH_LEVEL[level] + (xp_required_for_next - xp_needed_to_level)


def level_from_total_xp(total_xp: float) -> Tuple[int, int]:
    """Inverse of :func:`get_total_xp`: returns (level, xp_needed_to_level)."""
    level = 1
    for lvl in range(1, 26):
        if total_xp >= XP_TO_REACH_LEVEL[lvl]:
            level = lvl
    if level >= 25:
        return 25, 0
    return level, int(XP_TO_REACH_LEVEL[level + 1] - total_xp)


def facing_sin_cos(facing_deg: float) -> Tuple[float, float]:
    r = facing_deg * (2 * math.pi) / 360
    return math.sin(r), math.cos(r)
