"""Shaped reward (reference agent.py:118-158, 325-337, 829-833)."""
from __future__ import annotations

from typing import Dict, List, Optional

import numpy as np

from ..constants import REWARD_KEYS, get_total_xp
from ..protos import Status, TEAM_DIRE, TEAM_RADIANT
from .featurizer import get_mid_tower, get_player, get_unit

END_STATUS_TO_TEAM = {Status.RADIANT_WIN: TEAM_RADIANT, Status.DIRE_WIN: TEAM_DIRE}


def get_reward(prev_obs, obs, player_id: int) -> Dict[str, float]:
    """Nine shaped sub-rewards for one step. ``enemy`` and ``win`` are filled in by the game loop."""
    unit_init = get_unit(prev_obs, player_id=player_id)
    unit = get_unit(obs, player_id=player_id)
    player_init = get_player(prev_obs, player_id=player_id)
    player = get_player(obs, player_id=player_id)
    mid_tower_init = get_mid_tower(prev_obs, team_id=player.team_id)
    mid_tower = get_mid_tower(obs, team_id=player.team_id)

    reward = {key: 0. for key in REWARD_KEYS}
    xp_init = get_total_xp(level=unit_init.level, xp_needed_to_level=unit_init.xp_needed_to_level)
    xp = get_total_xp(level=unit.level, xp_needed_to_level=unit.xp_needed_to_level)
    reward['xp'] = (xp - xp_init) * 0.001
    if unit_init.is_alive and unit.is_alive:
        hp_rel_init = unit_init.health / unit_init.health_max
        hp_rel = unit.health / unit.health_max
        low_hp_factor = 1. + (1 - hp_rel) ** 2
        reward['hp'] = (hp_rel - hp_rel_init) * low_hp_factor * 0.2
    reward['kills'] = (player.kills - player_init.kills) * 0.4
    reward['death'] = (player.deaths - player_init.deaths) * -0.4
    reward['lh'] = (unit.last_hits - unit_init.last_hits) * 0.1
    reward['denies'] = (unit.denies - unit_init.denies) * 0.05
    reward['tower_hp'] = (mid_tower.health - mid_tower_init.health) / 1900.
    return reward


def end_state_reward(end_state: Optional[int], team_id: int) -> float:
    """+1 win, −1 loss, −0.25 if no winner (agent.py:325-337)."""
    if end_state in END_STATUS_TO_TEAM:
        return 1.0 if END_STATUS_TO_TEAM[end_state] == team_id else -1.0
    return -0.25


def pack_rewards(rewards: List[Dict[str, float]]) -> np.ndarray:
    """list of reward dicts → float64 (T, 9) in REWARD_KEYS order (agent.py:356-363)."""
    t = np.zeros([len(rewards), len(REWARD_KEYS)])
    for i, r in enumerate(rewards):
        for j, key in enumerate(REWARD_KEYS):
            t[i, j] = r[key]
    return t
