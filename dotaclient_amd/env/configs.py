"""Game configurations (reference agent.py:905-949)."""
from __future__ import annotations

import random
from typing import Optional

from ..constants import HOST_TIMESCALE, TICKS_PER_OBSERVATION
from ..protos import GameMode, Hero, HeroControlMode, HostMode, TEAM_DIRE, TEAM_RADIANT, pb

CONTROLLED = HeroControlMode.HERO_CONTROL_MODE_CONTROLLED
DEFAULT = HeroControlMode.HERO_CONTROL_MODE_DEFAULT
IDLE = HeroControlMode.HERO_CONTROL_MODE_IDLE


def _config(picks, seed: Optional[int] = None):
    return pb.GameConfig(ticks_per_observation=TICKS_PER_OBSERVATION, host_timescale=HOST_TIMESCALE,
                         host_mode=HostMode.HOST_MODE_DEDICATED, game_mode=GameMode.DOTA_GAMEMODE_1V1MID,
                         hero_picks=picks, seed=seed or 0)


def _team(team, first_mode, first_hero=Hero.NPC_DOTA_HERO_NEVERMORE, n_controlled=1):
    picks = []
    for i in range(5):
        if i < n_controlled:
            picks.append(pb.HeroPick(team_id=team, hero_id=first_hero, control_mode=first_mode))
        else:
            picks.append(pb.HeroPick(team_id=team, hero_id=Hero.NPC_DOTA_HERO_SNIPER, control_mode=IDLE))
    return picks


def get_1v1_selfplay_config(seed: Optional[int] = None):
    """Nevermore vs Nevermore, both controlled, 4 idle Snipers per team (agent.py:930-949)."""
    return _config(_team(TEAM_RADIANT, CONTROLLED) + _team(TEAM_DIRE, CONTROLLED), seed)


def get_1v1_bot_vs_default_config(seed: Optional[int] = None, rng: Optional[random.Random] = None):
    """Validation: one controlled hero vs the built-in default bot, sides randomised (agent.py:905-927)."""
    modes = [DEFAULT, CONTROLLED]
    (rng or random).shuffle(modes)
    return _config(_team(TEAM_RADIANT, modes[0]) + _team(TEAM_DIRE, modes[1]), seed)


def get_5v5_selfplay_config(seed: Optional[int] = None):
    """All 10 heroes controlled (BASELINE config 4)."""
    return _config(_team(TEAM_RADIANT, CONTROLLED, n_controlled=5) + _team(TEAM_DIRE, CONTROLLED, n_controlled=5),
                   seed)
