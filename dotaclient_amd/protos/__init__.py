"""DotaService / CMsgBotWorldState protobuf schema (runtime-built; see schema.py)."""
from .schema import (pb, Team, Status, HostMode, GameMode, HeroControlMode, Hero, UnitType, ActionType,  # noqa: F401
                     TEAM_RADIANT, TEAM_DIRE, FIELD_NUMBERS, SERVICE_NAME)
