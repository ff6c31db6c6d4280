"""Action decoding: sampled head indices → ``CMsgBotWorldState.Action`` (reference agent.py:665-695)."""
from __future__ import annotations

from typing import Dict

from ..constants import ENUM_ATTACK, ENUM_MOVE, ENUM_NONE, MOVE_ENUMS
from ..protos import ActionType, pb


def action_to_pb(action_dict: Dict[str, int], hero_location, unit_handles, player_id: int = None):
    """``action_dict`` holds python ints for the heads that were sampled (enum, and x/y or target_unit)."""
    action_pb = pb.CMsgBotWorldState.Action()
    action_pb.actionDelay = 0
    action_enum = int(action_dict['enum'])
    if action_enum == ENUM_NONE:
        action_pb.actionType = ActionType.DOTA_UNIT_ORDER_NONE
    elif action_enum == ENUM_MOVE:
        action_pb.actionType = ActionType.DOTA_UNIT_ORDER_MOVE_DIRECTLY
        loc = action_pb.moveDirectly.location
        loc.x = hero_location.x + float(MOVE_ENUMS[int(action_dict['x'])])
        loc.y = hero_location.y + float(MOVE_ENUMS[int(action_dict['y'])])
        loc.z = 0
    elif action_enum == ENUM_ATTACK:
        action_pb.actionType = ActionType.DOTA_UNIT_ORDER_ATTACK_TARGET
        if 'target_unit' in action_dict:
            action_pb.attackTarget.target = int(unit_handles[int(action_dict['target_unit'])])
        else:
            action_pb.attackTarget.target = -1
        action_pb.attackTarget.once = True
    else:
        raise ValueError(f'unknown action {action_enum}')
    if player_id is not None:
        action_pb.player = player_id
    return action_pb
