"""Runtime-built protobuf schema for the DotaService / CMsgBotWorldState contract.

The reference imports generated modules from the ``dotaservice`` package (agent.py:18-29), which is not
installable here and there is no ``protoc``. We therefore build the message classes at import time from a
``FileDescriptorProto``. Message and field *names* follow what the reference reads; the field
*numbers* are our own (wire-compatibility with Valve's .proto cannot be verified offline) and are mirrored
exactly by the C++ wire decoder in ``dotaclient_amd/native/featurizer.cpp`` — keep the two in sync (the
``FIELD_NUMBERS`` table below is exported for a test that checks this).

Usage::

    from dotaclient_amd.protos import pb
    ws = pb.CMsgBotWorldState(dota_time=1.5)
    u = ws.units.add(unit_type=pb.CMsgBotWorldState.UnitType.Value('HERO'))
"""
from __future__ import annotations

from types import SimpleNamespace
from typing import Dict, List, Tuple

from google.protobuf import descriptor_pb2, descriptor_pool, message_factory

F = descriptor_pb2.FieldDescriptorProto

_T = {
    'double': F.TYPE_DOUBLE, 'float': F.TYPE_FLOAT, 'int64': F.TYPE_INT64, 'uint64': F.TYPE_UINT64,
    'int32': F.TYPE_INT32, 'uint32': F.TYPE_UINT32, 'bool': F.TYPE_BOOL, 'string': F.TYPE_STRING,
    'bytes': F.TYPE_BYTES, 'sint32': F.TYPE_SINT32,
}

PACKAGE = 'dotaservice'

# (name, number, type, label, type_name)  label: 'opt' | 'rep'
# type may be a scalar key of _T, or 'msg:<Name>' / 'enum:<Name>' (fully-qualified under PACKAGE).
_VECTOR = [('x', 1, 'float'), ('y', 2, 'float'), ('z', 3, 'float')]

_UNIT_TYPES = ['INVALID', 'HERO', 'CREEP_HERO', 'LANE_CREEP', 'JUNGLE_CREEP', 'ROSHAN', 'TOWER', 'BARRACKS',
               'SHRINE', 'FORT', 'EFFIGY', 'WARD', 'COURIER']

_ACTION_TYPES = [('DOTA_UNIT_ORDER_NONE', 0), ('DOTA_UNIT_ORDER_MOVE_TO_POSITION', 1),
                 ('DOTA_UNIT_ORDER_MOVE_TO_TARGET', 2), ('DOTA_UNIT_ORDER_ATTACK_MOVE', 3),
                 ('DOTA_UNIT_ORDER_ATTACK_TARGET', 4), ('DOTA_UNIT_ORDER_STOP', 21),
                 ('DOTA_UNIT_ORDER_MOVE_DIRECTLY', 37)]

# Field-number table for CMsgBotWorldState.Unit — the C++ decoder mirrors this table.
UNIT_FIELDS: List[Tuple[str, int, str, str]] = [
    ('handle', 1, 'uint32', 'opt'),
    ('unit_type', 2, 'enum:CMsgBotWorldState.UnitType', 'opt'),
    ('name', 3, 'string', 'opt'),
    ('team_id', 4, 'uint32', 'opt'),
    ('level', 5, 'uint32', 'opt'),
    ('location', 6, 'msg:CMsgBotWorldState.Vector', 'opt'),
    ('is_alive', 7, 'bool', 'opt'),
    ('player_id', 8, 'int32', 'opt'),
    ('facing', 11, 'float', 'opt'),
    ('health', 20, 'int32', 'opt'),
    ('health_max', 21, 'int32', 'opt'),
    ('mana', 23, 'float', 'opt'),
    ('mana_max', 24, 'float', 'opt'),
    ('attack_range', 30, 'int32', 'opt'),
    ('attack_damage', 31, 'int32', 'opt'),
    ('attack_target_handle', 35, 'uint32', 'opt'),
    ('anim_activity', 40, 'int32', 'opt'),
    ('is_invulnerable', 50, 'bool', 'opt'),
    ('is_attack_immune', 51, 'bool', 'opt'),
    ('xp_needed_to_level', 60, 'uint32', 'opt'),
    ('last_hits', 61, 'uint32', 'opt'),
    ('denies', 62, 'uint32', 'opt'),
    ('incoming_tracking_projectiles', 70, 'msg:CMsgBotWorldState.TrackingProjectile', 'rep'),
    ('modifiers', 71, 'msg:CMsgBotWorldState.Modifier', 'rep'),
]

WORLD_STATE_FIELDS: List[Tuple[str, int, str, str]] = [
    ('team_id', 1, 'uint32', 'opt'),
    ('game_time', 2, 'float', 'opt'),
    ('dota_time', 3, 'float', 'opt'),
    ('game_state', 4, 'uint32', 'opt'),
    ('players', 10, 'msg:CMsgBotWorldState.Player', 'rep'),
    ('units', 11, 'msg:CMsgBotWorldState.Unit', 'rep'),
]

PLAYER_FIELDS = [('player_id', 1, 'int32', 'opt'), ('hero_id', 2, 'uint32', 'opt'),
                 ('is_alive', 3, 'bool', 'opt'), ('respawn_time', 4, 'float', 'opt'),
                 ('kills', 5, 'uint32', 'opt'), ('deaths', 6, 'uint32', 'opt'),
                 ('assists', 7, 'uint32', 'opt'), ('team_id', 8, 'uint32', 'opt')]

PROJECTILE_FIELDS = [('caster_handle', 1, 'uint32', 'opt'), ('location', 2, 'msg:CMsgBotWorldState.Vector', 'opt'),
                     ('is_attack', 4, 'bool', 'opt')]

FIELD_NUMBERS: Dict[str, Dict[str, int]] = {
    'WorldState': {n: k for n, k, _, _ in WORLD_STATE_FIELDS},
    'Unit': {n: k for n, k, _, _ in UNIT_FIELDS},
    'Player': {n: k for n, k, _, _ in PLAYER_FIELDS},
    'Projectile': {n: k for n, k, _, _ in PROJECTILE_FIELDS},
    'Vector': {n: k for n, k, _ in _VECTOR},
}


def _add_fields(msg: descriptor_pb2.DescriptorProto, fields):
    for spec in fields:
        name, number, typ = spec[0], spec[1], spec[2]
        label = spec[3] if len(spec) > 3 else 'opt'
        f = msg.field.add(name=name, number=number)
        f.label = F.LABEL_REPEATED if label == 'rep' else F.LABEL_OPTIONAL
        if typ.startswith('msg:'):
            f.type = F.TYPE_MESSAGE
            f.type_name = f'.{PACKAGE}.{typ[4:]}'
        elif typ.startswith('enum:'):
            f.type = F.TYPE_ENUM
            f.type_name = f'.{PACKAGE}.{typ[5:]}'
        else:
            f.type = _T[typ]


def _add_enum(parent, name, values):
    e = parent.enum_type.add(name=name)
    for i, v in enumerate(values):
        if isinstance(v, tuple):
            e.value.add(name=v[0], number=v[1])
        else:
            e.value.add(name=v, number=i)
    return e


def _build_file() -> descriptor_pb2.FileDescriptorProto:
    fd = descriptor_pb2.FileDescriptorProto(name='dotaclient_amd/dotaservice.proto', package=PACKAGE,
                                            syntax='proto2')
    # ---- CMsgBotWorldState ----
    ws = fd.message_type.add(name='CMsgBotWorldState')
    _add_enum(ws, 'UnitType', _UNIT_TYPES)
    vec = ws.nested_type.add(name='Vector')
    _add_fields(vec, _VECTOR)
    proj = ws.nested_type.add(name='TrackingProjectile')
    _add_fields(proj, PROJECTILE_FIELDS)
    mod = ws.nested_type.add(name='Modifier')
    _add_fields(mod, [('name', 1, 'string'), ('stack_count', 2, 'uint32')])
    player = ws.nested_type.add(name='Player')
    _add_fields(player, PLAYER_FIELDS)
    unit = ws.nested_type.add(name='Unit')
    _add_fields(unit, UNIT_FIELDS)
    action = ws.nested_type.add(name='Action')
    _add_enum(action, 'Type', _ACTION_TYPES)
    mtl = action.nested_type.add(name='MoveToLocation')
    _add_fields(mtl, [('units', 1, 'int32', 'rep'), ('location', 2, 'msg:CMsgBotWorldState.Vector')])
    att = action.nested_type.add(name='AttackTarget')
    _add_fields(att, [('units', 1, 'int32', 'rep'), ('target', 2, 'int32'), ('once', 3, 'bool')])
    _add_fields(action, [
        ('actionType', 1, 'enum:CMsgBotWorldState.Action.Type'),
        ('player', 2, 'int32'),
        ('actionDelay', 3, 'int32'),
        ('moveDirectly', 10, 'msg:CMsgBotWorldState.Action.MoveToLocation'),
        ('moveToLocation', 11, 'msg:CMsgBotWorldState.Action.MoveToLocation'),
        ('attackTarget', 12, 'msg:CMsgBotWorldState.Action.AttackTarget'),
    ])
    actions = ws.nested_type.add(name='Actions')
    _add_fields(actions, [('dota_time', 1, 'float'), ('actions', 2, 'msg:CMsgBotWorldState.Action', 'rep')])
    _add_fields(ws, WORLD_STATE_FIELDS)

    # ---- DotaService messages ----
    _add_enum(fd, 'Team', [('TEAM_UNKNOWN', 0), ('TEAM_RADIANT', 2), ('TEAM_DIRE', 3)])
    _add_enum(fd, 'Status', [('OK', 0), ('RADIANT_WIN', 1), ('DIRE_WIN', 2), ('RESOURCE_EXHAUSTED', 3)])
    _add_enum(fd, 'HostMode', ['HOST_MODE_DEDICATED', 'HOST_MODE_GUI', 'HOST_MODE_GUI_MENU'])
    _add_enum(fd, 'GameMode', [('DOTA_GAMEMODE_NONE', 0), ('DOTA_GAMEMODE_AP', 1), ('DOTA_GAMEMODE_1V1MID', 21)])
    _add_enum(fd, 'HeroControlMode', ['HERO_CONTROL_MODE_IDLE', 'HERO_CONTROL_MODE_DEFAULT',
                                      'HERO_CONTROL_MODE_CONTROLLED'])
    _add_enum(fd, 'Hero', [('NPC_DOTA_HERO_NONE', 0), ('NPC_DOTA_HERO_SNIPER', 35), ('NPC_DOTA_HERO_NEVERMORE', 11)])
    hp = fd.message_type.add(name='HeroPick')
    _add_fields(hp, [('team_id', 1, 'enum:Team'), ('hero_id', 2, 'enum:Hero'),
                     ('control_mode', 3, 'enum:HeroControlMode')])
    gc = fd.message_type.add(name='GameConfig')
    _add_fields(gc, [('ticks_per_observation', 1, 'int32'), ('host_timescale', 2, 'float'),
                     ('host_mode', 3, 'enum:HostMode'), ('game_mode', 4, 'enum:GameMode'),
                     ('hero_picks', 5, 'msg:HeroPick', 'rep'), ('seed', 6, 'uint64')])
    oc = fd.message_type.add(name='ObserveConfig')
    _add_fields(oc, [('team_id', 1, 'enum:Team')])
    ob = fd.message_type.add(name='Observation')
    _add_fields(ob, [('status', 1, 'enum:Status'), ('world_state', 2, 'msg:CMsgBotWorldState'),
                     ('team_id', 3, 'enum:Team')])
    pl = fd.message_type.add(name='Player')
    _add_fields(pl, [('id', 1, 'int32'), ('hero', 2, 'enum:Hero'), ('is_bot', 3, 'bool'),
                     ('team_id', 4, 'enum:Team')])
    io_ = fd.message_type.add(name='InitialObservation')
    _add_fields(io_, [('status', 1, 'enum:Status'), ('world_state_radiant', 2, 'msg:CMsgBotWorldState'),
                      ('world_state_dire', 3, 'msg:CMsgBotWorldState'), ('players', 4, 'msg:Player', 'rep')])
    acts = fd.message_type.add(name='Actions')
    _add_fields(acts, [('actions', 1, 'msg:CMsgBotWorldState.Actions'), ('team_id', 2, 'enum:Team')])
    fd.message_type.add(name='Empty')
    svc = fd.service.add(name='DotaService')
    for name, inp, out in [('reset', 'GameConfig', 'InitialObservation'), ('observe', 'ObserveConfig', 'Observation'),
                           ('act', 'Actions', 'Empty')]:
        svc.method.add(name=name, input_type=f'.{PACKAGE}.{inp}', output_type=f'.{PACKAGE}.{out}')
    return fd


_POOL = descriptor_pool.DescriptorPool()
_FD = _POOL.Add(_build_file())
_CLASSES = message_factory.GetMessageClassesForFiles([_FD.name], _POOL)


def _cls(name):
    return _CLASSES[f'{PACKAGE}.{name}']


def _enum_ns(enum_desc):
    ns = SimpleNamespace()
    for v in enum_desc.values:
        setattr(ns, v.name, v.number)
    return ns


pb = SimpleNamespace(
    CMsgBotWorldState=_cls('CMsgBotWorldState'),
    GameConfig=_cls('GameConfig'),
    HeroPick=_cls('HeroPick'),
    ObserveConfig=_cls('ObserveConfig'),
    Observation=_cls('Observation'),
    InitialObservation=_cls('InitialObservation'),
    Player=_cls('Player'),
    Actions=_cls('Actions'),
    Empty=_cls('Empty'),
    DESCRIPTOR=_FD,
)

_file_enums = {e.name: e for e in _FD.enum_types_by_name.values()}
Team = _enum_ns(_file_enums['Team'])
Status = _enum_ns(_file_enums['Status'])
HostMode = _enum_ns(_file_enums['HostMode'])
GameMode = _enum_ns(_file_enums['GameMode'])
HeroControlMode = _enum_ns(_file_enums['HeroControlMode'])
Hero = _enum_ns(_file_enums['Hero'])
UnitType = _enum_ns(_FD.message_types_by_name['CMsgBotWorldState'].enum_types_by_name['UnitType'])
ActionType = _enum_ns(_FD.message_types_by_name['CMsgBotWorldState'].nested_types_by_name['Action']
                      .enum_types_by_name['Type'])

TEAM_RADIANT = Team.TEAM_RADIANT
TEAM_DIRE = Team.TEAM_DIRE

SERVICE_NAME = f'{PACKAGE}.DotaService'
