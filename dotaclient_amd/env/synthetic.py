"""SyntheticDotaService: a deterministic 1v1-mid (and 5v5) lane simulator behind the DotaService contract.

The reference talks to the real Dota 2 engine through ``dotaservice`` over gRPC (reference agent.py:772,
805, 825). Neither is available here, so this module provides a self-contained, seeded game
that produces ``CMsgBotWorldState`` protobufs with every field the featurizer / reward function read:

* two controlled Nevermores (player 0 radiant, player 5 dire) plus idle Snipers at the fountains
  (reference agent.py:930-949), or 5 controlled heroes per side in 5v5 mode;
* creep waves every 30 s (3 melee + 1 ranged) walking the mid lane, creep/tower aggro, ranged projectiles
  (``incoming_tracking_projectiles``), tower ``anim_activity`` 1500 idle / 1503 attacking (agent.py:548);
* XP sharing, last hits, denies, kills/deaths, respawn timers, 1v1 end conditions (2 kills or the T1 tower);
* per-team fog of war (vision radius around allied units);
* a scripted ``HERO_CONTROL_MODE_DEFAULT`` bot for the validation runner (agent.py:905-927).

The service is advanced after *both* teams have acted (the reference loop is observe(R) → act(R) →
observe(D) → act(D), agent.py:802-827). One observation = ``ticks_per_observation`` ticks at 30 tps.

This module is also the ORACLE of the native vectorised engine (``native/vecenv.h``, :mod:`dotaclient_amd.env.vec`),
which reproduces it bit for bit: CPython's MT19937 seeding and ``random()``, dict-ordered unit iteration, and
geometry written with operations that are correctly rounded in both languages (``_dist`` is sqrt(dx²+dy²), not
``math.hypot``, whose CPython algorithm differs from libm's).
"""
from __future__ import annotations

import asyncio
import math
import random
from dataclasses import dataclass, field
from typing import Dict, List, Optional

from ..constants import TICKS_PER_SECOND, level_from_total_xp
from ..protos import (ActionType, HeroControlMode, Status, TEAM_DIRE, TEAM_RADIANT, UnitType, pb)

# --- map geometry (world units), roughly the Dota mid lane -----------------------------------------------
FOUNTAIN = {TEAM_RADIANT: (-6700.0, -6200.0), TEAM_DIRE: (6600.0, 6000.0)}
CREEP_SPAWN = {TEAM_RADIANT: (-4700.0, -4300.0), TEAM_DIRE: (4000.0, 3600.0)}
T1_MID = {TEAM_RADIANT: (-1544.0, -1408.0), TEAM_DIRE: (524.0, 652.0)}
ANCIENT = {TEAM_RADIANT: (-5400.0, -5000.0), TEAM_DIRE: (5200.0, 4700.0)}
OPP = {TEAM_RADIANT: TEAM_DIRE, TEAM_DIRE: TEAM_RADIANT}

def _hypot(dx: float, dy: float) -> float:
    return math.sqrt(dx * dx + dy * dy)


ANIM_TOWER_IDLE = 1500
ANIM_TOWER_ATTACK = 1503
VISION_RADIUS = 1800.0
XP_RADIUS = 1300.0


@dataclass
class SimUnit:
    handle: int
    unit_type: int
    name: str
    team_id: int
    x: float
    y: float
    hp: float
    hp_max: float
    damage: float
    attack_range: float
    attack_period: float
    speed: float
    player_id: int = -1
    mana: float = 0.0
    mana_max: float = 0.0
    level: int = 1
    total_xp: float = 0.0
    facing: float = 0.0
    alive: bool = True
    cooldown: float = 0.0
    target: int = 0            # attack target handle (0 = none)
    last_hits: int = 0
    denies: int = 0
    respawn_at: float = 0.0
    move_to: Optional[tuple] = None
    control: int = HeroControlMode.HERO_CONTROL_MODE_IDLE
    projectiles: List[tuple] = field(default_factory=list)   # (caster_handle, is_attack) arriving this obs
    invulnerable: bool = False
    last_attacker_player: int = -1


@dataclass
class PlayerStats:
    player_id: int
    team_id: int
    hero_id: int
    kills: int = 0
    deaths: int = 0


class SyntheticGame:
    """The core simulator (synchronous)."""

    def __init__(self, config, seed: Optional[int] = None, start_time: float = -10.0,
                 fog_of_war: bool = True):
        self.config = config
        self.rng = random.Random(seed if seed is not None else (config.seed or 0))
        self.dt = config.ticks_per_observation / TICKS_PER_SECOND if config.ticks_per_observation else 0.5
        self.dota_time = start_time
        self.fog = fog_of_war
        self.units: Dict[int, SimUnit] = {}
        self.players: Dict[int, PlayerStats] = {}
        self._next_handle = 100
        self.status = Status.OK
        self._pending: Dict[int, list] = {}
        self._last_wave = None
        self.n_steps = 0
        self._setup()

    # -------------------------------------------------------------------------------------------------
    def _handle(self) -> int:
        self._next_handle += 1
        return self._next_handle

    def _setup(self):
        pid = {TEAM_RADIANT: 0, TEAM_DIRE: 5}
        for pick in self.config.hero_picks:
            team = pick.team_id
            p = pid[team]
            pid[team] += 1
            controlled = pick.control_mode != HeroControlMode.HERO_CONTROL_MODE_IDLE
            fx, fy = FOUNTAIN[team]
            # Controlled heroes start near their tower; idle ones stay at the fountain.
            if controlled:
                tx, ty = T1_MID[team]
                d = 400.0 if team == TEAM_RADIANT else -400.0
                fx, fy = tx - d + self.rng.uniform(-100, 100), ty - d + self.rng.uniform(-100, 100)
            hero_name = 'npc_dota_hero_nevermore' if pick.hero_id == 11 else 'npc_dota_hero_sniper'
            u = SimUnit(handle=self._handle(), unit_type=UnitType.HERO, name=hero_name, team_id=team,
                        x=fx, y=fy, hp=600.0, hp_max=600.0, damage=55.0, attack_range=500.0,
                        attack_period=1.6, speed=315.0, player_id=p, mana=290.0, mana_max=290.0,
                        facing=45.0 if team == TEAM_RADIANT else 225.0, control=pick.control_mode)
            self.units[u.handle] = u
            self.players[p] = PlayerStats(player_id=p, team_id=team, hero_id=pick.hero_id)
        for team in (TEAM_RADIANT, TEAM_DIRE):
            side = 'goodguys' if team == TEAM_RADIANT else 'badguys'
            tx, ty = T1_MID[team]
            t = SimUnit(handle=self._handle(), unit_type=UnitType.TOWER, name=f'npc_dota_{side}_tower1_mid',
                        team_id=team, x=tx, y=ty, hp=1800.0, hp_max=1800.0, damage=100.0, attack_range=700.0,
                        attack_period=1.0, speed=0.0)
            self.units[t.handle] = t
            # Tier-2 tower (not featurized: the reference only uses the "1_mid" tower, agent.py:479).
            t2 = SimUnit(handle=self._handle(), unit_type=UnitType.TOWER, name=f'npc_dota_{side}_tower2_mid',
                         team_id=team, x=tx * 2.2, y=ty * 2.2, hp=1800.0, hp_max=1800.0, damage=100.0,
                         attack_range=700.0, attack_period=1.0, speed=0.0, invulnerable=True)
            self.units[t2.handle] = t2

    def _spawn_wave(self):
        for team in (TEAM_RADIANT, TEAM_DIRE):
            sx, sy = CREEP_SPAWN[team]
            side = 'goodguys' if team == TEAM_RADIANT else 'badguys'
            for k in range(4):
                ranged = k == 3
                c = SimUnit(handle=self._handle(), unit_type=UnitType.LANE_CREEP,
                            name=f'npc_dota_creep_{side}_{"ranged" if ranged else "melee"}', team_id=team,
                            x=sx + self.rng.uniform(-80, 80), y=sy + self.rng.uniform(-80, 80),
                            hp=300.0 if ranged else 550.0, hp_max=300.0 if ranged else 550.0,
                            damage=24.0 if ranged else 21.0, attack_range=500.0 if ranged else 100.0,
                            attack_period=1.0, speed=325.0,
                            facing=45.0 if team == TEAM_RADIANT else 225.0)
                self.units[c.handle] = c

    # -------------------------------------------------------------------------------------------------
    @staticmethod
    def _dist(a: SimUnit, b: SimUnit) -> float:
        return _hypot(a.x - b.x, a.y - b.y)

    def _move_towards(self, u: SimUnit, tx: float, ty: float, dt: float):
        dx, dy = tx - u.x, ty - u.y
        d = _hypot(dx, dy)
        if d < 1e-3:
            return
        step = min(d, u.speed * dt)
        u.x += dx / d * step
        u.y += dy / d * step
        u.facing = (math.degrees(math.atan2(dy, dx)) + 360.0) % 360.0
        u.x = max(-8000.0, min(8000.0, u.x))
        u.y = max(-8000.0, min(8000.0, u.y))

    def _alive_enemies(self, team):
        return [v for v in self.units.values() if v.alive and v.team_id != team and not v.invulnerable]

    def _nearest(self, u: SimUnit, cands, max_range: float):
        best, bd = None, max_range
        for v in cands:
            d = self._dist(u, v)
            if d <= bd:
                best, bd = v, d
        return best

    def _attack(self, attacker: SimUnit, target: SimUnit):
        attacker.target = target.handle
        attacker.facing = (math.degrees(math.atan2(target.y - attacker.y, target.x - attacker.x)) + 360.0) % 360.0
        if attacker.cooldown > 0:
            return
        attacker.cooldown = attacker.attack_period
        if attacker.attack_range > 150:
            target.projectiles.append((attacker.handle, True))
        dmg = attacker.damage * self.rng.uniform(0.9, 1.1)
        target.hp -= dmg
        if attacker.unit_type == UnitType.HERO:
            target.last_attacker_player = attacker.player_id
        if target.hp <= 0:
            self._kill(target, attacker)

    def _kill(self, target: SimUnit, killer: SimUnit):
        target.alive = False
        target.hp = 0.0
        target.target = 0
        if target.unit_type == UnitType.HERO:
            self.players[target.player_id].deaths += 1
            target.respawn_at = self.dota_time + 6.0 + 2.0 * target.level
            kp = killer.player_id if killer.unit_type == UnitType.HERO else target.last_attacker_player
            if kp >= 0 and self.players[kp].team_id != target.team_id:
                self.players[kp].kills += 1
            self._share_xp(target, 100 + 20 * target.level)
        elif target.unit_type == UnitType.LANE_CREEP:
            if killer.unit_type == UnitType.HERO:
                if killer.team_id != target.team_id:
                    killer.last_hits += 1
                else:
                    killer.denies += 1
            if killer.team_id != target.team_id:
                self._share_xp(target, 69.0 if 'ranged' in target.name else 57.0)
        elif target.unit_type == UnitType.TOWER and 'tower1_mid' in target.name:
            self.status = Status.DIRE_WIN if target.team_id == TEAM_RADIANT else Status.RADIANT_WIN

    def _share_xp(self, dead: SimUnit, xp: float):
        heroes = [h for h in self.units.values() if h.unit_type == UnitType.HERO and h.alive
                  and h.team_id != dead.team_id and self._dist(h, dead) <= XP_RADIUS]
        for h in heroes:
            h.total_xp += xp / len(heroes)
            lvl, _ = level_from_total_xp(h.total_xp)
            if lvl > h.level:
                h.hp_max += 20.0 * (lvl - h.level)
                h.damage += 3.0 * (lvl - h.level)
                h.level = lvl

    # -------------------------------------------------------------------------------------------------
    def _apply_action(self, hero: SimUnit, action):
        t = action.actionType
        if t == ActionType.DOTA_UNIT_ORDER_MOVE_DIRECTLY or t == ActionType.DOTA_UNIT_ORDER_MOVE_TO_POSITION:
            loc = action.moveDirectly.location if action.HasField('moveDirectly') else action.moveToLocation.location
            hero.move_to = (loc.x, loc.y)
            hero.target = 0
        elif t == ActionType.DOTA_UNIT_ORDER_ATTACK_TARGET:
            tgt = self.units.get(action.attackTarget.target)
            hero.move_to = None
            hero.target = tgt.handle if (tgt is not None and tgt.alive) else 0
        else:  # NONE / STOP
            hero.move_to = None
            hero.target = 0

    def _default_bot(self, hero: SimUnit):
        """Scripted laning bot (HERO_CONTROL_MODE_DEFAULT): last-hit/deny, retreat on low hp."""
        if hero.hp < 0.3 * hero.hp_max:
            hero.move_to = T1_MID[hero.team_id]
            hero.target = 0
            return
        cands = [v for v in self.units.values() if v.alive and v.unit_type == UnitType.LANE_CREEP
                 and self._dist(hero, v) <= 900.0]
        enemies = [v for v in cands if v.team_id != hero.team_id]
        allies = [v for v in cands if v.team_id == hero.team_id and v.hp < 0.5 * v.hp_max]
        lowest = min(enemies + allies, key=lambda v: v.hp, default=None)
        if lowest is not None and lowest.hp <= hero.damage * 1.3:
            hero.target, hero.move_to = lowest.handle, None
        elif enemies:
            # Hold position behind the allied creeps.
            ex = sum(v.x for v in enemies) / len(enemies)
            ey = sum(v.y for v in enemies) / len(enemies)
            d = 450.0 if hero.team_id == TEAM_RADIANT else -450.0
            hero.move_to, hero.target = (ex - d, ey - d), 0
        else:
            hero.move_to, hero.target = (T1_MID[hero.team_id][0] * 0.3, T1_MID[hero.team_id][1] * 0.3), 0

    def step(self, actions_by_team: Dict[int, list]):
        """Advance one observation interval with the given per-team Action lists."""
        if self.status != Status.OK:
            return
        dt = self.dt
        for u in self.units.values():
            u.projectiles = []
        heroes = {u.player_id: u for u in self.units.values() if u.unit_type == UnitType.HERO}
        for team, actions in actions_by_team.items():
            for a in actions:
                h = heroes.get(a.player)
                if h is not None and h.alive and h.team_id == team:
                    self._apply_action(h, a)
        # Creep waves every 30 s starting at 0:00.
        wave = math.floor(self.dota_time / 30.0) if self.dota_time >= 0 else None
        if wave is not None and wave != self._last_wave:
            self._last_wave = wave
            self._spawn_wave()
        for u in list(self.units.values()):
            u.cooldown = max(0.0, u.cooldown - dt)
            if not u.alive:
                if u.unit_type == UnitType.HERO and self.dota_time >= u.respawn_at:
                    u.alive, u.hp = True, u.hp_max
                    u.x, u.y = FOUNTAIN[u.team_id]
                    u.move_to, u.target = None, 0
                continue
            if u.unit_type == UnitType.HERO:
                if u.control == HeroControlMode.HERO_CONTROL_MODE_IDLE:
                    continue
                if u.control == HeroControlMode.HERO_CONTROL_MODE_DEFAULT:
                    self._default_bot(u)
                u.hp = min(u.hp_max, u.hp + 1.5 * dt)
                if u.target:
                    tgt = self.units.get(u.target)
                    if tgt is None or not tgt.alive or tgt.invulnerable:
                        u.target = 0
                    elif self._dist(u, tgt) <= u.attack_range:
                        self._attack(u, tgt)
                    else:
                        self._move_towards(u, tgt.x, tgt.y, dt)
                elif u.move_to is not None:
                    self._move_towards(u, u.move_to[0], u.move_to[1], dt)
            elif u.unit_type == UnitType.LANE_CREEP:
                enemies = self._alive_enemies(u.team_id)
                tgt = self._nearest(u, [v for v in enemies if v.unit_type != UnitType.HERO], 500.0) or \
                    self._nearest(u, enemies, 500.0)
                if tgt is not None:
                    if self._dist(u, tgt) <= u.attack_range + 40.0:
                        self._attack(u, tgt)
                    else:
                        u.target = 0
                        self._move_towards(u, tgt.x, tgt.y, dt)
                else:
                    u.target = 0
                    ex, ey = ANCIENT[OPP[u.team_id]]
                    self._move_towards(u, ex, ey, dt)
            elif u.unit_type == UnitType.TOWER and not u.invulnerable:
                enemies = self._alive_enemies(u.team_id)
                tgt = self._nearest(u, [v for v in enemies if v.unit_type != UnitType.HERO], u.attack_range) or \
                    self._nearest(u, enemies, u.attack_range)
                if tgt is not None:
                    self._attack(u, tgt)
                else:
                    u.target = 0
        # Remove creeps that died before this step (dead creeps linger for one observation).
        for h in [h for h, u in self.units.items() if not u.alive and u.unit_type == UnitType.LANE_CREEP
                  and u.respawn_at == -1.0]:
            del self.units[h]
        for u in self.units.values():
            if not u.alive and u.unit_type == UnitType.LANE_CREEP:
                u.respawn_at = -1.0
        # 1v1 mid: first to 2 kills wins.
        for p in self.players.values():
            if p.kills >= 2 and self._is_1v1():
                self.status = Status.RADIANT_WIN if p.team_id == TEAM_RADIANT else Status.DIRE_WIN
        self.dota_time += dt
        self.n_steps += 1

    def _is_1v1(self) -> bool:
        return sum(1 for u in self.units.values() if u.unit_type == UnitType.HERO
                   and u.control != HeroControlMode.HERO_CONTROL_MODE_IDLE) <= 2

    # -------------------------------------------------------------------------------------------------
    def world_state(self, team_id: int):
        ws = pb.CMsgBotWorldState(team_id=team_id, dota_time=self.dota_time, game_time=self.dota_time + 90.0)
        for p in self.players.values():
            ws.players.add(player_id=p.player_id, team_id=p.team_id, hero_id=p.hero_id, kills=p.kills,
                           deaths=p.deaths)
        allies = [u for u in self.units.values() if u.team_id == team_id and u.alive]
        for u in self.units.values():
            if self.fog and u.team_id != team_id and u.unit_type != UnitType.TOWER:
                if not any(_hypot(a.x - u.x, a.y - u.y) <= VISION_RADIUS for a in allies):
                    continue
            m = ws.units.add(handle=u.handle, unit_type=u.unit_type, name=u.name, team_id=u.team_id,
                             level=u.level, is_alive=u.alive, player_id=u.player_id, facing=u.facing,
                             health=int(max(0.0, u.hp)), health_max=int(u.hp_max), mana=u.mana,
                             mana_max=u.mana_max, attack_range=int(u.attack_range), attack_damage=int(u.damage),
                             attack_target_handle=u.target, is_invulnerable=u.invulnerable,
                             last_hits=u.last_hits, denies=u.denies)
            m.location.x, m.location.y, m.location.z = u.x, u.y, 128.0
            if u.unit_type == UnitType.TOWER:
                m.anim_activity = ANIM_TOWER_ATTACK if u.target else ANIM_TOWER_IDLE
            if u.unit_type == UnitType.HERO:
                lvl, need = level_from_total_xp(u.total_xp)
                m.xp_needed_to_level = need
            for caster, is_attack in u.projectiles:
                m.incoming_tracking_projectiles.add(caster_handle=caster, is_attack=is_attack)
        return ws


class SyntheticDotaService:
    """Async DotaService stand-in with the reference's ``reset/observe/act`` contract (agent.py:772-825)."""

    def __init__(self, seed: int = 0, start_time: float = -10.0, fog_of_war: bool = True):
        self.seed = seed
        self.start_time = start_time
        self.fog = fog_of_war
        self.game: Optional[SyntheticGame] = None
        self._acted: Dict[int, list] = {}
        self.n_resets = 0

    # sync API -------------------------------------------------------------------------------------
    def reset_sync(self, config):
        seed = config.seed if config.seed else self.seed + self.n_resets
        self.n_resets += 1
        self.game = SyntheticGame(config, seed=seed, start_time=self.start_time, fog_of_war=self.fog)
        self._acted = {}
        players = []
        for p in self.game.players.values():
            pick_bot = True
            players.append(pb.Player(id=p.player_id, hero=p.hero_id, is_bot=pick_bot, team_id=p.team_id))
        return pb.InitialObservation(status=Status.OK, world_state_radiant=self.game.world_state(TEAM_RADIANT),
                                     world_state_dire=self.game.world_state(TEAM_DIRE), players=players)

    def observe_sync(self, observe_config):
        team = observe_config.team_id
        return pb.Observation(status=self.game.status, world_state=self.game.world_state(team), team_id=team)

    def act_sync(self, actions_msg):
        self._acted[actions_msg.team_id] = list(actions_msg.actions.actions)
        if TEAM_RADIANT in self._acted and TEAM_DIRE in self._acted:
            self.game.step(self._acted)
            self._acted = {}
        return pb.Empty()

    # async API (what the reference's Game.play awaits) ----------------------------------------------
    async def reset(self, config):
        return self.reset_sync(config)

    async def observe(self, observe_config):
        return self.observe_sync(observe_config)

    async def act(self, actions_msg):
        return self.act_sync(actions_msg)


def run_sync(coro):
    """Drive a coroutine from sync code (tests / scripts)."""
    return asyncio.run(coro)
