"""Actor runtime: players, self-play games and the batched many-game actor.

Reference behaviour (agent.py:267-852) kept:

* per observation, teams alternate observe(team) → per-player reward + action → act(team) (agent.py:800-827);
* shaped rewards (features/reward.py), zero-sum ``enemy`` term after both teams acted (agent.py:829-833);
* rollout every ``rollout_size`` steps and at game end (agent.py:835-847), end-state win/loss/−0.25 (325-337);
* opponent sampling: w.p. 1 − ``latest_weights_prob`` one random team plays the *oldest* stored weights and does
  not roll out (agent.py:760-765, 445-448); synced players follow hot-swapped latest weights mid-game;
* validation mode vs the default bot writes ``game/*`` metrics instead of experience (agent.py:415-434, 905-927);
* creep-spawn sanity check (agent.py:621-627); trajectory canvas (719-741).

MI355X redesign: an :class:`Actor` drives MANY games in lockstep and runs ONE batched policy step per team-turn for
every player that shares a policy (on the GPU, a hipGraph-captured fused step), instead of one batch-1 CPU forward
per player. Experience records also carry the behaviour log-prob, value and LSTM state for PPO/R2D2.
"""
from __future__ import annotations

import logging
import random
import uuid
from collections import Counter
from datetime import datetime
from typing import Callable, Dict, List, NamedTuple, Optional

import numpy as np

from ..constants import (LAYOUT_1V1, OPPOSITE_TEAM, UnitLayout)
from ..features.actions import action_to_pb
from ..features.featurizer import featurize, get_unit
from ..features.reward import end_state_reward, get_reward, pack_rewards
from ..protos import HeroControlMode, Status, TEAM_DIRE, TEAM_RADIANT, pb
from ..transport.codec import Rollout, encode
from ..utils.faults import faults
from .drawing import Drawing

logger = logging.getLogger(__name__)


class Player:
    def __init__(self, game_id: str, player_id: int, team_id: int, hero: int, policy, use_latest_weights: bool,
                 drawing: Drawing, validation: bool, layout: UnitLayout, hidden_size: Optional[int],
                 hidden_stride: int = 0):
        self.game_id = game_id
        self.player_id = player_id
        self.team_id = team_id
        self.hero = hero
        self.policy = policy
        self.use_latest_weights = use_latest_weights
        self.drawing = drawing
        self.validation = validation
        self.layout = layout
        self.hidden_size = hidden_size
        self.hidden_stride = hidden_stride
        self.hidden = None if hidden_size is None else (np.zeros(hidden_size, np.float32),
                                                       np.zeros(hidden_size, np.float32))
        self.creeps_had_spawned = False
        self.total_steps = 0
        self.pending: Optional[Rollout] = None   # rollout waiting for its bootstrap value
        self.rewarded = False
        self.runner = None                       # stateful (GPU-slot) runner holding this player's LSTM state
        self._reset_buffers()

    def _reset_buffers(self):
        self.env, self.units, self.actions, self.masks = [], [], [], []
        self.rewards: List[Dict[str, float]] = []
        self.logp, self.values, self.hiddens = [], [], []

    @property
    def steps_queued(self) -> int:
        return len(self.rewards)

    @property
    def weight_version(self) -> int:
        return getattr(self.policy, 'weight_version', -1)

    def summed_subrewards(self):
        c = Counter()
        for r in self.rewards:
            c.update(r)
        return dict(c)

    def compute_reward(self, prev_obs, obs):
        self.drawing.step(state=obs, team_id=self.team_id, player_id=self.player_id)
        self.rewards.append(get_reward(prev_obs=prev_obs, obs=obs, player_id=self.player_id))

    def featurize(self, obs):
        hero = get_unit(obs, player_id=self.player_id)
        f = featurize(obs, self.player_id, self.team_id, layout=self.layout, hero_unit=hero)
        self.check_creeps(f.n_allied_creep, obs.dota_time)
        return f, hero

    def check_creeps(self, n_allied_creep: int, dota_time: float):
        """Creep-spawn sanity check (agent.py:621-627)."""
        if not self.creeps_had_spawned and dota_time > 0.:
            self.creeps_had_spawned = n_allied_creep > 0
            if not self.creeps_had_spawned:
                raise ValueError(f'Creeps have not spawned at timestep {dota_time}')

    def record(self, f, out, i: int):
        """Store the step's policy input / sampled action / masks / behaviour data (agent.py:702-704)."""
        if self.hidden is not None and self.hidden_stride and (len(self.env) % self.hidden_stride == 0):
            self.hiddens.append(np.stack(self.hidden))
        self.env.append(f.env)
        self.units.append(f.units)
        self.actions.append(out.actions[i])
        self.masks.append(out.masks[i])
        self.logp.append(out.logp[i])
        self.values.append(out.value[i])
        self.total_steps += 1

    def process_endstate(self, end_state):
        if not self.rewards:
            return
        self.rewards[-1]['win'] = end_state_reward(end_state, self.team_id)

    def make_rollout(self, done: bool, canvas) -> Optional[Rollout]:
        if not self.rewards:
            return None
        T = len(self.rewards)
        return Rollout(game_id=self.game_id, team_id=self.team_id, player_id=self.player_id,
                       env=np.stack(self.env[:T]), units=np.stack(self.units[:T]),
                       actions=np.stack(self.actions[:T]).astype(np.uint8), masks=np.stack(self.masks[:T]).astype(np.uint8),
                       rewards=pack_rewards(self.rewards), weight_version=self.weight_version,
                       canvas=None if canvas is None else canvas.copy(),
                       logp=np.asarray(self.logp[:T], np.float32), values=np.asarray(self.values[:T], np.float32),
                       hiddens=np.stack(self.hiddens) if self.hiddens else None, hidden_stride=self.hidden_stride,
                       done=done, layout=self.layout.counts)


class _NativeFeat(NamedTuple):
    """Rows of one native ``featurize_batch`` call (same fields the actor reads from ``Featurized``)."""
    env: np.ndarray
    units: np.ndarray
    handles: np.ndarray
    n_allied_creep: int


class _GameSlot:
    def __init__(self, service, game_id: str):
        self.service = service
        self.game_id = game_id
        self.players: Dict[int, List[Player]] = {TEAM_RADIANT: [], TEAM_DIRE: []}
        self.prev_obs = {}
        self.done = False
        self.end_state = None
        self.opponent_version = None  # snapshot version the non-latest team played (league games)
        self.dota_time = -float('inf')
        self.drawing = Drawing()
        self.n_steps = 0
        self.reward_sum = {TEAM_RADIANT: 0.0, TEAM_DIRE: 0.0}
        self.cur_obs = None


class Actor:
    """Drives ``len(services)`` games in lockstep with one batched policy step per team-turn.

    ``publish(bytes)`` receives encoded experience; ``weight_store`` supplies latest/old policies; ``runner_for``
    maps a policy object to its (cached) batched runner.
    """

    def __init__(self, services, weight_store, runner_for: Callable, publish: Optional[Callable[[bytes], None]],
                 config_fn: Callable, rollout_size: int = 10 ** 9, max_dota_time: float = 600.0,
                 latest_weights_prob: float = 1.0, validation: bool = False, layout: UnitLayout = LAYOUT_1V1,
                 hidden_size: Optional[int] = None, hidden_stride: int = 0, wire: str = 'dcx1',
                 metrics=None, rng: Optional[random.Random] = None, league=None,
                 native_featurize: Optional[bool] = None, featurize_threads: int = 4):
        self.services = list(services)
        self.weight_store = weight_store
        self.runner_for = runner_for
        self.publish = publish
        self.config_fn = config_fn
        self.rollout_size = int(rollout_size)
        self.max_dota_time = max_dota_time
        self.latest_weights_prob = latest_weights_prob
        self.validation = validation
        self.layout = layout
        self.hidden_size = hidden_size
        self.hidden_stride = hidden_stride
        self.wire = wire
        self.metrics = metrics
        self.rng = rng or random.Random()
        self.league = league          # actor/league.py; None = the reference's oldest-snapshot opponent
        # featurize every player of a team-turn in ONE native call (C++ protobuf decode + featurizer, threads,
        # GIL released; bit-identical to features/featurizer.py) instead of a python featurize per player
        from .. import native
        self.native_featurize = native.AVAILABLE if native_featurize is None else bool(native_featurize)
        if self.native_featurize and not native.AVAILABLE:
            raise RuntimeError('native_featurize=True but the native module is not built')
        self.featurize_threads = int(featurize_threads)
        self.slots: List[Optional[_GameSlot]] = [None] * len(self.services)
        self.games_finished = 0
        self.steps_taken = 0
        self.rollouts_sent = 0

    # ----------------------------------------------------------------------------------------------------
    def _start_game(self, i: int):
        service = self.services[i]
        game_id = f"{datetime.now().strftime('%b%d_%H-%M-%S')}_{uuid.uuid4().hex[:6]}"
        slot = _GameSlot(service, game_id)
        use_latest = {TEAM_RADIANT: True, TEAM_DIRE: True}
        if self.rng.random() > self.latest_weights_prob:
            use_latest[self.rng.choice([TEAM_RADIANT, TEAM_DIRE])] = False
        config = self.config_fn()
        response = service.reset_sync(config)
        old_policy = None
        for p_req, p_res in zip(config.hero_picks, response.players):
            if p_res.is_bot and p_req.control_mode == HeroControlMode.HERO_CONTROL_MODE_CONTROLLED:
                latest = use_latest[p_res.team_id]
                if latest and not self.validation:
                    policy = self.weight_store.latest_policy     # synced: sees hot-swapped weights mid-game
                elif self.validation:
                    policy = self.weight_store.policy_for(self.weight_store.latest_weights())
                else:
                    if old_policy is None:
                        if self.league is not None:
                            vs = self.league.sample()
                            old_policy = self.league.policy(vs)
                        else:
                            vs = self.weight_store.oldest_weights()
                            old_policy = self.weight_store.policy_for(vs)
                        slot.opponent_version = int(vs[0])
                    policy = old_policy
                slot.players[p_res.team_id].append(Player(
                    game_id, p_res.id, p_res.team_id, p_res.hero, policy, latest, slot.drawing, self.validation,
                    self.layout, self.hidden_size, self.hidden_stride))
        slot.prev_obs = {TEAM_RADIANT: response.world_state_radiant, TEAM_DIRE: response.world_state_dire}
        self.slots[i] = slot

    def _send(self, player: Player, rollout: Rollout):
        if self.publish is None or self.validation or not player.use_latest_weights:
            return
        body = encode(rollout) if self.wire == 'dcx1' else __import__('pickle').dumps(rollout.to_reference_dict())
        f = faults()
        if f.active:
            if f.should('drop_xp'):
                return
            if f.should('corrupt_xp'):
                body = f.corrupt(body)
        self.publish(body)
        self.rollouts_sent += 1

    def _rollout(self, player: Player, slot: _GameSlot, done: bool, bootstrap: float = 0.0):
        r = player.make_rollout(done, slot.drawing.canvas)
        player._reset_buffers()
        if r is None:
            return
        if done:
            self._send(player, r)
        else:
            player.pending = r     # published once the next step's value (bootstrap) is known

    def _finish(self, slot: _GameSlot):
        if self.league is not None and slot.opponent_version is not None:
            latest_team = next((t for t in (TEAM_RADIANT, TEAM_DIRE)
                                if any(p.use_latest_weights for p in slot.players[t])), None)
            if latest_team is not None:
                won = {Status.RADIANT_WIN: TEAM_RADIANT, Status.DIRE_WIN: TEAM_DIRE}.get(slot.end_state)
                self.league.record(slot.opponent_version, 0.5 if won is None else float(won == latest_team))
        for team in (TEAM_RADIANT, TEAM_DIRE):
            for p in slot.players[team]:
                if p.runner is not None:
                    p.runner.release(id(p))
                    p.runner = None
                p.process_endstate(slot.end_state)
                if p.pending is not None:
                    p.pending.bootstrap_value = 0.0
                    self._send(p, p.pending)
                    p.pending = None
                if self.validation:
                    self._write_validation(p)
                else:
                    self._rollout(p, slot, done=True)
        self.games_finished += 1

    def _write_validation(self, p: Player):
        if self.metrics is None:
            return
        it = p.weight_version
        sub = p.summed_subrewards()
        self.metrics.add_image('game/canvas', p.drawing.canvas, it)
        vals = {'game/steps': p.steps_queued, 'game/rewards_sum': sum(sub.values())}
        vals.update({f'game/rewards_{k}': v for k, v in sub.items()})
        self.metrics.add_scalars(vals, it)
        self.metrics.flush()

    # ----------------------------------------------------------------------------------------------------
    def _team_turn(self, team: int, active: List[int]):
        batch = []   # (slot, player, featurized, hero)
        for i in active:
            slot = self.slots[i]
            resp = slot.service.observe_sync(pb.ObserveConfig(team_id=team))
            if resp.status != Status.OK:
                slot.end_state = resp.status
                slot.done = True
                continue
            obs = resp.world_state
            slot.dota_time = obs.dota_time
            slot.cur_obs = obs
            for p in slot.players[team]:
                p.compute_reward(prev_obs=slot.prev_obs[team], obs=obs)
                slot.reward_sum[team] += sum(p.rewards[-1].values())
                p.rewarded = True
                if self.native_featurize:
                    batch.append((slot, p, obs, None))
                else:
                    f, hero = p.featurize(obs)
                    batch.append((slot, p, f, hero))
        if self.native_featurize and batch:
            batch = self._featurize_native(batch)
        # one batched policy step per distinct policy object
        # (a player bound to a stateful runner stays with it: its recurrent state lives there)
        groups: Dict[int, List[int]] = {}
        for k, (_, p, _, _) in enumerate(batch):
            groups.setdefault(id(p.runner) if p.runner is not None else id(p.policy), []).append(k)
        actions_by_slot: Dict[int, list] = {}
        for _, idxs in groups.items():
            pol = batch[idxs[0]][1].policy
            runner = batch[idxs[0]][1].runner or self.runner_for(pol)
            env = np.stack([batch[k][2].env for k in idxs])
            units = np.stack([batch[k][2].units for k in idxs])
            handles = np.stack([batch[k][2].handles for k in idxs])
            hidden = new_hidden = None
            if getattr(runner, 'stateful', False):
                # LSTM state stays in the runner's device slots; fetch it only where the record stores it
                players = [batch[k][1] for k in idxs]
                need = [p.hidden is not None and bool(p.hidden_stride) and len(p.env) % p.hidden_stride == 0
                        for p in players]
                out, prev = runner.step_players(env, units, handles, [id(p) for p in players], need)
                for j, p in enumerate(players):
                    p.runner = runner
                    if prev is not None and j in prev:
                        p.hidden = prev[j]
            else:
                if pol.is_recurrent:
                    hidden = (np.stack([batch[k][1].hidden[0] for k in idxs]),
                              np.stack([batch[k][1].hidden[1] for k in idxs]))
                out, new_hidden = runner.step(env, units, handles, hidden)
            for j, k in enumerate(idxs):
                slot, p, f, hero = batch[k]
                if p.pending is not None:          # truncated rollout: bootstrap from this step's value
                    p.pending.bootstrap_value = float(out.value[j])
                    self._send(p, p.pending)
                    p.pending = None
                p.record(f, out, j)
                if new_hidden is not None:
                    p.hidden = (new_hidden[0][j], new_hidden[1][j])
                a = action_to_pb(out.action_dict(j), hero.location, f.handles, player_id=p.player_id)
                actions_by_slot.setdefault(id(slot), []).append(a)
        for i in active:
            slot = self.slots[i]
            if slot.done:
                continue
            acts = pb.CMsgBotWorldState.Actions(actions=actions_by_slot.get(id(slot), []))
            acts.dota_time = slot.cur_obs.dota_time
            slot.service.act_sync(pb.Actions(actions=acts, team_id=team))
            slot.prev_obs[team] = slot.cur_obs

    def _featurize_native(self, batch):
        """(slot, player, obs, None) → (slot, player, features, hero unit): one serialisation per observation, one
        native call for all players of the team-turn."""
        from .. import native
        wire, states = {}, []
        for _, _, obs, _ in batch:
            b = wire.get(id(obs))
            if b is None:
                b = wire[id(obs)] = obs.SerializeToString()
            states.append(b)
        env, units, handles, ncreep = native.featurize_batch(
            states, [p.player_id for _, p, _, _ in batch], [p.team_id for _, p, _, _ in batch],
            list(self.layout.counts), self.featurize_threads)
        out = []
        for k, (slot, p, obs, _) in enumerate(batch):
            hero = get_unit(obs, player_id=p.player_id)
            p.check_creeps(int(ncreep[k]), obs.dota_time)
            out.append((slot, p, _NativeFeat(env[k], units[k], handles[k], int(ncreep[k])), hero))
        return out

    def step(self):
        """One observation interval for every game (both teams), starting/finishing games as needed."""
        if faults().should('actor_crash'):
            raise RuntimeError('injected actor crash (DCA_FAULTS actor_crash)')
        for i in range(len(self.slots)):
            if self.slots[i] is None:
                self._start_game(i)
        active = [i for i, s in enumerate(self.slots) if not s.done]
        for i in active:
            self.slots[i].reward_sum = {TEAM_RADIANT: 0.0, TEAM_DIRE: 0.0}
            for ps in self.slots[i].players.values():
                for p in ps:
                    p.rewarded = False
        for team in (TEAM_RADIANT, TEAM_DIRE):
            self._team_turn(team, [i for i in active if not self.slots[i].done])
        for i in active:
            slot = self.slots[i]
            if not self.validation:
                # zero-sum shaping: subtract the opponent team's summed step reward (agent.py:829-833)
                for team in (TEAM_RADIANT, TEAM_DIRE):
                    for p in slot.players[team]:
                        if p.rewarded:
                            p.rewards[-1]['enemy'] = -slot.reward_sum[OPPOSITE_TEAM[team]]
                for p in [*slot.players[TEAM_RADIANT], *slot.players[TEAM_DIRE]]:
                    if p.steps_queued > 0 and p.steps_queued % self.rollout_size == 0:
                        self._rollout(p, slot, done=False)
            slot.n_steps += 1
            self.steps_taken += sum(len(v) for v in slot.players.values())
            if slot.done or slot.dota_time >= self.max_dota_time:
                self._finish(slot)
                self.slots[i] = None

    def run(self, n_games: Optional[int] = None, max_steps: Optional[int] = None):
        steps = 0
        while (n_games is None or self.games_finished < n_games) and (max_steps is None or steps < max_steps):
            self.step()
            steps += 1
        return self.games_finished
