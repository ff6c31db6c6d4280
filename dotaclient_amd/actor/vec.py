"""High-throughput self-play actor: the native vectorised runtime + one GPU-resident batched policy.

The reference actor is one process per game: protobuf observation → featurize → ``policy.single`` → sample →
``action_to_pb`` → gRPC, one player at a time (agent.py:641-660, 768-835). :class:`~dotaclient_amd.actor.game.Actor`
keeps that structure (any DotaService, protobuf all the way). :class:`VecActor` is the MI355X-shaped runtime for
the synthetic engine: thousands of games live in C++ (:class:`dotaclient_amd.native.VecEnv`, ``native/vecenv.h`` —
engine step, featurize, shaped reward, trajectory canvas, trajectory recording, action decoding and DCX1 rollout
encoding on a thread pool, bit-identical to the python Actor's rollouts, ``tests/test_vecenv.py``) and every
player of every game is stepped by ONE hipGraph replay of :class:`~dotaclient_amd.actor.batched.GpuActorPolicy`
(LSTM state resident in device slots).

The games are split into ``groups`` (default 2) of equal size, each with its own VecEnv and GPU policy, and the
groups are software-pipelined: while the GPU steps group ``k`` the host threads act/observe group ``k+1``, so the
host engine work and the GPU step overlap.

League play (reference mini-league, agent.py:760-765, and :class:`~dotaclient_amd.actor.league.League`): with
probability ``1 − latest_weights_prob`` one team of a new game plays an old snapshot and does not roll out. A game
keeps its opponent snapshot for its whole length: each group holds up to two opponent policies (same slots, same
staged observations, their own LSTM state) — new opponent games join the *current* one; every
``opponent_refresh`` finished opponent games a fresh snapshot is sampled into the *other* one once its games have
drained, and it becomes current. Results are fed back to the league per game.
"""
from __future__ import annotations

import logging
import time
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from ..protos import Status
from .batched import make_slot_policy

logger = logging.getLogger(__name__)

MODES = {'1v1': 0, '5v5': 1, 'vs_default_bot': 2, 'vs_default_bot_5v5': 3}


class _Opponent:
    def __init__(self, gp):
        self.gp = gp
        self.version: Optional[int] = None
        self.games = 0          # games in flight bound to this policy


class _Group:
    def __init__(self, actor: 'VecActor', index: int, n_games: int, seed: int):
        a = actor
        self.raw = a.raw
        self.ve = a._native.VecEnv(n_games, mode=MODES[a.mode], seed=seed, max_dota_time=a.max_dota_time,
                                   rollout_size=a.rollout_size, hidden_stride=a.hidden_stride if a.H else 0,
                                   hidden_size=a.H, counts=list(a.cfg.layout.counts), threads=a.threads,
                                   latest_weights_prob=a.latest_weights_prob, start_time=a.start_time, fog=a.fog,
                                   tag=f'{a.tag}{index}', stagger=a.stagger, wire=a.wire, raw=self.raw)
        if a.ring_sink is not None:
            self.ve.set_ring_sink(a.ring_sink.ring, -1.0, bool(a.ring_sink.drop_oldest))
        self.S = self.ve.slots
        self.ppg = self.ve.players_per_game
        self.gp = make_slot_policy(a.policy, self.S, device=a.device, seed=seed, **a._policy_kw())
        self.env = self.gp.h_env.numpy()
        if self.raw:
            # raw unit records staged for the GPU featurizer; the host keeps only the handles (action targets)
            self.hero = self.gp.h_hero.numpy()
            self.rawbuf = self.gp.h_raw.numpy()
            self.handles = np.full((self.S, a.cfg.layout.max_units), -1, np.int64)
        else:
            self.units = self.gp.h_units.numpy()
            self.handles = self.gp.h_handles.numpy()
        self.active = np.zeros(self.S, np.uint8)
        self.opp: List[_Opponent] = []
        self.cur_opp = 0
        self.game_opp = np.full(n_games, -1, np.int64)    # opponent policy index per game (-1: none)
        self.refresh_mark = 0
        self.seed = seed
        self.version: Optional[int] = None
        self.need = np.zeros(0, np.int32)
        self.opp_rows: Dict[int, np.ndarray] = {}


class VecActor:
    """``n_games`` synthetic games stepped in lockstep by one batched GPU policy per group.

    ``publish(bytes)`` receives DCX1 rollouts (the reference's ``experience`` queue); ``weight_store`` supplies the
    latest weights (hot-swapped into the captured graphs between steps) and the snapshot history for opponents.
    ``ring_sink`` (a :class:`~dotaclient_amd.transport.shm.ShmBroker`): the native engine's worker threads encode
    every finished rollout straight into a reserved region of that node ring instead (``publish`` is then unused):
    no intermediate string, no Python bytes object built under the GIL, no second copy by a publish call — ≈0.5 ms
    of this process's main thread per whole-game rollout.
    ``raw`` (default: on with a fused GPU policy step): the engine stages compact raw unit records instead of
    features (features/raw.py; the fp8 step their 16-byte form), the step's first kernel featurizes them
    (ops/csrc/featurize.hip), and the rollouts carry the records (``units_raw`` / ``hero``) for the learner's device
    featurization.
    """

    def __init__(self, weight_store, n_games: int, publish: Optional[Callable[[bytes], None]], device='cuda',
                 mode: str = '1v1', seed: int = 0, rollout_size: int = 10 ** 9, max_dota_time: float = 600.0,
                 latest_weights_prob: float = 1.0, hidden_stride: int = 256, threads: int = 8, groups: int = 2,
                 league=None, opponent_refresh: int = 64, start_time: float = -10.0,
                 fog: bool = True, tag: str = 'vec', stagger: bool = False, wire: bool = False,
                 precision: str = 'bf16', ring_sink=None, raw: Optional[bool] = None):
        from .. import native
        if not native.AVAILABLE:
            raise RuntimeError('VecActor needs the native module (python -m dotaclient_amd.native.build)')
        if mode not in MODES:
            raise ValueError(f'mode must be one of {sorted(MODES)}')
        self._native = native._native
        self.store = weight_store
        self.policy = weight_store.latest_policy
        self.cfg = self.policy.config
        if (mode in ('5v5', 'vs_default_bot_5v5')) != (self.cfg.layout.counts[0] > 1):
            raise ValueError(f'mode {mode!r} does not match the policy layout {self.cfg.layout.counts}')
        self.publish = publish
        self.ring_sink = ring_sink
        self.device = torch.device(device)
        self.mode = mode
        self.rollout_size = int(rollout_size)
        self.max_dota_time = float(max_dota_time)
        self.latest_weights_prob = float(latest_weights_prob)
        self.hidden_stride = int(hidden_stride)
        self.H = self.cfg.hidden if self.cfg.rnn == 'lstm' else 0
        self.threads = int(threads)
        self.league = league
        self.opponent_refresh = int(opponent_refresh)
        self.start_time = float(start_time)
        self.fog = bool(fog)
        self.tag = tag
        self.stagger = bool(stagger)     # staggered first games (no lockstep bursts of whole-game rollouts)
        # observations as serialised CMsgBotWorldState protobufs through the native wire decoder + featurizer, and
        # orders as Actions protobufs (the reference actor's observe / act path, agent.py:805-825)
        self.wire = bool(wire)
        # policy-step precision: bf16 (GpuActorPolicy), fp32 (F32ActorPolicy, the reference actor's precision) or fp8
        # (Fp8ActorPolicy, BASELINE config 5)
        from .batched import ACTOR_PRECISIONS
        if precision not in ACTOR_PRECISIONS:
            raise ValueError(f'precision must be one of {ACTOR_PRECISIONS}, got {precision!r}')
        self.precision = precision
        # GPU featurization (features/raw.py, ops/csrc/featurize.hip): the engine stages raw unit records and ships
        # them in the rollouts; the step's first kernel featurizes them. Default: on wherever the policy step is a
        # fused GPU policy (the eager CPU / torch policy consumes host features)
        from .batched import TorchSlotPolicy, slot_policy_class
        fused = slot_policy_class(self.policy, self.device, precision) is not TorchSlotPolicy
        if raw and not fused:
            raise ValueError('raw observation staging needs a fused GPU actor policy')
        self.raw = fused if raw is None else bool(raw)
        groups = max(1, min(int(groups), n_games))
        sizes = [n_games // groups + (1 if i < n_games % groups else 0) for i in range(groups)]
        self.groups = [_Group(self, i, sizes[i], seed * 7919 + i) for i in range(groups)]
        self.opp_games_finished = 0
        self.games_finished = 0
        self._published = 0
        self._primed = False      # group 0 has a step in flight
        self._wcache = None       # (version, kernel operands, ready event, stream built on): shared by the groups

    # ------------------------------------------------------------------------------------------------
    def _version(self) -> int:
        return int(getattr(self.policy, 'weight_version', -1))

    def _sync_weights(self, g: _Group):
        """Hot-swap the latest weights into the group's captured policy step. The kernels' operand set of a version
        (H2D of the state dict, casts, fragment images / fp8 quantisation: tens of launches) is built ONCE per version
        and copied into every group's buffers — the learner publishes every iteration, and building it per group was
        host time taken from the host-bound actor loop."""
        v = self._version()
        if g.version == v:
            return
        if not hasattr(g.gp, 'load_weight_dict'):
            lock = getattr(self.store, '_lock', None)
            if lock is not None:
                with lock:
                    g.gp.load_weights(self.policy)
                    v = self._version()
            else:
                g.gp.load_weights(self.policy)
            g.version = v
            return
        c = self._wcache
        if c is None or c[0] != v:
            lock = getattr(self.store, '_lock', None)
            if lock is not None:
                with lock:
                    w, ev = g.gp.weight_dict(self.policy)
                    v = self._version()
            else:
                w, ev = g.gp.weight_dict(self.policy)
            c = self._wcache = (v, w, ev, g.gp.stream)
        g.gp.load_weight_dict(c[1], ready=c[2], producer=c[3])
        g.version = c[0]

    def _policy_kw(self) -> dict:
        kw = {'precision': self.precision}
        if self.precision == 'fp8':
            kw['compact'] = False          # (feature staging: the native VecEnv writes the fp32 buffers in place)
        if self.raw:
            kw['raw'] = True
        return kw

    def _sample_opponent(self):
        if self.league is not None:
            return self.league.sample()
        return self.store.oldest_weights()

    def _opponent(self, g: _Group, k: int) -> _Opponent:
        while len(g.opp) <= k:
            gp = make_slot_policy(self.policy, g.S, device=self.device, seed=g.seed + 104729 * (len(g.opp) + 1),
                                  inputs_from=g.gp, **self._policy_kw())
            g.opp.append(_Opponent(gp))
        return g.opp[k]

    def _load_opponent(self, o: _Opponent):
        vs = self._sample_opponent()
        o.gp.load_weights(vs[1])
        o.version = int(vs[0])

    def _assign_opponents(self, g: _Group, reset: np.ndarray):
        """Bind new opponent games (slots just reset that play old weights) to the current opponent policy."""
        if len(reset) == 0:
            return
        opp_slots = g.ve.opponent_slots()
        if len(opp_slots) == 0:
            return
        new_games = np.unique(np.intersect1d(opp_slots, reset) // g.ppg)
        if len(new_games) == 0:
            return
        if not g.opp:
            self._load_opponent(self._opponent(g, 0))
            g.cur_opp = 0
            g.refresh_mark = self.opp_games_finished
        elif self.opp_games_finished - g.refresh_mark >= self.opponent_refresh:
            other = self._opponent(g, 1 - g.cur_opp)
            if other.games == 0:      # rotate once the other policy's games have drained
                self._load_opponent(other)
                g.cur_opp = 1 - g.cur_opp
                g.refresh_mark = self.opp_games_finished
        g.game_opp[new_games] = g.cur_opp
        g.opp[g.cur_opp].games += len(new_games)

    def _finish_results(self, g: _Group):
        for gi, latest_team, end_state in g.ve.pop_results():
            self.games_finished += 1
            k = int(g.game_opp[gi])
            if k < 0:
                continue
            g.game_opp[gi] = -1
            o = g.opp[k]
            o.games -= 1
            self.opp_games_finished += 1
            if self.league is not None and latest_team:
                won = {Status.RADIANT_WIN: 2, Status.DIRE_WIN: 3}.get(end_state)
                self.league.record(o.version, 0.5 if won is None else float(won == latest_team))

    # ------------------------------------------------------------------------------------------------
    def _observe_and_launch(self, g: _Group):
        reset = g.ve.begin_step()
        self._assign_opponents(g, reset)
        if g.raw and g.gp.RAW_WORDS == 4:        # fp8 step: the 16-byte records staged, the full ones kept
            need = g.ve.observe_raw16(g.env, g.hero, g.rawbuf, g.handles, g.active)
        elif g.raw:
            need = g.ve.observe_raw(g.env, g.hero, g.rawbuf, g.handles, g.active)
        else:
            need = g.ve.observe(g.env, g.units, g.handles, g.active)
        g.gp.h_keep.numpy()[reset, 0] = 0.0
        self._sync_weights(g)
        act = g.active.astype(np.float32)
        g.opp_rows = {}
        busy = [k for k, o in enumerate(g.opp) if o.games > 0]
        if busy:
            slot_opp = np.repeat(g.game_opp, g.ppg)
            opp_mask = np.zeros(g.S, bool)
            opp_mask[g.ve.opponent_slots()] = True
            for k in busy:
                o = g.opp[k]
                mine = opp_mask & (slot_opp == k)
                o.gp.h_active.numpy()[:] = act * mine
                o.gp.h_keep.numpy()[reset, 0] = 0.0
                g.opp_rows[k] = np.flatnonzero(mine)
                o.gp.step_async()
            act = act * ~opp_mask
            # opponent trajectories are never published: their stored LSTM states are not fetched
            need = need[~opp_mask[need]]
        g.gp.h_active.numpy()[:] = act
        g.need = need
        g.gp.step_async(snapshot_rows=need if self.H else None)

    def _collect_and_act(self, g: _Group):
        out = g.gp.wait()
        for k, rows in g.opp_rows.items():
            oo = g.opp[k].gp.wait()
            for name in ('idx', 'logp', 'value', 'actions', 'masks'):
                out[name][rows] = oo[name][rows]
        hidden = hslots = None
        if self.H and len(g.need):
            hidden, hslots = out['hidden'], np.ascontiguousarray(g.need, dtype=np.int32)
        g.ve.act(out['idx'], out['actions'], out['masks'], out['logp'], out['value'], hidden, hslots, g.handles,
                 g.version)
        rollouts = g.ve.pop_rollouts()
        if self.publish is not None:
            for b in rollouts:
                self.publish(b)
        self._published += len(rollouts)
        self._finish_results(g)

    # ------------------------------------------------------------------------------------------------
    @property
    def rollouts_sent(self) -> int:
        """Rollouts handed to ``publish`` or encoded into the ring sink."""
        return self._published + (sum(int(g.ve.rollouts_sent) for g in self.groups) if self.ring_sink is not None else 0)

    @property
    def sink_lost(self) -> int:
        """Rollouts the ring sink could not take (no space within the timeout / abandoned)."""
        return sum(int(g.ve.sink_lost) for g in self.groups)

    @property
    def steps_taken(self) -> int:
        return sum(int(g.ve.steps_taken) for g in self.groups)

    @property
    def wire_bytes(self) -> int:
        """Protobuf bytes serialised and decoded so far (wire mode)."""
        return sum(int(g.ve.wire_bytes) for g in self.groups)

    def step(self):
        """One observation interval of every game. Groups are software-pipelined: the host observes group i+1
        while the GPU steps group i, then acts on group i's outputs while the GPU steps group i+1. Between calls
        group 0 has a step in flight."""
        G = len(self.groups)
        if not self._primed:
            self._observe_and_launch(self.groups[0])
            self._primed = True
        for i in range(G):
            if G > 1:
                self._observe_and_launch(self.groups[(i + 1) % G])
            self._collect_and_act(self.groups[i])
        if G == 1:
            self._observe_and_launch(self.groups[0])

    def run(self, n_games: Optional[int] = None, max_steps: Optional[int] = None, log_every: float = 30.0):
        steps = 0
        t0, last = time.time(), self.steps_taken
        while (n_games is None or self.games_finished < n_games) and (max_steps is None or steps < max_steps):
            self.step()
            steps += 1
            if log_every and time.time() - t0 > log_every:
                logger.info('vec actor: %.0f player-steps/s, games finished: %d, rollouts: %d',
                            (self.steps_taken - last) / (time.time() - t0), self.games_finished, self.rollouts_sent)
                t0, last = time.time(), self.steps_taken
        return self.games_finished

    def close(self):
        """Drain the in-flight GPU step."""
        if self._primed and self.device.type == 'cuda':
            torch.cuda.synchronize(self.device)


def measure_vec_actor(policy, device='cuda', n_games: int = 2048, steps: int = 100, warmup: int = 10,
                      threads: int = 8, groups: int = 2, hidden_stride: int = 1400, rollout_size: int = 9999,
                      max_dota_time: float = 600.0, wire: bool = False, precision: str = 'bf16',
                      ring: bool = True) -> Dict[str, float]:
    """Whole-runtime actor throughput: player-steps/s of :class:`VecActor` self-play (engine + featurize + reward +
    GPU policy + trajectory recording + rollout encoding), rollouts counted. Deploy shape (params.libsonnet:16-19):
    whole-game rollouts (``rollout_size`` 9999) of 600 s games, with staggered first games so the measured window sees
    the steady-state rate of finished games (and their encoding). ``ring`` (default): rollouts are encoded into a
    shared-memory experience ring as in the node loop (VecActor ring_sink), drained by a thread that claims and
    releases them without copying (the learner's consumption cost belongs to the learner process); otherwise they are
    published as Python bytes into a list."""
    import threading
    import uuid
    from .weights import WeightStore
    ws = WeightStore(policy.config, device='cpu')
    ws.add(0, {k: v.detach().cpu() for k, v in policy.state_dict().items()})
    sink = []
    br = drain = None
    stop = threading.Event()
    drained = [0, 0]
    if ring:
        from ..transport.shm import ShmBroker
        br = ShmBroker(f'dca_actor_{uuid.uuid4().hex[:10]}', capacity=1 << 28, create=True, drop_oldest=True)

        def run():
            while not stop.is_set():
                got = br.claim_experience(0.05)
                if got is not None:
                    drained[0] += 1
                    drained[1] += int(got[0].nbytes)
                    br.release_experience(got[1])
        drain = threading.Thread(target=run, name='actor-bench-drain', daemon=True)
        drain.start()
    try:
        va = VecActor(ws, n_games, lambda b: sink.append(len(b)), device=device, seed=1, threads=threads,
                      groups=groups, hidden_stride=hidden_stride, rollout_size=rollout_size,
                      max_dota_time=max_dota_time, stagger=True, wire=wire, precision=precision, ring_sink=br)
        sync = (lambda: torch.cuda.synchronize(va.device)) if va.device.type == 'cuda' else (lambda: None)
        for _ in range(warmup):
            va.step()
        sync()
        s0, r0, k0, w0, b0 = va.steps_taken, va.rollouts_sent, len(sink), va.wire_bytes, drained[1]
        t0 = time.perf_counter()
        for _ in range(steps):
            va.step()
        sync()
        dt = time.perf_counter() - t0
        n = va.steps_taken - s0
        mb = (drained[1] - b0) if ring else sum(sink[k0:])
        return {'steps_per_s': n / dt, 'ms_per_step': dt / steps * 1e3, 'games': n_games,
                'player_steps': n, 'rollouts_per_s': (va.rollouts_sent - r0) / dt,
                'rollout_mb_per_s': mb / dt / 1e6, 'threads': threads, 'groups': groups,
                'rollout_size': rollout_size, 'wire': wire, 'protobuf_mb_per_s': (va.wire_bytes - w0) / dt / 1e6,
                'precision': precision, 'publish': 'shm ring (in-place encode)' if ring else 'python bytes'}
    finally:
        stop.set()
        if drain is not None:
            drain.join(timeout=10)
        if br is not None:
            br.close(unlink=True)
