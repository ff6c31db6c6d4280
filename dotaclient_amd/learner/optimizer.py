"""Learner runtime: ingest rollouts → returns/advantages → sequences → DP optimizer steps → checkpoint + publish.

Capability parity with the reference's ``DotaOptimizer`` (optimizer.py:209-715):

* consume rollouts from the experience queue until ≥ ``seq_per_epoch`` sequences (optimizer.py:441-453);
* pad each rollout to a multiple of ``seq_len``, compute returns over the WHOLE rollout before slicing (so returns
  carry across chunks), per-team EMA(0.99) reward normalisation, slice into ``Sequence`` chunks (345-422);
* ``epochs`` passes of shuffled minibatches of ``batch_size`` sequences (458-471); ``seq_per_epoch % batch_size == 0``;
* metrics with the reference's tag names (476-561), checkpoint ``model_%09d.pt`` + model publish every iteration
  (563, 691-715), resume from the latest checkpoint (244-272), optional pretrained weights (strict=False, 271-272).

Beyond the reference: PPO + GAE (``algo='ppo'``, the north star), LSTM chunks start from the actor's stored hidden
state, on-device minibatching (one H2D upload per iteration, then index_select on HBM), full trainer state in the
checkpoint, NaN guard without a per-step host sync (checked once per iteration), per-stage timers, and every rank
resumes from the same iteration (reference quirk §2.10-7).
"""
from __future__ import annotations

import copy
import logging
import os
import random
import socket
import time
from dataclasses import asdict, dataclass, field
from datetime import datetime
from typing import Dict, List, Optional

import numpy as np
import torch

from ..constants import EPS, OBSERVATIONS_PER_SECOND, REWARD_KEYS
from ..models.policy import Policy, get_config
from ..parallel import dist as pdist
from ..transport.codec import CorruptMessage, Rollout, decode_any
from ..utils import checkpoint as ckpt
from ..utils.faults import faults
from ..utils.metrics import MetricsWriter, StageTimer
from .engine import Learner, LossConfig
from .returns import RunningMeanStd, discount, gae

logger = logging.getLogger(__name__)


def default_log_dir():
    return '{}_{}'.format(datetime.now().strftime('%b%d_%H-%M-%S'), socket.gethostname())


@dataclass
class OptimizerConfig:
    log_dir: str = field(default_factory=default_log_dir)
    epochs: int = 4                    # optimizer.py:774
    seq_per_epoch: int = 16            # optimizer.py:775
    batch_size: int = 4                # optimizer.py:776
    seq_len: int = 256                 # optimizer.py:777
    learning_rate: float = 1e-4
    entropy_coef: float = 0.01
    vf_coef: float = 0.5
    pretrained_model: Optional[str] = None
    mq_prefetch_count: int = 4
    run_local: bool = True
    iterations: int = 10000            # optimizer.py:238
    algo: str = 'ppo'
    model: str = 'lstm512'
    gamma: float = 0.98
    gae_lambda: float = 0.95
    clip_eps: float = 0.1
    max_grad_norm: float = 0.5
    compat_value_bug: bool = False
    normalize_advantages: bool = True
    device: str = 'auto'
    backend: str = 'auto'
    precision: str = 'fp32-exact'      # 'fp32-exact' (reference precision, IEEE fp32 products) | 'fp32' (bf16x3 operands) | 'bf16'
    checkpoint_keep: int = 0
    histogram_freq: int = 128          # optimizer.py:214
    xp_timeout: Optional[float] = None
    seed: int = 7
    replay_gb: float = 0.0             # on-HBM replay budget (GB); 0 with replay_capacity 0 = reference behaviour
    replay_capacity: int = 0           # sequences (overrides replay_gb)
    replay_recent: int = 0             # sample from the newest N sequences (0 = whole buffer)
    replay_prefill: bool = False       # fill the ring to capacity from the first ingest (benchmarks, HbmReplay.prefill)
    ingest: str = 'auto'               # 'device' (HIP return/GAE scan over the uploaded rollouts) | 'host' | 'auto'
    artifact_url: Optional[str] = None  # off-node mirror of checkpoints + events (reference: GCS bucket, §utils.artifacts)
    allow_pickle_experience: bool = False  # accept reference-agent pickles (restricted unpickler); off: DCX1 only
    graph: bool = True                 # capture the fused train step in a hipGraph (learner/engine.py enable_graph)
    async_checkpoint: bool = False     # write checkpoint files on a background thread (the model is published first)
    prefetch_rollouts: int = 0         # >0: consume + decode up to N rollouts ahead on a background thread (overlaps
                                       #     the next iteration's decode with this one's training); 0: inline
    record_consumed: int = 0           # keep the keys (game, team, player, version, length) of the last N rollouts
                                       #     consumed (competing-consumer tests; 0 = off)
    lookahead_ingest: bool = True
    # non-compat: pack whole zero-state rollouts first-fit into the free tails of the iteration's sequences (episode
    # starts flagged, the recurrence resets h, c there) instead of padding each rollout to seq_len (learner/ingest.py)
    pack_sequences: bool = False
    # PPO advantages / value targets of stale experience (PPO + device ingest):
    # * 'vtrace-step' (default): V-trace INSIDE every learner step — the minibatch's advantages and value targets from
    #   the step's own values and log-probs (the weights being trained) with truncated importance weights against the
    #   actor's behaviour log-probs (LossConfig.vtrace, ops/csrc/scan.hip vtrace_step_kernel): correct for fresh and
    #   for replayed experience alike, ≈0.1 ms per step;
    # * 'vtrace-iteration': the reference's policy_old (optimizer.py:279, 474) — once per iteration, before its
    #   minibatches, the iteration's experience is evaluated at the iteration's starting weights (Learner.
    #   evaluate_sequences, the step's forward kernels) and V-trace GAE computed from those values (a whole extra
    #   forward per iteration: ≈30 % of the node loop's rate);
    # * 'gae': the actor's values from collection time (on-policy only at weight age 0; rounds 1-5).
    advantages: str = 'vtrace-step'
    # the PPO ratio's denominator: 'actor' = the behaviour log-prob (the clip is a trust region around what the actors
    # played — measured stable at weight age 18); 'learner' = the iteration's starting policy (with 'vtrace-iteration';
    # decoupled PPO: measured to drift and collapse at weight age ≥ 6, profiles/r6_*)
    old_logp: str = 'actor'
    vtrace_rho_bar: float = 1.0
    vtrace_c_bar: float = 1.0
    # policy term on replayed experience (replay_gb / replay_capacity): 'tis' = truncated importance weight
    # min(1, π/π_old) (never zero on many-versions-old samples), 'clip' = PPO's clipped surrogate
    replay_offpolicy: str = 'tis'
    # pipelined GPU learner with async_checkpoint: publish each iteration's weights right after its steps are queued
    # and finalise its metrics (the one device→host sync) during the NEXT iteration — no blocking sync per iteration
    defer_metrics: bool = True
                                       # pipelined GPU ingest: take and expand the NEXT iteration's staged rollouts
                                       #     while this iteration's steps run on the GPU (its host work then overlaps
                                       #     the training instead of leaving the GPU idle between iterations)


class Sequence:
    """One ``seq_len`` chunk of a rollout (optimizer.py:165-200), plus PPO/LSTM extras."""

    def __init__(self, game_id, env, units, actions, masks, rewards, returns, norm_returns, adv, logp, values,
                 weight_version, team_id, hidden, valid):
        self.game_id = game_id
        self.env, self.units, self.actions, self.masks = env, units, actions, masks
        self.rewards = rewards
        self.discounted_rewards = returns
        self.norm_discounted_rewards = norm_returns
        self.adv, self.logp, self.values = adv, logp, values
        self.weight_version = weight_version
        self.team_id = team_id
        self.hidden = hidden
        self.valid = valid


class _IterationPool:
    """Per-iteration sequence pool of the GPU learner (see :meth:`DotaOptimizer._iteration_pool`)."""

    def __init__(self, like: Dict[str, torch.Tensor], capacity: int, S: int):
        self.capacity, self.S = int(capacity), int(S)
        self.data = {k: torch.zeros((self.capacity,) + tuple(v.shape[1:]), dtype=v.dtype, device=v.device)
                     for k, v in like.items()}

    def gather(self, idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        return {k: v.index_select(0, idx) for k, v in self.data.items()}


class DotaOptimizer:
    SPEED_KEY = 'steps per s'
    MAX_TEAMS = 16

    def __init__(self, cfg: OptimizerConfig, broker, checkpoint: Optional[bool] = None):
        self.cfg = cfg
        assert cfg.seq_per_epoch >= cfg.batch_size and cfg.seq_per_epoch % cfg.batch_size == 0
        self.broker = broker
        self.checkpoint = pdist.is_master() if checkpoint is None else checkpoint
        dev = cfg.device
        if dev == 'auto':
            dev = f'cuda:{pdist.local_rank()}' if torch.cuda.is_available() else 'cpu'
        self.device = torch.device(dev)
        random.seed(cfg.seed)
        np.random.seed(cfg.seed)
        torch.manual_seed(cfg.seed)
        self.policy_cfg = get_config(cfg.model)
        self.policy = Policy(self.policy_cfg)
        self.running = RunningMeanStd(0.99)
        self.team_keys: Dict[int, int] = {}     # team_id -> row of the device EMA state
        self.iteration_start = 1
        self.writer = MetricsWriter(cfg.log_dir if self.checkpoint else None)
        self.timer = StageTimer()
        pretrained = cfg.pretrained_model
        if pretrained:
            from ..utils.artifacts import resolve_model_path
            pretrained = resolve_model_path(pretrained)
        # artifact store (reference: GCS bucket 'dotaservice', disabled by --run-local)
        from ..utils.artifacts import Uploader, fetch_latest_checkpoint, open_store
        self.store = open_store(cfg.artifact_url) if (cfg.artifact_url and not cfg.run_local) else None
        self.store_prefix = os.path.basename(os.path.normpath(cfg.log_dir))
        self.uploader = Uploader(self.store) if (self.store is not None and self.checkpoint) else None
        trainer_state = None
        latest = ckpt.latest_model(cfg.log_dir)
        if latest is None and self.store is not None and self.checkpoint:
            os.makedirs(cfg.log_dir, exist_ok=True)
            latest = fetch_latest_checkpoint(self.store, self.store_prefix, cfg.log_dir)
        if latest is not None:
            logger.info('resuming from %s', latest)
            self.iteration_start = ckpt.iteration_from_model_filename(latest) + 1
            pretrained = latest
            trainer_state = ckpt.load_trainer_state(cfg.log_dir, self.iteration_start - 1)
        if pretrained is not None:
            self.policy.load_state_dict(ckpt.load_model_file(pretrained), strict=False)
        replay_on = bool(cfg.replay_capacity or cfg.replay_gb)
        if cfg.advantages not in ('vtrace-step', 'vtrace-iteration', 'gae'):
            raise ValueError(f'advantages must be vtrace-step, vtrace-iteration or gae, got {cfg.advantages!r}')
        dev_ingest = (cfg.ingest if cfg.ingest != 'auto' else
                      ('device' if (cfg.device == 'auto' and torch.cuda.is_available()) or
                       str(cfg.device).startswith('cuda') else 'host'))
        self.vtrace_step = cfg.advantages == 'vtrace-step' and cfg.algo == 'ppo' and dev_ingest == 'device'
        lc = LossConfig(algo=cfg.algo, learning_rate=cfg.learning_rate, entropy_coef=cfg.entropy_coef,
                        vf_coef=cfg.vf_coef, clip_eps=cfg.clip_eps, gamma=cfg.gamma, gae_lambda=cfg.gae_lambda,
                        max_grad_norm=cfg.max_grad_norm, compat_value_bug=cfg.compat_value_bug,
                        # (in-step V-trace: the advantages already carry the truncated IS weight; the policy term
                        # stays PPO's clip around the behaviour policy, the trust region measured stable at high lag)
                        offpolicy=cfg.replay_offpolicy if (replay_on and not self.vtrace_step) else 'clip',
                        vtrace=self.vtrace_step,
                        vtrace_rho_bar=cfg.vtrace_rho_bar, vtrace_c_bar=cfg.vtrace_c_bar)
        prec = cfg.precision
        if prec == 'fp32-exact' and self.device.type == 'cuda' and cfg.batch_size > 32:
            # the exact VALU recurrence runs 1 / 2 / 4 sequences per XCD chain (8 teams): at most 32 per minibatch
            logger.info('fp32-exact takes at most 32 sequences per minibatch and GPU: training at fp32 with bf16x3 '
                        'operands (batch_size %d)', cfg.batch_size)
            prec = 'fp32'
        self.learner = Learner(self.policy, lc, device=self.device, backend=cfg.backend, precision=prec)
        if cfg.graph:
            self.learner.enable_graph(warmup=1)
        if trainer_state is not None:
            self.learner.load_state_dict(trainer_state['learner'])
            self.running.load_state_dict(trainer_state['running'])
        self.ingest = cfg.ingest if cfg.ingest != 'auto' else ('device' if self.device.type == 'cuda' else 'host')
        if cfg.pack_sequences and self.ingest != 'device':
            raise ValueError('pack_sequences needs the device ingest (ingest="device")')
        if cfg.old_logp not in ('learner', 'actor'):
            raise ValueError(f'old_logp must be learner or actor, got {cfg.old_logp!r}')
        if cfg.old_logp == 'learner' and cfg.advantages != 'vtrace-iteration':
            raise ValueError("old_logp='learner' needs advantages='vtrace-iteration' (the per-iteration policy_old pass)")
        if cfg.advantages != 'gae' and self.ingest != 'device' and cfg.algo == 'ppo':
            logger.warning('advantages=%s needs the device ingest: the host ingest computes GAE from the actor\'s '
                           'values', cfg.advantages)
        # per-team EMA(0.99) reward statistics as device state (mean, std, initialised) for the device ingest path
        self.ema = torch.zeros(self.MAX_TEAMS, 3, device=self.device)
        for team in self.running.mean:
            if self.running.mean[team] is not None:
                k = self._team_key(team)
                self.ema[k] = torch.tensor([self.running.mean[team], self.running.std[team], 1.0])
        # every rank starts from rank 0's iteration (reference workers restart at 1, §2.10-7) and with rank 0's
        # optimizer state (Adam moments / step counts): identical averaged gradients only keep the replicas in sync
        # if every replica applies them with the same optimizer state
        if pdist.is_distributed():
            t = torch.tensor([self.iteration_start], device=self.device if self.device.type == 'cuda' else 'cpu')
            torch.distributed.broadcast(t, 0)
            self.iteration_start = int(t.item())
            self.learner.broadcast_state(0)
            self._broadcast_reward_stats(0)
        self.corrupt_rollouts = 0
        self.n_published = 0               # model messages this rank published (rank 0 only, reference :284-287)
        self.consumed = None
        if cfg.record_consumed:
            import collections
            self.consumed = collections.deque(maxlen=cfg.record_consumed)
        self.replay = None
        if cfg.replay_capacity or cfg.replay_gb:
            from .replay import HbmReplay
            hid = self.policy_cfg.hidden if self.policy.is_recurrent else None
            pk = bool(cfg.pack_sequences)             # packed sequences keep their episode-start flags in the ring
            gb = cfg.replay_gb
            if not cfg.replay_capacity and self.device.type == 'cuda':
                # never more than the GPU can hold beside this learner, the node loop's actor process and whatever
                # else is resident: a replay that oversubscribes HBM turns into device-wide stalls of many seconds per
                # step (round 5: a box with 262 GB already in use). Keep 24 GB of headroom.
                free = torch.cuda.mem_get_info(self.device)[0] / 1e9
                if gb > free - 24.0:
                    fit = max(1.0, free - 24.0)
                    logger.warning('replay_gb %.0f > %.0f GB free on %s: the replay takes %.0f GB', gb, free,
                                   self.device, fit)
                    gb = fit
            cap = cfg.replay_capacity or HbmReplay.capacity_for_bytes(gb * 1e9, cfg.seq_len,
                                                                       self.policy_cfg.layout, hid, pk,
                                                                       vtrace=self.vtrace_step)
            self.replay = HbmReplay(cap, cfg.seq_len, self.policy_cfg.layout, hid, self.device, seed=cfg.seed,
                                    reset=pk, vtrace=self.vtrace_step)
            logger.info('on-device replay: %d sequences, %.2f GB', cap, self.replay.nbytes / 1e9)
        self.time_last_step = time.time()
        if self.iteration_start == 1:
            self.upload_model(version=0)

    def _broadcast_reward_stats(self, src: int = 0):
        """Every rank normalises returns with rank ``src``'s per-team EMA(0.99) statistics after a resume (only rank
        0 reads the trainer state): the team→row map, the device EMA rows and the host RunningMeanStd."""
        import torch.distributed as tdist
        keys = [sorted(self.team_keys.items())]
        tdist.broadcast_object_list(keys, src)
        self.team_keys = dict(keys[0])
        run = [self.running.state_dict()]
        tdist.broadcast_object_list(run, src)
        self.running.load_state_dict(run[0])
        ema = self.ema if self.device.type == 'cuda' else self.ema.contiguous()
        tdist.broadcast(ema, src)
        self.ema.copy_(ema)

    def _agree_steps(self, n: int) -> int:
        """Sequences this rank trains on this iteration: its full minibatches, reduced to the MINIMUM over the DP
        ranks — ranks receive rollouts of different lengths, and a rank running one more train_step than the others
        would pair its gradient all-reduce with the next iteration's (or hang on the last one)."""
        if not pdist.is_distributed():
            return n
        t = torch.tensor([n], dtype=torch.int64, device=self.device if self.device.type == 'cuda' else 'cpu')
        torch.distributed.all_reduce(t, op=torch.distributed.ReduceOp.MIN)
        return int(t.item())

    # ------------------------------------------------------------------------------------------------
    def get_rollout(self) -> Rollout:
        """Next decoded rollout: from the decode-ahead thread when ``prefetch_rollouts`` > 0, else inline."""
        r = self._next_rollout()
        if self.consumed is not None:
            self.consumed.append((r.game_id, int(r.team_id), int(r.player_id), int(r.weight_version), r.length))
        return r

    def _next_rollout(self) -> Rollout:
        if self.cfg.prefetch_rollouts > 0:
            pf = getattr(self, '_prefetcher', None)
            if pf is None:
                # a blocking client of its own when the broker has one (TCP): the main thread's broker calls
                # (queue size, model publish) must not wait behind the thread's long polls
                mk = getattr(self.broker, 'consumer', None)
                self._xp_broker = mk() if mk is not None else self.broker
                # (copying consumption here: nothing stages these rollouts, so ring claims would never be released)
                pf = self._prefetcher = _RolloutPrefetcher(self._consume_decode, self.cfg.prefetch_rollouts)
                self.prefetch_dropped = 0
            return pf.get()
        return self._consume_decode()

    def close(self):
        """Stop the decode-ahead / stager thread (if any) and join it; rollouts it had already taken from the queue
        are dropped and counted in ``prefetch_dropped``."""
        pf = getattr(self, '_prefetcher', None)
        pl = getattr(self, '_pipeline', None)
        dropped = 0
        ahead = getattr(self, '_lookahead', None)
        if ahead is not None:
            # taken off the queue (and logged as consumed) for an iteration that will never run
            dropped += len(ahead[0])
            self._lookahead = None
        if pl is not None:                   # the stager first: its fetch returns None once it is stopping
            dropped += pl.close()
            self._pipeline = None
        if pf is not None or pl is not None or dropped:
            if pf is not None:
                dropped += pf.close()
                self._prefetcher = None
            self.prefetch_dropped = getattr(self, 'prefetch_dropped', 0) + dropped
            xb = getattr(self, '_xp_broker', None)
            if xb is not None and xb is not self.broker and hasattr(xb, 'close'):
                xb.close()
            self._xp_broker = None

    def _consume_decode(self, stop=None, claim: bool = False) -> Rollout:
        """Next decodable rollout from the queue. With ``stop`` (the decode-ahead thread's event) the queue is polled
        in bounded slices so that :meth:`close` ends the thread promptly instead of leaving it blocked inside the
        broker; returns None once ``stop`` is set.

        ``claim`` (the GPU learner's stager pipeline on the node's shared-memory ring): the rollout's arrays VIEW the
        message inside the ring — no copy out of it; the stager copies the fields straight into its pinned upload slot
        and gives the region back (:meth:`Rollout.detach_shared`). One host copy per message instead of two (ring →
        heap → pinned). Claims are budgeted to half the ring (split over the node's learner ranks), beyond that the
        copying path is taken, so held claims can never starve the producers."""
        broker = getattr(self, '_xp_broker', None) or self.broker
        if claim and stop is not None and hasattr(broker, 'claim_experience'):
            cb = self.__dict__.get('_claim_budget')
            if cb is None:
                # half the ring, shared by the node's learner ranks (competing consumers of the one ring)
                ranks = max(1, int(os.environ.get('LOCAL_WORLD_SIZE', os.environ.get('WORLD_SIZE', '1')) or 1))
                cb = self.__dict__.setdefault('_claim_budget',
                                              _ClaimBudget(getattr(broker, 'capacity', 0) // (2 * ranks)))
            t0 = time.monotonic()
            while cb.available():
                got = None
                tw = time.perf_counter()
                while got is None:
                    if stop.is_set():
                        return None
                    if self.cfg.xp_timeout is not None and time.monotonic() - t0 > self.cfg.xp_timeout:
                        raise TimeoutError('no experience received')
                    got = broker.claim_experience(timeout=0.25)
                td = time.perf_counter()
                st = self.__dict__.setdefault('_claim_stats', [0, 0.0, 0.0])   # messages, claim wait s, decode s
                st[1] += td - tw
                view, token = got
                rel = _RingClaim(broker, token, cb.take(view.nbytes), cb)
                try:
                    r = decode_any(view, allow_pickle=self.cfg.allow_pickle_experience)
                except CorruptMessage as e:
                    rel()
                    self.corrupt_rollouts += 1
                    logger.warning('dropping corrupted experience message (%s); %d so far', e, self.corrupt_rollouts)
                    continue
                r.release = rel
                st[0] += 1
                st[2] += time.perf_counter() - td
                return r
        checked = getattr(broker, 'consume_experience_checked', None)    # shm ring: CRC verified during the copy
        consume = checked or getattr(broker, 'consume_experience_view', None) or broker.consume_experience
        total = self.cfg.xp_timeout
        while True:
            if stop is None:
                body = consume(timeout=total)
            else:
                t0 = time.monotonic()
                body = None
                while body is None and not stop.is_set():
                    left = None if total is None else total - (time.monotonic() - t0)
                    if left is not None and left <= 0:
                        break
                    body = consume(timeout=0.25 if left is None else min(0.25, left))
                if body is None and stop.is_set():
                    return None
            if body is None:
                raise TimeoutError('no experience received')
            ok = None
            if checked is not None:
                body, ok = body
            try:
                if ok is False:
                    raise CorruptMessage('experience message CRC mismatch (corrupted or truncated)')
                return decode_any(body, allow_pickle=self.cfg.allow_pickle_experience, crc_checked=ok is True)
            except CorruptMessage as e:       # drop it, like a lost message; the actors keep producing
                self.corrupt_rollouts += 1
                logger.warning('dropping corrupted experience message (%s); %d so far', e, self.corrupt_rollouts)

    def experiences_from_rollout(self, r: Rollout) -> List[Sequence]:
        S = self.cfg.seq_len
        T = r.length
        pad = (S - T % S) % S
        n_seq = (T + pad) // S

        def padt(a, fill=0):
            if a is None or pad == 0:
                return a
            w = [(0, pad)] + [(0, 0)] * (a.ndim - 1)
            return np.pad(a, w, mode='constant', constant_values=fill)
        rewards = padt(r.rewards)
        summed = rewards.sum(axis=1)
        valid = np.concatenate([np.ones(T, np.float32), np.zeros(pad, np.float32)])
        if self.cfg.algo == 'ppo' and r.values is not None:
            values = padt(r.values.astype(np.float32))
            adv, ret = gae(summed[:T], r.values, r.bootstrap_value, self.cfg.gamma, self.cfg.gae_lambda, done=r.done)
            adv, ret = padt(adv), padt(ret)
            self.running.update(ret[:T], r.team_id)
            norm = adv
        else:
            # reference: discounted return over the full (padded) rollout, γ = 0.98 (optimizer.py:382)
            ret = discount(summed, self.cfg.gamma)
            self.running.update(ret, r.team_id)
            norm = self.running.normalize(ret, r.team_id)
            adv = norm
            values = np.zeros(T + pad, np.float32)
        logp = padt(r.logp.astype(np.float32)) if r.logp is not None else np.zeros(T + pad, np.float32)
        env, units = padt(r.env), padt(r.ensure_units().units)      # (a raw rollout: host features, exact)
        actions, masks = padt(r.actions), padt(r.masks)
        seqs = []
        H = self.policy_cfg.hidden
        for s in range(n_seq):
            a, b = s * S, (s + 1) * S
            hidden = None
            if self.policy.is_recurrent:
                hidden = np.zeros((2, H), np.float32)
                if r.hiddens is not None and r.hidden_stride and a % r.hidden_stride == 0 \
                        and a // r.hidden_stride < len(r.hiddens):
                    hidden = r.hiddens[a // r.hidden_stride]
            seqs.append(Sequence(r.game_id, env[a:b], units[a:b], actions[a:b], masks[a:b], rewards[a:b], ret[a:b],
                                 norm[a:b], adv[a:b], logp[a:b], values[a:b], r.weight_version, r.team_id, hidden,
                                 valid[a:b]))
        return seqs

    def _team_key(self, team: int) -> int:
        k = self.team_keys.get(team)
        if k is None:
            if len(self.team_keys) >= self.MAX_TEAMS:
                raise ValueError(f'more than {self.MAX_TEAMS} distinct team ids')
            k = self.team_keys[team] = len(self.team_keys)
        return k

    def _ingest_device(self, rollouts: List[Rollout], n_keep: int) -> Dict[str, torch.Tensor]:
        """Device ingest, inline: stage + upload this iteration's rollouts (valid rows only) and expand them on the
        device (:mod:`learner.ingest`), then the return / GAE scan. The pipelined form runs the staging on the
        stager thread one iteration ahead (``prefetch_rollouts`` > 0 on a GPU learner)."""
        return self._finish_ingest(self._ingest_pipeline(thread=False).stage(rollouts), n_keep)

    def ingest_stats(self) -> Dict[str, float]:
        """Decode-side counters of the zero-copy path (node-loop diagnostics): messages claimed, total seconds the
        decode threads waited in the ring's claim and spent decoding (CRC + header), and waited on the full queue."""
        st = self.__dict__.get('_claim_stats', [0, 0.0, 0.0])
        pf = getattr(self, '_prefetcher', None)
        return {'claimed': int(st[0]), 'claim_wait_s': float(st[1]), 'decode_s': float(st[2]),
                'queue_put_wait_s': float(pf.put_wait) if pf is not None else float('nan')}

    def _ingest_pipeline(self, thread: bool):
        pl = getattr(self, '_pipeline', None)
        if pl is None:
            from .ingest import IngestPipeline
            H = self.policy_cfg.hidden if self.policy.is_recurrent else 0
            fetch = None
            if thread:
                # a blocking client of its own when the broker has one (TCP): the main thread's broker calls
                # (queue size, model publish) must not wait behind the stager's long polls
                mk = getattr(self.broker, 'consumer', None)
                self._xp_broker = mk() if mk is not None else self.broker
                # consume + decode (CRC with the GIL released) on a thread of their own, so the stager packs and
                # uploads iteration k+1 while the rollouts of k+2 are being decoded; on the node's shm ring zero-copy
                # (claimed regions, released once staged — IngestPipeline.stage)
                # (one decode thread: with zero-copy its CRC pass is ≈30 % of a core at the loop's 2 000 rollouts/s;
                # three measured no faster, round 5)
                zc = hasattr(self._xp_broker, 'claim_experience')
                pf = self._prefetcher = _RolloutPrefetcher(lambda stop: self._consume_decode(stop, claim=zc),
                                                           self.cfg.prefetch_rollouts)
                fetch = pf.get_until
            pl = self._pipeline = IngestPipeline(fetch, self.cfg.seq_len, self.cfg.seq_per_epoch, self.cfg.algo, H,
                                                 self.device, pack=self.cfg.pack_sequences)
        return pl

    def _finish_ingest(self, st, n_keep: int) -> Dict[str, torch.Tensor]:
        """Expand a staged iteration into the padded layout and run the HIP segmented reverse scan (returns / GAE +
        per-team EMA(0.99) normalisation, ``ops/csrc/scan.hip``) over all its rollouts at once; the learner's
        sequences are a reshape of the result. Same numbers as :meth:`experiences_from_rollout` + :meth:`_to_device`
        (the host path)."""
        from ..ops.scan import compute_returns
        cfg = self.cfg
        S = cfg.seq_len
        pad = self.__dict__.setdefault('_pad_bufs', {})
        x = self._pipeline.expand(st, pad)
        d = {'env': x['env'], 'units': x['units'], 'actions': x['actions'], 'masks': x['masks'],
             'logp_old': x['logp'], 'valid': x['valid']}
        rollouts = st.rollouts
        keys = [self._team_key(r.team_id) for r in rollouts]
        values, mode, lr = (x.get('values'), 'gae', None) if st.gae_mode else (None, 'discount', None)
        prox = None
        if st.gae_mode and cfg.advantages == 'vtrace-iteration':
            # the reference's policy_old, refreshed every iteration (optimizer.py:279, 474): the iteration's
            # sequences evaluated at the weights its first minibatch will see (this is enqueued behind the previous
            # iteration's steps in stream order — the look-ahead — so those ARE the weights it reads), its log-probs
            # the PPO ratio's denominator, its values the V-trace GAE baseline with truncated importance weights
            # against the actor's behaviour log-probs (stale experience: the actor played version − weight age)
            lp, values, prox = self._evaluate_iteration(x, st.n_seq)
            lr = lp - x['logp']
            if cfg.old_logp == 'learner':
                d['logp_old'] = lp
            mode = 'vtrace'
        out = compute_returns(x['rewards'], values, st.off.astype(np.int32),
                              st.lens, [r.bootstrap_value for r in rollouts], [bool(r.done) for r in rollouts], keys,
                              self.ema, mode, gamma=cfg.gamma, lam=cfg.gae_lambda,
                              factor=self.running.factor, lr=lr, rho_bar=cfg.vtrace_rho_bar, c_bar=cfg.vtrace_c_bar)
        d['ret'], d['adv'] = out['ret'], out['adv']
        d['norm_ret'] = out['norm'] if not st.gae_mode else out['adv']
        if self.vtrace_step and st.gae_mode:
            d['vt'] = self._vtrace_rows(x, st)
        n_rows = n_keep * S
        d = {k: v[:n_rows].reshape((n_keep, S) + tuple(v.shape[1:])) for k, v in d.items()}
        if self.policy.is_recurrent:
            h = x['hid'][:n_keep]
            d['h0'], d['c0'] = h[:, 0].contiguous(), h[:, 1].contiguous()
            if 'reset' in x:
                d['reset'] = x['reset'][:n_rows].view(n_keep, S)
        self._normalize_advantages(d)
        if prox is not None:
            d['_prox'] = prox          # (metrics; popped by run_iteration before the data is used)
        return d

    def _vtrace_rows(self, x: Dict[str, torch.Tensor], st) -> torch.Tensor:
        """Per-row inputs of the in-step V-trace (LossConfig.vtrace) in the padded layout: (L, 4) = {summed reward,
        bootstrap, valid, last}. ``last`` marks where an episode segment ends inside its sequence: the rollout's last
        row (bootstrap 0 at a terminal, else the actor's bootstrap value) and every sequence boundary the rollout
        runs past (bootstrap: the actor's value of the next row, the first row of the next sequence)."""
        S = self.cfg.seq_len
        L = st.L
        dev = x['rewards'].device
        vt = torch.zeros(L, 4, device=dev)
        vt[:, 0] = x['rewards'][:L].float().sum(1)
        vt[:, 2] = x['valid'][:L]
        starts = np.asarray(st.off[:-1], np.int64)
        lens = np.asarray(st.lens, np.int64)
        ends = starts + lens - 1
        boot = np.asarray([0.0 if r.done else float(r.bootstrap_value) for r in st.rollouts], np.float32)
        bnd = [np.arange((a // S + 1) * S - 1, a + T - 1, S, dtype=np.int64) for a, T in zip(starts, lens)]
        bnd = np.concatenate(bnd) if bnd else np.zeros(0, np.int64)
        cuda = dev.type == 'cuda'

        def up(a):      # small host arrays: pinned (the caching host allocator keeps a block until its copy ran)
            t = torch.from_numpy(a)
            return t.pin_memory().to(dev, non_blocking=True) if cuda else t
        e_d, b_d = up(ends), up(boot)
        vt[:, 3].index_fill_(0, e_d, 1.0)
        vt[:, 1].index_copy_(0, e_d, b_d)
        if len(bnd):
            n_d = up(bnd)
            vt[:, 3].index_fill_(0, n_d, 1.0)
            vt[:, 1].index_copy_(0, n_d, x['values'][:L].float().index_select(0, n_d + 1))
        return vt

    def _evaluate_iteration(self, x: Dict[str, torch.Tensor], n_seq: int):
        """Learner-side log-probs and values of the expanded iteration ``x`` (padded layout, ``n_seq`` sequences of
        ``seq_len`` rows) at the current weights, plus device metrics of how far the behaviour policy was:
        ``offpolicy/behaviour_kl`` (mean log μ − log π over valid rows), ``offpolicy/rho_mean`` (mean truncated
        importance weight), ``offpolicy/rho_truncated`` (fraction of rows with π > μ) and
        ``offpolicy/max_abs_logratio``. Returns (logp (L,), value (L,), metrics)."""
        S = self.cfg.seq_len
        L = n_seq * S
        view = {k: x[k][:L].reshape((n_seq, S) + tuple(x[k].shape[1:])) for k in ('units', 'env', 'actions', 'masks')}
        if 'hid' in x:
            view['h0'], view['c0'] = x['hid'][:, 0].contiguous(), x['hid'][:, 1].contiguous()
        if 'reset' in x:
            view['reset'] = x['reset'][:L].reshape(n_seq, S)
        lp, v = self.learner.evaluate_sequences(view, n_seq)
        lp, v = lp.reshape(L), v.reshape(L)
        valid = x['valid'][:L]
        nv = valid.sum().clamp_min(1.0)
        # a row whose recorded action the learner gives no probability (−inf: a mask that excludes it) or a padding
        # row keeps the actor's log-prob: a −inf denominator would make the PPO ratio NaN
        ok = torch.isfinite(lp) & (valid > 0)
        bad = ((~torch.isfinite(lp)).float() * valid).sum()
        lp = torch.where(ok, lp, x['logp'][:L])
        v = torch.where(torch.isfinite(v), v, torch.zeros_like(v))
        dlt = (lp - x['logp'][:L]) * valid
        w = torch.exp(dlt.clamp(max=30.0))
        m = {'offpolicy/behaviour_kl': -dlt.sum() / nv,
             'offpolicy/rho_mean': (w.clamp(max=self.cfg.vtrace_rho_bar) * valid).sum() / nv,
             'offpolicy/rho_truncated': ((w > self.cfg.vtrace_rho_bar).float() * valid).sum() / nv,
             'offpolicy/max_abs_logratio': dlt.abs().max(),
             'offpolicy/logratio_gt1_frac': ((dlt.abs() > 1.0).float() * valid).sum() / nv,
             'offpolicy/nonfinite_rows': bad}
        return lp, v, m

    def _staging(self, name: str, shape, dtype, pin: bool) -> torch.Tensor:
        """Host staging buffer for one ingest field (contents undefined: the caller writes every row), reused across
        iterations (pinned allocations cost milliseconds each). Safe to overwrite: the previous iteration's uploads
        were consumed before its training finished (the iteration ends with a device synchronise)."""
        if not pin:                 # CPU learner: .to(cpu) would alias the buffer into the iteration's data
            return torch.empty(shape, dtype=dtype)
        cache = self.__dict__.setdefault('_stage_bufs', {})
        n = int(np.prod(shape))
        buf = cache.get(name)
        if buf is None or buf.dtype != dtype or buf.numel() < n:
            buf = cache[name] = torch.empty(max(n, 2 * (buf.numel() if buf is not None else 0)), dtype=dtype,
                                            pin_memory=pin)
        return buf[:n].view(shape)

    def _iteration_pool(self, data: Dict[str, torch.Tensor], n: int):
        """The iteration's sequences copied once into a persistent device pool (fixed addresses, so the graph-captured
        step replays with its gather inside) instead of an ``index_select`` of every field per minibatch followed by
        the step's own batch-major → time-major copies."""
        pool = getattr(self, '_pool', None)
        fields = [k for k in Learner.STEP_FIELDS + ('h0', 'c0', 'reset', 'vt') if k in data]
        if pool is None or pool.capacity < n or set(pool.data) != set(fields) or any(
                pool.data[k].shape[1:] != data[k].shape[1:] or pool.data[k].dtype != data[k].dtype for k in fields):
            cap = max(n, 2 * self.cfg.seq_per_epoch)
            if pool is not None:
                # geometric growth (a slowly rising n reallocates O(log n) times, not once per new maximum), and
                # the captured steps bound to the old storage are released before it is freed
                cap = max(cap, 2 * pool.capacity)
                # with deferred metrics the previous iteration's replays (reading the old pool, running in the
                # graphs' private memory pools) may still be in flight: wait for them before the graphs and the
                # storage go
                prev = getattr(self, '_pending_metrics', None)
                if prev is not None and prev.get('done') is not None:
                    prev['done'].synchronize()
                if self.device.type == 'cuda':
                    torch.cuda.current_stream(self.device).synchronize()
                self.learner.release_graphs(pool)
            pool = self._pool = _IterationPool({k: data[k] for k in fields}, cap, self.cfg.seq_len)
        dst = [pool.data[k][:n] for k in fields]
        src = [data[k][:n] for k in fields]
        if self.device.type == 'cuda' and all(t.is_contiguous() and t.data_ptr() % 16 == 0 for t in dst + src):
            from ..ops import require
            require().multi_copy(dst, src)            # one launch for every field (was one copy launch each)
        else:
            for d, t in zip(dst, src):
                d.copy_(t)
        return pool

    def _sync_running(self, ema: Optional[torch.Tensor] = None):
        """Mirror the device EMA state (or a snapshot of it) into the host RunningMeanStd (metrics + checkpoint)."""
        e = (self.ema if ema is None else ema).cpu()
        for team, k in self.team_keys.items():
            if e[k, 2] != 0:
                self.running.mean[team] = float(e[k, 0])
                self.running.std[team] = float(e[k, 1])

    def _normalize_advantages(self, d):
        if self.cfg.algo == 'ppo' and self.cfg.normalize_advantages:
            a, v = d['adv'], d['valid']
            if a.is_cuda and a.is_contiguous() and v.is_contiguous() and a.dtype == v.dtype == torch.float32:
                # one single-workgroup kernel (ops/csrc/ingest.hip) instead of ≈10 small launches
                from ..ops import require
                out = torch.empty_like(a)
                require().adv_normalize(a, v, out, float(EPS))
                d['adv'] = out
                return
            v = d['valid']
            n = v.sum().clamp_min(1.0)
            mu = (d['adv'] * v).sum() / n
            sd = (((d['adv'] - mu) ** 2 * v).sum() / n).sqrt()
            d['adv'] = ((d['adv'] - mu) / (sd + EPS)) * v

    def _to_device(self, seqs: List[Sequence]) -> Dict[str, torch.Tensor]:
        def st(name, dtype):
            a = np.stack([getattr(s, name) for s in seqs])
            t = torch.from_numpy(np.ascontiguousarray(a)).to(dtype)
            if self.device.type == 'cuda':
                t = t.pin_memory()
            return t.to(self.device, non_blocking=True)
        d = {'env': st('env', torch.float32), 'units': st('units', torch.float32),
             'actions': st('actions', torch.uint8), 'masks': st('masks', torch.uint8),
             'ret': st('discounted_rewards', torch.float32), 'norm_ret': st('norm_discounted_rewards', torch.float32),
             'adv': st('adv', torch.float32), 'logp_old': st('logp', torch.float32), 'valid': st('valid', torch.float32)}
        if self.policy.is_recurrent:
            h = st('hidden', torch.float32)
            d['h0'], d['c0'] = h[:, 0].contiguous(), h[:, 1].contiguous()
        self._normalize_advantages(d)
        return d

    # ------------------------------------------------------------------------------------------------
    def run(self, iterations: Optional[int] = None):
        cfg = self.cfg
        end = self.iteration_start + iterations if iterations is not None else cfg.iterations
        try:
            for it in range(self.iteration_start, end):
                self._last_iteration = it == end - 1      # no look-ahead: nothing would train on it
                self.run_iteration(it)
            self.flush_metrics()
        finally:
            self._last_iteration = False
            self.close()
            self.flush_checkpoints()
            if self.uploader is not None:
                self.uploader.flush()
        return end

    def flush_checkpoints(self):
        """Wait for the background publishes / checkpoint writes (``async_checkpoint``); re-raises the first failure
        on this thread, as the synchronous path would have. A publish coalesced away at the end of the run (the
        writer was busy) is made here, so the last iteration's model and trainer state always reach the actors and
        the disk."""
        skipped = getattr(self, '_pub_skipped', None)
        if skipped is not None:
            f = getattr(self, '_pub_future', None)
            if f is not None:
                f.result()
            self._pub_skipped = None
            self._upload_model_async(skipped)
        self._check_background(wait=True)

    def _check_background(self, wait: bool = False):
        """Surface failures of the ordered background writer: a failed model publish or checkpoint write must stop
        the learner (actors would otherwise keep playing stale weights with nothing reported)."""
        pending = self.__dict__.setdefault('_bg_futures', [])
        keep = []
        for f in pending:
            if wait or f.done():
                f.result()                  # raises the writer's exception here
            else:
                keep.append(f)
        self._bg_futures = keep

    def _submit_background(self, fn, *args):
        self._check_background()
        f = self._ckpt_pool_get().submit(fn, *args)
        self.__dict__.setdefault('_bg_futures', []).append(f)
        return f

    def _pipelined(self) -> bool:
        return self.ingest == 'device' and self.device.type == 'cuda' and self.cfg.prefetch_rollouts > 0

    def run_iteration(self, it: int):
        cfg = self.cfg
        self.timer.start('ingest')
        experiences: List[Sequence] = []
        rollouts: List[Rollout] = []
        n_seq = 0
        staged = None
        ahead = getattr(self, '_lookahead', None)
        self._lookahead = None
        if ahead is not None:
            # taken and expanded on the device by the previous iteration, behind its training steps
            rollouts, n_seq, n_ahead, data_ahead = ahead
        elif self._pipelined():
            # staged (decoded, packed, uploaded) by the stager thread while the previous iteration trained
            staged = self._ingest_pipeline(thread=True).get()
            rollouts, n_seq = staged.rollouts, staged.n_seq
            if self.consumed is not None:
                self.consumed.extend((r.game_id, int(r.team_id), int(r.player_id), int(r.weight_version), r.length)
                                     for r in rollouts)
        else:
            while n_seq < cfg.seq_per_epoch:
                r = self.get_rollout()
                if self.ingest == 'device':
                    rollouts.append(r)
                    n_seq += -(-r.length // cfg.seq_len)
                else:
                    experiences.extend(self.experiences_from_rollout(r))
                    n_seq = len(experiences)
                if self.ingest != 'device':
                    rollouts.append(r)
        subrewards = [r.rewards.sum(axis=0) for r in rollouts]
        rollout_lens = [r.length for r in rollouts]
        weight_ages = [it - r.weight_version for r in rollouts]
        canvas = rollouts[-1].canvas
        self.timer.stop('ingest')
        # all sequences of this iteration go to the device once; minibatches are gathered on-device
        self.timer.start('h2d')
        if ahead is not None:
            n, data = n_ahead, data_ahead
        else:
            n = self._agree_steps(n_seq - n_seq % cfg.batch_size)
            if staged is not None:
                data = self._finish_ingest(staged, n)
            elif self.ingest == 'device':
                data = self._ingest_device(rollouts, n)
            else:
                data = self._to_device(experiences[:n])
        self.timer.stop('h2d')
        self.timer.start('train')
        losses, metrics_acc = [], {}
        prox = data.pop('_prox', None) if isinstance(data, dict) else None
        if prox:
            for k, v in prox.items():
                metrics_acc[k] = [v]
        g = torch.Generator().manual_seed(cfg.seed * 1000003 + it)
        cuda = self.device.type == 'cuda'
        ev_t0 = ev_t1 = None
        if cuda:
            # in-loop GPU time of this iteration's steps (e2e.learner_gpu_ms_per_step): actor graph replays on the same
            # device, host enqueue gaps and all
            ev_t0 = torch.cuda.Event(enable_timing=True)
            ev_t0.record()
        if self.replay is not None:
            # fresh sequences go into the on-HBM ring; minibatches are sampled from it on-device
            self.replay.add(data, version=it)
            if cfg.replay_prefill and self.replay.fill_fraction < 1.0:
                self.replay.prefill()
            for _ in range(cfg.epochs * (n // cfg.batch_size)):
                m = self.learner.train_step_replay(self.replay, cfg.batch_size, cfg.replay_recent or None)
                losses.append(m['loss'])
                for k, v in m.items():
                    metrics_acc.setdefault(k, []).append(v)
        pool = self._iteration_pool(data, n) if (self.replay is None and self.learner.direct()) else None
        for ep in range(cfg.epochs if self.replay is None else 0):
            perm = torch.randperm(n, generator=g)
            if cuda:
                # one pinned, non-blocking upload per epoch: a pageable .to(device) per minibatch made the host wait
                # for the GPU to drain every previous step before it could enqueue the next (a bubble per step)
                perm = perm.pin_memory().to(self.device, non_blocking=True)
            for b0 in range(0, n, cfg.batch_size):
                idx = perm[b0:b0 + cfg.batch_size]
                if not cuda:
                    idx = idx.to(self.device)
                if pool is not None:
                    # the captured step gathers its minibatch time-major from the pool itself (replay_gather)
                    m = self.learner.train_step_indices(pool, idx)
                else:
                    batch = {k: v.index_select(0, idx) for k, v in data.items()}
                    m = self.learner.train_step(batch)
                losses.append(m['loss'])
                for k, v in m.items():
                    metrics_acc.setdefault(k, []).append(v)
        if cuda:
            ev_t1 = torch.cuda.Event(enable_timing=True)
            ev_t1.record()
        defer = self._defer_metrics()
        published = False
        if defer and self.checkpoint:
            # publish BEFORE the look-ahead: the device snapshot of this iteration's weights is queued behind its
            # steps now, so actors get them one iteration sooner than after the next iteration's data arrived
            # (a non-finite step never reaches the weights: the fused Adam skips it on the device)
            self.timer.stop('train')
            self.timer.start('publish')
            self.upload_model(version=it)
            self.timer.stop('publish')
            self.timer.start('train')
            published = True
        ema_snap = self.ema.clone() if (self.ingest == 'device' and (defer or cfg.lookahead_ingest)) else None
        if self._pipelined() and cfg.lookahead_ingest and not getattr(self, '_last_iteration', False):
            # the next iteration's rollouts: staged data taken now and expanded + scanned on the device behind this
            # iteration's steps (the pool / replay copy above already holds this iteration's rows); the EMA state
            # this iteration reports is the snapshot above (the look-ahead scan advances it)
            self.timer.stop('train')
            self.timer.start('lookahead')
            st2 = self._ingest_pipeline(thread=True).get()
            self.timer.add('stage', st2.stage_s)
            self.timer.add('gather', st2.gather_s)
            self.timer.add('stage_wait', st2.wait_s)
            self.timer.add('stage_copy', st2.copy_s)
            self.timer.add('stage_release', st2.release_s)
            if self.consumed is not None:
                self.consumed.extend((r.game_id, int(r.team_id), int(r.player_id), int(r.weight_version), r.length)
                                     for r in st2.rollouts)
            n2 = self._agree_steps(st2.n_seq - st2.n_seq % cfg.batch_size)
            self._lookahead = (st2.rollouts, st2.n_seq, n2, self._finish_ingest(st2, n2))
            self.timer.stop('lookahead')
            self.timer.start('train')
        done = None
        host = None
        if cuda:
            host = self._host_snapshot(losses, metrics_acc, ema_snap) if defer else None
            # a blocking-sync event: the host thread sleeps until the GPU is done instead of spinning a core that
            # the node's actor threads (same CPU share) can use
            done = torch.cuda.Event(blocking=True)
            done.record()
        pending = dict(it=it, losses=losses, metrics_acc=metrics_acc, ema_snap=ema_snap, n_seq=n_seq,
                       subrewards=subrewards, rollout_lens=rollout_lens, weight_ages=weight_ages, canvas=canvas,
                       done=done, ev=(ev_t0, ev_t1), n_train=len(losses), published=published,
                       n_rollouts=len(rollouts), host=host)
        self.timer.stop('train')
        if defer:
            # one-iteration-deferred metrics: this iteration's steps stay queued on the GPU while the host finalises
            # the PREVIOUS iteration (its event has long completed) and returns to ingest the next one
            prev, self._pending_metrics = getattr(self, '_pending_metrics', None), pending
            if prev is not None:
                self._finalize_iteration(prev)
        else:
            self._finalize_iteration(pending)

    def _host_snapshot(self, losses, metrics_acc, ema_snap):
        """Everything :meth:`_finalize_iteration` reads from the device — the losses, every metric's iteration mean, the
        reward-EMA snapshot and the learner's error flags — packed into ONE vector and copied into pinned host memory
        behind this iteration's steps (no host sync). Finalising the previous iteration with ``.cpu()`` / ``.item()``
        reads instead queued those copies behind the CURRENT iteration's steps and made the host wait for the GPU to
        drain before it could enqueue the next iteration: a GPU bubble of host time per iteration in the node loop."""
        if not losses or not all(torch.is_tensor(x) and x.is_cuda for x in losses):
            return None
        keys = list(metrics_acc)
        # every per-step value flat in ONE concatenation (the per-key means are taken on the host): a stack + mean
        # per metric key was ≈40 small launches per iteration on the learner's stream
        parts = [x.reshape(-1).float() for x in losses]
        seg = []
        for k in keys:
            vs = [v.reshape(-1).float() for v in metrics_acc[k]]
            seg.append(sum(v.numel() for v in vs))
            parts += vs
        n_ema = 0
        if ema_snap is not None:
            parts.append(ema_snap.float().reshape(-1))
            n_ema = ema_snap.numel()
        flags = [f.float().reshape(-1)[:1] for f in self.learner.error_flags()]
        parts += flags
        vec = torch.cat(parts)
        buf = self.__dict__.setdefault('_host_bufs', [])
        # two pinned buffers alternate (the previous iteration's is read while this one's copy is in flight)
        while len(buf) < 2:
            buf.append(torch.empty(0, dtype=torch.float32).pin_memory())
        i = self.__dict__.get('_host_buf_i', 0)
        self._host_buf_i = 1 - i
        if buf[i].numel() < vec.numel():
            buf[i] = torch.empty(max(vec.numel(), 2 * buf[i].numel()), dtype=torch.float32).pin_memory()
        h = buf[i][:vec.numel()]
        h.copy_(vec, non_blocking=True)
        return dict(vec=h, n_loss=sum(x.numel() for x in losses), keys=keys, seg=seg, n_ema=n_ema,
                    ema_shape=tuple(ema_snap.shape) if ema_snap is not None else None, n_flags=len(flags))

    def _defer_metrics(self) -> bool:
        return self._pipelined() and self.cfg.defer_metrics and self.cfg.async_checkpoint

    def flush_metrics(self):
        """Finalise the iteration whose metrics are still pending (deferred mode): the last one of a run."""
        prev = getattr(self, '_pending_metrics', None)
        self._pending_metrics = None
        if prev is not None:
            self._finalize_iteration(prev)

    def _finalize_iteration(self, p):
        """Metrics, NaN / kernel-error checks, logs and (unless already done) the model publish of iteration
        ``p['it']`` — the reference's end of iteration (optimizer.py:476-563)."""
        cfg = self.cfg
        it = p['it']
        if p['done'] is not None:
            p['done'].synchronize()
        hs = p.get('host')
        if hs is not None:
            # the pinned snapshot of the device values (_host_snapshot): complete once ``done`` is, no further syncs
            v = hs['vec'].clone()
            nl, ne = hs['n_loss'], hs['n_ema']
            loss_t = v[:nl]
            means, o = [], nl
            for c in hs['seg']:
                means.append(float(v[o:o + c].double().mean()) if c else float('nan'))
                o += c
            ema_host = v[o:o + ne].view(hs['ema_shape']) if ne else None
            flags = v[o + ne:]
        else:
            loss_t = torch.stack(p['losses']).float().cpu()
        if faults().nan_loss(it):
            loss_t[0] = float('nan')
        if torch.isnan(loss_t).any():
            raise ValueError(f'NaN loss at iteration {it}: {loss_t.tolist()}')
        if hs is None or bool((flags != 0).any()):
            self.learner.check_error()          # (the snapshot path: host syncs only when a flag is up)
        n_steps = p['n_seq'] * cfg.seq_len
        if self.ingest == 'device':
            self._sync_running(ema_host if (hs is not None and ema_host is not None) else p['ema_snap'])
        now = time.time()
        steps_per_s = n_steps / max(now - self.time_last_step, 1e-9)
        self.time_last_step = now
        sub = np.stack(p['subrewards']) / n_steps * OBSERVATIONS_PER_SECOND
        rollout_rewards = sub.sum(axis=1)
        reward_dict = dict(zip(REWARD_KEYS, sub.sum(axis=0)))
        # every metric's iteration mean in ONE device→host copy (not one synchronising .item() per metric)
        metrics_acc = p['metrics_acc']
        if hs is not None:
            keys = hs['keys']
        else:
            keys = list(metrics_acc)
            means = torch.stack([torch.stack(metrics_acc[k]).float().mean() for k in keys]).cpu().tolist()
        mean = dict(zip(keys, means))
        rollout_lens, weight_ages = p['rollout_lens'], p['weight_ages']
        metrics = {
            self.SPEED_KEY: steps_per_s,
            'samples per s per gpu': steps_per_s * cfg.epochs,
            'reward_per_sec/sum': float(rollout_rewards.sum()),
            'loss/sum': mean['loss'], 'loss/policy': mean['policy_loss'], 'loss/entropy': mean['entropy_loss'],
            'loss/advantage': mean['advantage_loss'], 'entropy': mean['entropy'], 'advantage': mean['advantage'],
            'avg_rollout_len': float(np.mean(rollout_lens)), 'avg_weight_age': float(np.mean(weight_ages)),
            'experience_steps': float(np.sum(rollout_lens)),
            'rollouts_consumed': float(p['n_rollouts']),
            'grad_norm': mean['grad_norm'],
        }
        e0, e1 = p['ev']
        if e0 is not None and p['n_train']:
            metrics['time/gpu_train_ms_per_step'] = e0.elapsed_time(e1) / p['n_train']
        for k in ('approx_kl', 'clipfrac'):
            if k in mean:
                metrics[k] = mean[k]
        for k in mean:
            if k.startswith('offpolicy/'):
                metrics[k] = mean[k]
        if self.replay is not None:
            metrics['replay/size'] = float(len(self.replay))
        for team, v in self.running.mean.items():
            metrics[f'rewards/running_mean_{team}'] = v
        for team, v in self.running.std.items():
            metrics[f'rewards/running_std_{team}'] = v
        for k in ('enum', 'x', 'y', 'target_unit'):
            metrics[f'entropy/{k}'] = mean[f'entropy/{k}']
        for k, v in reward_dict.items():
            metrics[f'reward_per_sec/{k}'] = float(v)
        metrics.update(self.timer.pop())
        logger.info('it=%d steps_per_s=%.1f avg_weight_age=%.1f reward_per_sec=%.4f loss=%.4f entropy=%.3f', it,
                    steps_per_s, metrics['avg_weight_age'], metrics['reward_per_sec/sum'], metrics['loss/sum'],
                    metrics['entropy'])
        self.last_metrics = metrics
        if self.checkpoint:
            self.timer.start('log')
            hist = None
            if it % cfg.histogram_freq == 1:
                hist = {name: p_.detach().float().cpu().numpy() for name, p_ in self.policy.named_parameters()}
            qs = getattr(self.broker, 'xp_queue_size', None)
            job = (self._write_logs, it, metrics, loss_t.numpy(), np.asarray(rollout_lens), np.asarray(weight_ages),
                   rollout_rewards, hist, p['canvas'], qs)
            if cfg.async_checkpoint and self.device.type == 'cuda':
                self._submit_background(*job)         # tensorboard events + their upload on the ordered writer
            else:
                job[0](*job[1:])
            self.timer.stop('log')
            if not p['published']:
                self.timer.start('publish')
                self.upload_model(version=it)
                self.timer.stop('publish')

    def _write_logs(self, it, metrics, losses, rollout_lens, weight_ages, rollout_rewards, hist, canvas, qs):
        """The reference's tensorboard scalars / histograms / canvas image (optimizer.py:500-561) and the events
        file upload (GCS role, :559-561)."""
        w = self.writer
        w.add_scalars(metrics, it)
        w.add_histogram('losses', losses, it)
        w.add_histogram('rollout_lens', rollout_lens, it)
        w.add_histogram('weight_age', weight_ages, it)
        w.add_histogram('rewards_per_sec_per_rollout', rollout_rewards, it)
        if hist is not None:
            for name, v in hist.items():
                w.add_histogram('param/' + name, v, it)
            w.add_image('canvas', canvas, it)
        if qs is not None:
            w.add_scalar('mq_size', qs, it)
        w.flush()
        if self.uploader is not None and w.events_filename:
            # upload a snapshot: the live events file keeps growing while the uploader copies
            import shutil
            snap = w.events_filename + '.snapshot'
            shutil.copyfile(w.events_filename, snap)
            self.uploader.submit(snap, f'{self.store_prefix}/{os.path.basename(w.events_filename)}')

    def upload_model(self, version: int):
        if not self.checkpoint:
            return
        if self.cfg.async_checkpoint and self.device.type == 'cuda' and version > 0:
            return self._upload_model_async(version)
        import io
        sd = {k: v.detach().cpu() for k, v in self.policy.state_dict().items()}
        buf = io.BytesIO()
        torch.save(sd, buf)
        data = buf.getvalue()
        trainer = {'learner': _to_cpu(self.learner.state_dict()), 'running': self.running.state_dict(),
                   'iteration': version, 'config': asdict(self.cfg)}
        if not self.cfg.async_checkpoint:
            self._write_checkpoint(data, trainer, version)
            self.broker.publish_model(data, version)
            self.n_published += 1
            return
        # publish first (actors see the new weights now); the files follow on one ordered background writer
        self.broker.publish_model(data, version)
        self.n_published += 1
        self._submit_background(self._write_checkpoint, data, trainer, version)

    def _ckpt_pool_get(self):
        if getattr(self, '_ckpt_pool', None) is None:
            from concurrent.futures import ThreadPoolExecutor
            self._ckpt_pool = ThreadPoolExecutor(1, thread_name_prefix='ckpt')
        return self._ckpt_pool

    def _upload_model_async(self, version: int):
        """GPU learner with ``async_checkpoint``: the main thread only snapshots the weights and optimizer state ON
        THE DEVICE — four flat clones (parameters, Adam moments, step counts) queued behind this iteration's steps
        plus an event, no per-tensor launches, no host sync; host copies on a stream of the writer's own,
        state-dict assembly, serialisation, the model publish and the files run on the ordered background writer,
        overlapping the next iteration's ingest and training."""
        # coalescing: while the writer is still busy with the previous publish, this version is skipped (the next
        # iteration's publishes newer weights anyway). Without it a learner iterating faster than one serialise +
        # publish + checkpoint write (≈20 ms iterations vs ≈88 MB of files each) queued snapshots without bound —
        # device memory and weight age growing for the whole run
        f = getattr(self, '_pub_future', None)
        if f is not None and not f.done():
            self.n_publish_coalesced = getattr(self, 'n_publish_coalesced', 0) + 1
            self._pub_skipped = version
            return
        self._pub_skipped = None
        fl, opt = self.learner.flat, self.learner.opt
        snap = {'flat': fl.flat.detach().clone(), 'exp_avg': opt.exp_avg.clone(), 'exp_avg_sq': opt.exp_avg_sq.clone(),
                'steps': opt.steps.clone()}
        if self.ingest == 'device':
            # the reward-normalisation EMA as of these weights (the host mirror may still be an iteration behind
            # when metrics are deferred): copied with the snapshot, folded into the trainer state by the writer
            snap['ema'] = self.ema.clone()
        meta = {'n_steps': self.learner.n_steps, 'running': copy.deepcopy(self.running.state_dict()),
                'hparams': {'lr': opt.lr, 'betas': opt.betas, 'eps': opt.eps, 'max_grad_norm': opt.max_grad_norm},
                'layout': opt.layout()}
        ev = torch.cuda.Event()
        ev.record()
        self._pub_future = self._submit_background(self._publish_snapshot, snap, meta, ev, version)

    def _publish_snapshot(self, snap, meta, ev, version: int):
        import io
        from .engine import CAPTURE_LOCK
        # the device → host copies (and the release of the device snapshot) stay out of a step-graph capture window
        with CAPTURE_LOCK:
            st = getattr(self, '_pub_stream', None)
            if st is None:
                st = self._pub_stream = torch.cuda.Stream(device=self.device)
            with torch.cuda.stream(st):
                st.wait_event(ev)
                snap = _to_cpu(snap)
        fl = self.learner.flat
        flat = snap['flat']
        if 'ema' in snap:
            e = snap.pop('ema')
            run = meta['running']
            for team, k in self.team_keys.items():
                if e[k, 2] != 0:
                    run['mean'][team] = float(e[k, 0])
                    run['std'][team] = float(e[k, 1])
        # own storage per tensor: the message / checkpoint holds exactly the reference's 30 state_dict tensors
        params = {n: flat[o:o + k].view(p.shape).clone() for n, p, o, k in zip(fl.names, fl.params, fl.offsets,
                                                                               fl.numel)}
        sd = {k: params[k] for k in self.policy.state_dict().keys()}
        optim = {'exp_avg': snap['exp_avg'], 'exp_avg_sq': snap['exp_avg_sq'], 'steps': snap['steps'],
                 'layout': meta['layout'], **meta['hparams']}
        trainer = {'learner': {'optimizer': optim, 'n_steps': meta['n_steps']}, 'running': meta['running'],
                   'iteration': version, 'config': asdict(self.cfg)}
        buf = io.BytesIO()
        torch.save(sd, buf)
        data = buf.getvalue()
        self.broker.publish_model(data, version)
        self.n_published += 1
        self._write_checkpoint(data, trainer, version)

    def _write_checkpoint(self, data: bytes, trainer, version: int):
        path = ckpt.write_model_bytes(data, self.cfg.log_dir, version)
        spath = ckpt.save_trainer_state(trainer, self.cfg.log_dir, version)
        if self.uploader is not None:   # reference optimizer.py:713-715 (GCS upload of the model file)
            self.uploader.submit(path, f'{self.store_prefix}/{os.path.basename(path)}')
            self.uploader.submit(spath, f'{self.store_prefix}/{os.path.basename(spath)}')
            self.uploader.flush()       # a pruned file must not vanish before its upload
        ckpt.prune(self.cfg.log_dir, self.cfg.checkpoint_keep)


class _RingClaim:
    """The release of one claimed ring message (Rollout.release): exactly once, budget given back. ``release_all``
    gives a batch back under one ring lock per broker (the stager releases an iteration's rollouts together)."""
    __slots__ = ('broker', 'token', 'n', 'cb', 'done')

    def __init__(self, broker, token, n, cb):
        self.broker, self.token, self.n, self.cb, self.done = broker, token, n, cb, False

    def __call__(self):
        if not self.done:
            self.done = True
            self.broker.release_experience(self.token)
            self.cb.give(self.n)

    def valid(self) -> bool:
        """Whether the claim still owns its ring region (False once the ring abandoned and reclaimed it)."""
        f = getattr(self.broker, 'claim_valid', None)
        return True if (f is None or self.done) else f(self.token)

    @staticmethod
    def release_all(claims):
        groups = {}
        for c in claims:
            if not c.done:
                c.done = True
                groups.setdefault(id(c.broker), []).append(c)
        for cs in groups.values():
            b = cs[0].broker
            many = getattr(b, 'release_experience_many', None)
            if many is not None:
                many([c.token for c in cs])
            else:
                for c in cs:
                    b.release_experience(c.token)
            for c in cs:
                c.cb.give(c.n)


class _ClaimBudget:
    """Bytes of ring-resident (claimed, not yet released) messages the learner may hold at once."""

    def __init__(self, limit: int):
        import threading
        self.limit = int(limit)
        self.held = 0
        self.lock = threading.Lock()

    def available(self) -> bool:
        with self.lock:
            return self.held < self.limit

    def take(self, n: int) -> int:
        with self.lock:
            self.held += n
        return n

    def give(self, n: int):
        with self.lock:
            self.held -= n


class _RolloutPrefetcher:
    """Background consume + decode of experience messages into a bounded queue. The learner's main thread then only
    waits when the actors are behind; DCX1 decode (CRC, array views) and broker waits overlap the GPU training of the
    previous iteration. An exception in the thread (e.g. the experience timeout) is re-raised by :meth:`get`.

    ``threads`` > 1: several decode threads feed the queue (arrival order is then not the queue's order, as with
    competing consumers anyway). The node loop uses one: its 2 000 rollouts/s once looked decode-bound at ≈15 ms of
    stager wait per iteration, which was the look-ahead ingest's GIL-held stream wait (returns scan), not the CRC."""

    def __init__(self, fetch, depth: int, threads: int = 1):
        import queue
        import threading
        self._queue_mod = queue
        self.q = queue.Queue(maxsize=max(1, depth))
        self.fetch = fetch
        self.err: Optional[BaseException] = None
        self.lost = 0
        self.put_wait = 0.0                 # s the decode threads waited for room in the queue (stager behind)
        self._lost_lock = threading.Lock()
        self.stop = threading.Event()
        self.threads = [threading.Thread(target=self._run, name=f'xp-prefetch-{i}', daemon=True)
                        for i in range(max(1, int(threads)))]
        self.th = self.threads[0]
        for t in self.threads:
            t.start()

    def _run(self):
        try:
            while not self.stop.is_set():
                r = self.fetch(self.stop)
                if r is None:
                    break
                tp = time.perf_counter()
                while True:
                    try:
                        self.q.put(r, timeout=0.1)
                        self.put_wait += time.perf_counter() - tp
                        break
                    except self._queue_mod.Full:
                        if self.stop.is_set():
                            with self._lost_lock:
                                self.lost += 1
                            _release(r)
                            return
        except BaseException as e:       # surfaced on the consumer's thread
            self.err = e

    def get(self) -> Rollout:
        while True:
            try:
                return self.q.get(timeout=0.05)
            except self._queue_mod.Empty:
                if self.err is not None:
                    raise self.err
                if not any(t.is_alive() for t in self.threads):
                    raise RuntimeError('experience prefetch thread exited')

    def get_until(self, stop) -> Optional[Rollout]:
        """:meth:`get` for a consumer thread of its own (the ingest stager): None once ``stop`` is set."""
        while not stop.is_set():
            try:
                return self.q.get(timeout=0.05)
            except self._queue_mod.Empty:
                if self.err is not None:
                    raise self.err
                if not any(t.is_alive() for t in self.threads):
                    raise RuntimeError('experience prefetch thread exited')
        return None

    def close(self) -> int:
        """Stop and join the thread (it polls the queue in bounded slices); returns the decoded rollouts dropped."""
        self.stop.set()
        for t in self.threads:
            t.join(timeout=30.0)
        if any(t.is_alive() for t in self.threads):
            raise RuntimeError('experience prefetch thread did not stop')
        n = self.lost
        while True:
            try:
                _release(self.q.get_nowait())
            except self._queue_mod.Empty:
                break
            n += 1
        return n


def _release(r):
    """Give a ring-resident rollout's region back (a dropped one: nothing of it is read any more)."""
    rel = getattr(r, 'release', None)
    if rel is not None:
        r.release = None
        rel()


def _to_cpu(x):
    """Host snapshot of a (nested) state dict: device tensors copied now, so a background writer sees this step."""
    if isinstance(x, torch.Tensor):
        return x.detach().cpu()
    if isinstance(x, dict):
        return {k: _to_cpu(v) for k, v in x.items()}
    if isinstance(x, (list, tuple)):
        return type(x)(_to_cpu(v) for v in x)
    return x
