"""Learner engine: one optimizer step (forward → loss → backward → DP all-reduce → clip + Adam).

This is the inner hot loop of the reference's ``DotaOptimizer.train`` (optimizer.py:565-688), re-organised around
flat parameter/gradient buffers so that the data-parallel reduction is a few bucketed RCCL collectives and the
optimizer is one fused HIP kernel pair.

Backends for the model math:

* ``'fused'`` (default on GPU): :class:`~dotaclient_amd.models.fused.FusedPolicy` — every product of the step in a
  hand-written gfx950 HIP kernel (entity encoder, attention block, forward / ∂X chains, recurrence, heads + loss,
  split-K weight-gradient GEMMs, clip + Adam); no vendor GEMM.
* ``'torch'``: the eager reference model (``models.policy.Policy``, the oracle): fp32, or under bf16 autocast on GPU
  with ``precision='bf16'`` (the only way a bf16 learner runs: the fused step has no bf16 branch).

``precision``: ``'fp32-exact'`` — the reference's training precision (optimizer.py:281 trains the fp32 module) with
every product an IEEE fp32 FMA; the default of the CLI, the presets and ``bench.py`` (``OptimizerConfig.precision``).
``'fp32'`` (this class's default, kept for the many short-horizon tests) keeps activations, gradients and
accumulation in fp32 with bf16x3-split MFMA operands (``models/fused.py``); ``'bf16'`` = torch backend under autocast.

Batches are dicts of device tensors (see :func:`dotaclient_amd.learner.synthetic.make_batch` for the schema):
``env (B,S,3) f32``, ``units (B,S,U,10) f32``, ``actions``/``masks (B,S,A) u8`` (flat ``enum|x|y|target_unit``),
``adv``/``ret``/``logp_old``/``norm_ret (B,S) f32`` and for recurrent policies ``h0``/``c0 (B,H) f32``.
"""
from __future__ import annotations

import contextlib
import itertools
import os
import threading
from dataclasses import dataclass
from typing import Dict, List, Optional

import torch

from ..models.policy import Policy
from ..parallel.dp import DataParallel, FlatParams
from .losses import ppo_loss, split_heads, vpg_loss
from .optim import FlatAdam


# Held while the learner captures a step graph: background threads of the learner process (the ingest stager's
# rare buffer growth) take it around their pinned / device allocations, so no allocation from another thread lands
# inside a capture window (HIP invalidates a capture on some cross-thread API calls even in thread-local mode).
CAPTURE_LOCK = threading.RLock()


_GRAPH_TOKENS = itertools.count(1)   # replay-graph cache tokens (Learner._replay_key)


def _capture_stream(device):
    """The graph-capture stream (default priority: high priority measured slower, profiles/r4_stream_priority_ab.txt)."""
    return torch.cuda.Stream(device=device)


@dataclass

class LossConfig:
    algo: str = 'ppo'                 # 'ppo' (north star) | 'vpg' (reference objective)
    learning_rate: float = 1e-4       # optimizer.py:778
    entropy_coef: float = 0.01        # optimizer.py:779
    vf_coef: float = 0.5              # optimizer.py:780
    clip_eps: float = 0.1             # e_clip, optimizer.py:239
    gamma: float = 0.98               # optimizer.py:382
    gae_lambda: float = 0.95
    max_grad_norm: float = 0.5        # optimizer.py:215
    compat_value_bug: bool = False    # optimizer.py:603 broadcast quirk
    # PPO policy term: 'clip' = the clipped surrogate against logp_old (fresh experience: logp_old is the learner's own
    # log-prob at the iteration's weights, learner/optimizer.py old_logp='learner'); 'tis' = off-policy policy
    # gradient with the truncated importance weight min(1, π/π_old) (replayed experience, V-trace style)
    offpolicy: str = 'clip'
    # V-trace inside the step: the advantages and value targets of every minibatch recomputed from the step's own
    # values and log-probs against the actor's behaviour log-prob (``logp_old``) — batches carry the per-row ``vt``
    # field {reward, bootstrap, valid, last} (learner/optimizer.py advantages='vtrace-step'); ``adv`` / ``ret`` unused
    vtrace: bool = False
    vtrace_rho_bar: float = 1.0
    vtrace_c_bar: float = 1.0


class Learner:
    def __init__(self, policy: Policy, loss_cfg: LossConfig, device='cpu', backend: str = 'auto',
                 bucket_cap_mb: float = 8.0, overlap: bool = True, dp: bool = True, precision: str = 'fp32'):
        if precision not in ('fp32', 'bf16', 'fp32-exact'):
            raise ValueError(f'precision must be fp32, fp32-exact or bf16, got {precision!r}')
        self.device = torch.device(device)
        self.cfg = loss_cfg
        self.precision = precision
        self.policy = policy.to(self.device)
        auto = backend == 'auto'
        if auto:
            backend = 'fused' if self.device.type == 'cuda' else 'torch'
        self.backend = backend
        self.flat = FlatParams(self.policy, device=self.device)
        self.dp = DataParallel(self.policy, flat=self.flat, bucket_cap_mb=bucket_cap_mb, overlap=overlap,
                               broadcast=dp)
        self.opt = FlatAdam(self.flat, lr=loss_cfg.learning_rate, max_grad_norm=loss_cfg.max_grad_norm,
                            use_kernels=self.device.type == 'cuda')
        self.model = self.policy
        if backend == 'fused':
            from ..models.fused import FusedPolicy
            fused = FusedPolicy(self.policy, loss_cfg, precision=precision)
            if fused.use_pipeline():
                self.model = fused
                self.model.attach_flat(self.flat.flat)
            elif auto:
                self.backend = backend = 'torch'     # a configuration the kernels do not cover
            else:
                raise ValueError(f'backend fused: no kernel path for {self.policy.config} at {precision}')
        self.counts = self.policy.layout.action_counts()
        self.n_steps = 0
        self.graph = None                 # captured forward+backward (see enable_graph)
        self._static_idx: Dict[tuple, torch.Tensor] = {}    # per replay-graph key: its captured index buffer
        self._graph_warmup = 0

    def enable_graph(self, warmup: int = 2):
        """Capture forward + loss + backward of the fused step in a hipGraph after ``warmup`` eager steps. The
        step launches a few hundred kernels (per-chunk GEMMs, the persistent recurrence, fused kernels); eager
        Python + hipBLASLt launch cost is several ms per step, a graph replay is one launch. The DP all-reduce and
        the fused Adam stay outside the graph (RCCL collectives are not captured). Inputs are copied into
        static buffers before each replay; the batch shapes must not change."""
        if self.backend != 'fused' or self.device.type != 'cuda':
            return False
        # only the forward-computed step (models/pipelined.py) is captured: it has no work in an autograd
        # backward thread (capturing _PolicyLoss's autograd backward gave wrong gradients on replay)
        if not self.model.use_pipeline():
            return False
        self._graph_warmup = max(1, int(warmup))
        return True

    # ------------------------------------------------------------------------------------------------
    def _autocast(self):
        if self.backend == 'torch' and self.device.type == 'cuda' and self.precision == 'bf16':
            return torch.autocast('cuda', dtype=torch.bfloat16)
        return contextlib.nullcontext()

    def hidden_from_batch(self, batch):
        if not self.policy.is_recurrent:
            return None
        return (batch['h0'].unsqueeze(0).contiguous(), batch['c0'].unsqueeze(0).contiguous())

    def loss(self, batch: Dict[str, torch.Tensor]):
        cfg = self.cfg
        stable = not self.policy.config.compat_bugs
        if self.backend == 'fused':
            return self.model.loss(batch, cfg)
        with self._autocast():
            logits, values, _ = self.model.forward_packed(batch['env'], batch['units'], self.hidden_from_batch(batch),
                                                          reset=batch.get('reset'))
        logits = {k: v.float() for k, v in logits.items()}
        values = values.float()
        actions = split_heads(batch['actions'], self.counts)
        masks = split_heads(batch['masks'], self.counts)
        if cfg.algo == 'ppo':
            adv, ret, extra = batch['adv'], batch['ret'], {}
            if cfg.vtrace:
                adv, ret, extra = self._vtrace_torch(batch, logits, values, masks, actions)
            loss, metrics = ppo_loss(logits, values, actions, masks, adv, ret, batch['logp_old'],
                                     cfg.clip_eps, cfg.entropy_coef, cfg.vf_coef, stable=stable,
                                     offpolicy=cfg.offpolicy)
            metrics.update(extra)
            return loss, metrics
        return vpg_loss(logits, values, actions, masks, batch['norm_ret'], batch['ret'], cfg.entropy_coef,
                        cfg.vf_coef, compat_value_bug=cfg.compat_value_bug, stable=stable)

    def _vtrace_torch(self, batch, logits, values, masks, actions):
        """The torch oracle of the fused step's in-step V-trace (ops/scan.py vtrace_step over time-major rows): the
        step's own (detached) values and log-probs of the recorded actions against ``logp_old``; advantages
        normalised over the valid rows. Returns (adv (B,S), ret (B,S), off-policy metrics)."""
        from ..constants import EPS
        from ..ops.scan import vtrace_step
        from .losses import sampled_logp
        cfg = self.cfg
        B, S = batch['env'].shape[:2]
        tm = (lambda x: x.detach().float().reshape(B, S, *x.shape[2:]).transpose(0, 1).reshape(B * S, *x.shape[2:]))
        with torch.no_grad():
            lp = sampled_logp(logits, actions, masks, stable=not self.policy.config.compat_bugs)
            adv, ret, st = vtrace_step(tm(values.squeeze(-1)).cpu(), tm(lp).cpu(), tm(batch['logp_old']).cpu(),
                                       tm(batch['vt']).cpu(), B, S, cfg.gamma, cfg.gae_lambda, cfg.vtrace_rho_bar,
                                       cfg.vtrace_c_bar)
            dev = batch['env'].device
            back = (lambda x: x.reshape(S, B).t().contiguous().to(dev))
            adv, ret = back(adv), back(ret)
            v = batch['vt'][..., 2].float()
            n = v.sum().clamp_min(1.0)
            mu = (adv * v).sum() / n
            sd = (((adv - mu) ** 2 * v).sum() / n).sqrt()
            adv = ((adv - mu) / (sd + EPS)) * v
            s = st.sum(0)
            extra = {'offpolicy/rho_mean': (s[0] / s[3].clamp_min(1)).to(dev),
                     'offpolicy/rho_truncated': (s[1] / s[3].clamp_min(1)).to(dev),
                     'offpolicy/behaviour_kl': (s[2] / s[3].clamp_min(1)).to(dev)}
        return adv, ret, extra

    def _fwd_bwd(self, batch):
        self.dp.zero_grad()
        loss, metrics = self.loss(batch)
        loss.backward()
        if self.backend == 'fused' and getattr(self.model, 'direct_used', False):
            # the fused Functions accumulate straight into the flat gradient buffer (no per-parameter autograd
            # hooks fire); tell the DP layer which parameters received a gradient
            self.dp.has_grad.copy_(self.model.grad_mask)
        return {k: v.detach() for k, v in metrics.items()}

    # ---- direct (autograd-free) fused LSTM step ------------------------------------------------------
    def direct(self) -> bool:
        """The fused LSTM policy runs the autograd-free step (models/pipelined.py:train_direct)."""
        return self.backend == 'fused' and self.device.type == 'cuda' and self.model.use_pipeline()

    STEP_FIELDS = ('units', 'env', 'actions', 'masks', 'adv', 'ret', 'logp_old', 'norm_ret')

    @staticmethod
    def batch_to_time_major(batch):
        """Batch-major ``(B,S,…)`` fields → time-major rows ``(S·B,…)`` (row = t·B + b)."""
        B, S = batch['env'].shape[:2]
        out = {}
        for k in Learner.STEP_FIELDS:
            v = batch.get(k)
            if v is None:
                v = torch.zeros(B, S, device=batch['env'].device)
            out[k] = v.transpose(0, 1).reshape(S * B, *v.shape[2:]).contiguous()
        if 'reset' in batch:                # sequence packing: episode-start flags (B,S) u8 → time-major rows
            out['reset'] = batch['reset'].transpose(0, 1).reshape(S * B).contiguous()
        if 'vt' in batch:                   # in-step V-trace rows {reward, bootstrap, valid, last} (B,S,4)
            out['vt'] = batch['vt'].transpose(0, 1).reshape(S * B, 4).contiguous()
        for k in ('h0', 'c0'):
            if k in batch:
                out[k] = batch[k].contiguous()
        return out, B, S

    def gather_time_major(self, replay, idx, S: int):
        """Minibatch of replay rows ``idx`` gathered straight into time-major rows: one index_select per field
        over the pool viewed as (capacity·S, …) — no batch-major copy, no transpose."""
        B = idx.numel()
        fields = self.STEP_FIELDS + tuple(k for k in ('reset', 'vt') if k in replay.data)
        if idx.is_cuda:                 # one HIP launch for every field (ops/csrc/glue.hip replay_gather)
            from .. import ops
            seq = [k for k in ('h0', 'c0') if k in replay.data]
            outs = ops.require().replay_gather([replay.data[k] for k in fields] +
                                               [replay.data[k] for k in seq], len(fields),
                                               idx.contiguous())
            return dict(zip(list(fields) + seq, outs))
        ar = getattr(self, '_arange', None)
        if ar is None or ar.numel() < S or ar.device != idx.device:
            ar = self._arange = torch.arange(max(S, 1), device=idx.device, dtype=torch.long)
        rows = (idx.view(1, B) * S + ar[:S].view(S, 1)).reshape(-1)
        out = {}
        for k in fields:
            pool = replay.data[k]
            out[k] = pool.view(-1, *pool.shape[2:]).index_select(0, rows)
        for k in ('h0', 'c0'):
            if k in replay.data:
                out[k] = replay.data[k].index_select(0, idx)
        return out

    def _split_mode(self) -> bool:
        """Data-parallel direct step in two phases: the recurrence / pre-RNN / heads gradients are all-reduced on
        the comm stream while the encoder backward still runs (RCCL over xGMI overlapped with backward). The split
        needs the single-chunk step and a contiguous early-parameter range (DataParallel.split_buckets).
        ``DCA_DP_SPLIT=1`` forces it without a process group (single-GPU tests of the two-graph mechanics)."""
        import os
        if getattr(self, '_split', None) is None:
            force = os.environ.get('DCA_DP_SPLIT') == '1'
            ok = (self.direct() and (self.dp.enabled or force) and self.model.chunks == 1
                  and os.environ.get('DCA_DP_SPLIT', '') != '0')
            if ok:
                early = self.model.early_param_names()
                idx = [i for i, n in enumerate(self.model.param_names) if n in early]
                ok = self.dp.split_buckets(idx) if self.dp.enabled else bool(idx)
            self._split = bool(ok)
        return self._split

    def _direct_body(self, batch_tm, B, S, hook=None):
        self.flat.grad.zero_()
        if hook is None and self._split_mode():
            hook = self.dp.launch_early                   # eager step: launch the early buckets right away
        self.model.split_hook = hook
        try:
            vec = self.model.train_direct(batch_tm, B, S, self.cfg)
        finally:
            self.model.split_hook = None
        self.dp.has_grad.copy_(self.model.grad_mask)
        return vec

    def _metrics_from_vec(self, vec):
        from ..models.pipelined import METRIC_NAMES
        names = [n for n in METRIC_NAMES if (self.cfg.algo == 'ppo' or n not in ('approx_kl', 'clipfrac'))
                 and (self.cfg.vtrace or not n.startswith('offpolicy/'))]
        return {n: vec[METRIC_NAMES.index(n)] for n in names}

    def _graph_ready(self) -> bool:
        return bool(self._graph_warmup) and self.n_steps >= self._graph_warmup

    @staticmethod
    def _capture_mode() -> str:
        """Only this thread's HIP calls are capture-checked ('thread_local'): other threads of the process keep
        running while the learner captures — RCCL's watchdog querying events, or an in-process actor stepping its
        own graphs on its own streams (learner/e2e.py). Neither touches the capturing stream."""
        return 'thread_local'

    def _replay_split(self, key, body):
        """Split-mode capture/replay: ``body(hook)`` is captured as TWO graphs — the hook, called once by the step
        at its split point, ends the first capture and begins the second (same memory pool). Replay: graph 1, then
        the early buckets' all-reduce on the comm stream, then graph 2 overlapping it."""
        graphs = self.__dict__.setdefault('_graphs', {})
        if key not in graphs:
            if getattr(self, '_graph_stream', None) is None:
                self._graph_stream = _capture_stream(self.device)
            s = self._graph_stream
            cur = torch.cuda.current_stream(self.device)
            s.wait_stream(cur)
            with torch.cuda.stream(s):              # eager warm-up on the capture stream, no collectives
                body(lambda: None)
            cur.wait_stream(s)
            mode = self._capture_mode()
            g1, g2 = torch.cuda.CUDAGraph(), torch.cuda.CUDAGraph()
            switched = []

            def switch():
                g1.capture_end()
                g2.capture_begin(pool=g1.pool(), capture_error_mode=mode)
                switched.append(True)

            torch.cuda.synchronize(self.device)
            with CAPTURE_LOCK, torch.cuda.stream(s):
                g1.capture_begin(capture_error_mode=mode)
                out = body(switch)
                if not switched:
                    raise RuntimeError('direct step never reached its DP split point')
                g2.capture_end()
            cur.wait_stream(s)
            graphs[key] = ((g1, g2), out)
            self.graph = g1
        (g1, g2), out = graphs[key]
        g1.replay()
        self.dp.launch_early()
        g2.replay()
        return out

    def _replay_graph(self, key, body):
        """Capture ``body`` (a function of the static inputs) once per key, then replay it."""
        graphs = self.__dict__.setdefault('_graphs', {})
        if key not in graphs:
            # the capture stream must outlive the graph: hipBLASLt's per-stream workspace that the captured GEMM
            # nodes point at belongs to it
            if getattr(self, '_graph_stream', None) is None:
                self._graph_stream = _capture_stream(self.device)
            s = self._graph_stream
            cur = torch.cuda.current_stream(self.device)
            s.wait_stream(cur)
            with torch.cuda.stream(s):          # one more eager run on the capture stream (allocator warm-up)
                body()
            cur.wait_stream(s)
            g = torch.cuda.CUDAGraph()
            with CAPTURE_LOCK, torch.cuda.graph(g, stream=s, capture_error_mode=self._capture_mode()):
                out = body()
            graphs[key] = (g, out)
            self.graph = g
        g, out = graphs[key]
        g.replay()
        return out

    def _step_direct_batch(self, batch):
        if not self._graph_ready():
            bt, B, S = self.batch_to_time_major(batch)
            return self._direct_body(bt, B, S)
        B, S = batch['env'].shape[:2]
        key = ('batch', B, S, tuple(sorted(batch)))
        if key not in self.__dict__.get('_graphs', {}):
            self._static_in = {k: v.clone() for k, v in batch.items()}
        else:
            for k, v in batch.items():
                self._static_in[k].copy_(v, non_blocking=True)

        if self._split_mode():
            def body_split(hook):
                bt, B_, S_ = self.batch_to_time_major(self._static_in)
                return self._direct_body(bt, B_, S_, hook=hook)
            return self._replay_split(key, body_split)

        def body():
            bt, B_, S_ = self.batch_to_time_major(self._static_in)
            return self._direct_body(bt, B_, S_)
        return self._replay_graph(key, body)

    @staticmethod
    def _replay_key(replay, B: int, S: int):
        """Graph-cache key of a replay source. A token unique for the object's lifetime, never ``id()``: a later pool
        allocated at a freed pool's address must not find (and replay) a graph wired to the freed storage."""
        tok = replay.__dict__.get('_dca_graph_token')
        if tok is None:
            tok = replay.__dict__['_dca_graph_token'] = next(_GRAPH_TOKENS)
        return ('replay', tok, B, S)

    def release_graphs(self, replay) -> int:
        """Drop every captured step (and its private memory pool + static index buffer) bound to ``replay`` — call
        before its storage is reallocated or freed. Returns the number of graphs released."""
        tok = replay.__dict__.get('_dca_graph_token')
        if tok is None:
            return 0
        graphs = self.__dict__.get('_graphs', {})
        dead = [k for k in graphs if k[0] == 'replay' and k[1] == tok]
        for k in dead:
            g = graphs.pop(k)[0]
            if self.graph is g or (isinstance(g, tuple) and self.graph in g):
                self.graph = None
            self._static_idx.pop(k, None)
        return len(dead)

    def train_step_replay(self, replay, B: int, recent: Optional[int] = None) -> Dict[str, torch.Tensor]:
        """One DP optimizer step on a minibatch sampled from an on-device replay (``learner.replay.HbmReplay``).
        On the direct fused path the gather itself is part of the captured graph (only the sampled indices are
        copied in)."""
        if self.direct() and self._graph_ready() and getattr(replay, 'host_sampling', False):
            key = self._replay_key(replay, B, replay.S)
            if key in self.__dict__.get('_graphs', {}):
                # captured step: the sampled positions go straight into the graph's own index buffer (one copy)
                replay.sample_into(self._static_idx[key], recent)
                return self._step_replay_key(replay, key, None)
        return self.train_step_indices(replay, replay.sample_indices(B, recent))

    def train_step_indices(self, replay, idx: torch.Tensor) -> Dict[str, torch.Tensor]:
        """One DP optimizer step on the pool sequences ``idx`` (device int64) of ``replay`` — any object with
        ``data`` (field → (capacity, S, …) device tensors at fixed addresses), ``S`` and ``gather(idx)``: the HBM
        replay, or the optimizer's per-iteration pool (epoch permutations over the iteration's sequences)."""
        if not self.direct():
            return self.train_step(replay.gather(idx))
        if self._graph_ready():
            return self._step_replay_key(replay, self._replay_key(replay, idx.numel(), replay.S), idx)
        return self._finish(self._direct_body(self.gather_time_major(replay, idx, replay.S), idx.numel(), replay.S))

    def _step_replay_key(self, replay, key, idx: Optional[torch.Tensor]) -> Dict[str, torch.Tensor]:
        """Captured replay step of graph ``key``; every key owns its static index buffer (``idx`` None: already
        written into it)."""
        B, S = key[2], key[3]
        if key not in self.__dict__.get('_graphs', {}):
            self._static_idx[key] = idx.clone()
        elif idx is not None:
            self._static_idx[key].copy_(idx)
        sidx = self._static_idx[key]
        if self._split_mode():
            vec = self._replay_split(key, lambda hook: self._direct_body(
                self.gather_time_major(replay, sidx, S), B, S, hook=hook))
        else:
            vec = self._replay_graph(key, lambda: self._direct_body(self.gather_time_major(replay, sidx, S), B, S))
        return self._finish(vec)

    def _sync_and_step(self):
        """DP reduction + optimizer step. With the fused Adam on a multi-rank job the has-grad average is taken
        inside the optimizer kernels (no separate pass over the gradient buffer after the all-reduce). The fused
        model's persistent-kernel error flag rides in the count-carrying bucket: if the recurrence failed on ANY
        rank, every rank's Adam skips this step on the device (FusedPolicy.check_error raises at the iteration
        boundary) — the reference raises before optimizer.step() (optimizer.py:674-676)."""
        if self.backend == 'fused':
            self.dp.err_flag.copy_(self.model.err)
        fold = self.dp.enabled and self.opt.use_kernels
        self.dp.sync(scale=not fold)
        if self.backend == 'fused' and self.dp.enabled:
            # the reduced flag is non-zero on EVERY rank when any rank's recurrence failed: keep it sticky so that
            # all ranks raise together at the iteration boundary (check_error), not only the failing one
            sticky = getattr(self, '_err_any', None)
            if sticky is None:
                sticky = self._err_any = torch.zeros_like(self.dp.err_flag)
            torch.maximum(sticky, self.dp.err_flag, out=sticky)
        return self.opt.step(self.dp.counts, divide=fold, skip=self.dp.err_flag)

    def check_error(self):
        """Raise (on every DP rank alike) if a persistent kernel failed on any rank since the last call; host sync,
        call at iteration boundaries."""
        self.opt.check_nonfinite()
        if self.backend != 'fused':
            return
        sticky = getattr(self, '_err_any', None)
        if sticky is not None and float(sticky.item()) != 0.0:
            own = int(self.model.err.item())
            sticky.zero_()
            raise RuntimeError(f'persistent kernel error on a data-parallel rank (own code {own}): the step was '
                               'skipped by every rank\'s Adam')
        self.model.check_error()

    def error_flags(self) -> List[torch.Tensor]:
        """The device flags :meth:`check_error` reads (non-finite step, sticky DP error, recurrence error), for a
        caller that snapshots them asynchronously with its other per-iteration values: when the snapshot shows one
        non-zero it calls :meth:`check_error`, whose host syncs then only happen on the failure path."""
        flags = [self.opt.nonfinite]
        if self.backend == 'fused':
            sticky = getattr(self, '_err_any', None)
            if sticky is not None:
                flags.append(sticky)
            flags.append(self.model.err)
        return flags

    def _finish(self, vec):
        metrics = self._metrics_from_vec(vec.clone())
        # a copy: the optimizer's norm is ONE persistent tensor rewritten by every step, and with deferred metrics the
        # iteration's list is read only after the next iteration's steps were queued
        metrics['grad_norm'] = self._sync_and_step().clone()
        self.n_steps += 1
        return metrics

    def train_step(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """One synchronous DP optimizer step. Returns device-resident metric tensors (no host sync)."""
        if self.direct():
            return self._finish(self._step_direct_batch(batch))
        metrics = self._fwd_bwd(batch)
        metrics['grad_norm'] = self._sync_and_step().clone()
        self.n_steps += 1
        return metrics

    # ------------------------------------------------------------------------------------------------
    @torch.no_grad()
    def evaluate_sequences(self, data: Dict[str, torch.Tensor], n: int, chunk: int = 32):
        """Log-prob of the sampled actions and value of every step of sequences ``0..n-1`` of ``data`` (batch-major
        ``(≥n, S, …)`` fields ``units``, ``env``, ``actions``, ``masks`` (+ ``h0``/``c0``, ``reset``)) at the
        CURRENT weights, in stream order: the learner-side ``policy_old`` of the reference (optimizer.py:279, 474) —
        the PPO ratio's denominator and the GAE / V-trace values of the iteration's experience. Returns (logp (n, S),
        value (n, S)) f32 on the learner's device. The fused path runs the step's forward kernels (fp32-exact: IEEE
        fp32, ``chunk`` ≤ 32 sequences per launch — the exact recurrence's 4 rows per XCD chain); the torch path the
        eager module."""
        S = data['units'].shape[1]
        if self.direct():
            from .. import ops
            C = ops.require()
            fields = ('units', 'env', 'actions', 'masks') + (('reset',) if 'reset' in data else ())
            seq = [k for k in ('h0', 'c0') if k in data]
            lps, vals = [], []
            for i0 in range(0, n, chunk):
                i1 = min(n, i0 + chunk)
                idx = torch.arange(i0, i1, device=self.device, dtype=torch.int64)
                outs = C.replay_gather([data[k] for k in fields] + [data[k] for k in seq], len(fields), idx)
                bt = dict(zip(list(fields) + seq, outs))
                lp, v = self.model.forward_logp_value(bt, i1 - i0, S)
                lps.append(lp.view(S, i1 - i0).t())
                vals.append(v.view(S, i1 - i0).t())
            return torch.cat(lps, 0).contiguous(), torch.cat(vals, 0).contiguous()
        from .losses import sampled_logp
        hidden = None
        if self.policy.is_recurrent and 'h0' in data:
            hidden = (data['h0'][:n].unsqueeze(0).contiguous(), data['c0'][:n].unsqueeze(0).contiguous())
        with self._autocast():
            logits, values, _ = self.model.forward_packed(data['env'][:n], data['units'][:n], hidden,
                                                          reset=data['reset'][:n] if 'reset' in data else None)
        logits = {k: v.float() for k, v in logits.items()}
        lp = sampled_logp(logits, split_heads(data['actions'][:n], self.counts), split_heads(data['masks'][:n],
                                                                                             self.counts),
                          stable=not self.policy.config.compat_bugs)
        return lp.float(), values.float().reshape(n, S)

    def state_dict(self):
        return {'optimizer': self.opt.state_dict(), 'n_steps': self.n_steps}

    def broadcast_state(self, src: int = 0):
        """Make every rank's optimizer state (Adam moments, per-parameter step counts) equal to rank ``src``'s."""
        import torch.distributed as dist
        for t in (self.opt.exp_avg, self.opt.exp_avg_sq, self.opt.steps):
            dist.broadcast(t, src)
        n = torch.tensor([self.n_steps], dtype=torch.int64, device=self.opt.steps.device)
        dist.broadcast(n, src)
        self.n_steps = int(n.item())

    def load_state_dict(self, d):
        self.opt.load_state_dict(d['optimizer'])
        self.n_steps = d.get('n_steps', 0)

    def after_load_weights(self):
        """Call after ``policy.load_state_dict`` so the flat buffers see the new weights."""
        self.flat.rebind()
        if self.backend == 'fused':
            self.model.refresh()
