"""Learner engine: one optimizer step (forward → loss → backward → DP all-reduce → clip + Adam).

This is the inner hot loop of the reference's ``DotaOptimizer.train`` (optimizer.py:565-688), re-organised around
flat parameter/gradient buffers so that the data-parallel reduction is a few bucketed RCCL collectives and the
optimizer is one fused HIP kernel pair.

Backends for the model math:

* ``'fused'`` (default on GPU): :class:`~dotaclient_amd.models.fused.FusedPolicy` — hand-written gfx950 HIP kernels
  for the entity encoder, LSTM recurrence and heads+loss; plain GEMMs through hipBLASLt.
* ``'torch'``: the eager reference model (``models.policy.Policy``) under bf16 autocast on GPU, fp32 on CPU.

Batches are dicts of device tensors (see :func:`dotaclient_amd.learner.synthetic.make_batch` for the schema):
``env (B,S,3) f32``, ``units (B,S,U,10) f32``, ``actions``/``masks (B,S,A) u8`` (flat ``enum|x|y|target_unit``),
``adv``/``ret``/``logp_old``/``norm_ret (B,S) f32`` and for recurrent policies ``h0``/``c0 (B,H) f32``.
"""
from __future__ import annotations

import contextlib
from dataclasses import dataclass
from typing import Dict, Optional

import torch

from ..models.policy import Policy
from ..parallel.dp import DataParallel, FlatParams
from .losses import ppo_loss, split_heads, vpg_loss
from .optim import FlatAdam


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


class Learner:
    def __init__(self, policy: Policy, loss_cfg: LossConfig, device='cpu', backend: str = 'auto',
                 bucket_cap_mb: float = 8.0, overlap: bool = True, dp: bool = True):
        self.device = torch.device(device)
        self.cfg = loss_cfg
        self.policy = policy.to(self.device)
        if backend == 'auto':
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
            self.model = FusedPolicy(self.policy, loss_cfg)
        self.counts = self.policy.layout.action_counts()
        self.n_steps = 0
        self.graph = None                 # captured forward+backward (see enable_graph)
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
        if self.backend == 'torch' and self.device.type == 'cuda':   # 'torch-fp32' = fp32 oracle
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
            logits, values, _ = self.model.forward_packed(batch['env'], batch['units'], self.hidden_from_batch(batch))
        logits = {k: v.float() for k, v in logits.items()}
        values = values.float()
        actions = split_heads(batch['actions'], self.counts)
        masks = split_heads(batch['masks'], self.counts)
        if cfg.algo == 'ppo':
            return ppo_loss(logits, values, actions, masks, batch['adv'], batch['ret'], batch['logp_old'],
                            cfg.clip_eps, cfg.entropy_coef, cfg.vf_coef, stable=stable)
        return vpg_loss(logits, values, actions, masks, batch['norm_ret'], batch['ret'], cfg.entropy_coef,
                        cfg.vf_coef, compat_value_bug=cfg.compat_value_bug, stable=stable)

    def _fwd_bwd(self, batch):
        self.dp.zero_grad()
        loss, metrics = self.loss(batch)
        loss.backward()
        if self.backend == 'fused' and getattr(self.model, 'direct_used', False):
            # the fused Functions accumulate straight into the flat gradient buffer (no per-parameter autograd
            # hooks fire); tell the DP layer which parameters received a gradient
            self.dp.has_grad.copy_(self.model.grad_mask)
        return {k: v.detach() for k, v in metrics.items()}

    def _graphed_fwd_bwd(self, batch):
        if self.graph is None:
            self._static_in = {k: v.clone() for k, v in batch.items()}
            # the capture stream must outlive the graph: hipBLASLt's per-stream workspace that the captured GEMM
            # nodes point at belongs to it
            s = self._graph_stream = torch.cuda.Stream(device=self.device)
            s.wait_stream(torch.cuda.current_stream(self.device))
            with torch.cuda.stream(s):          # one more eager run on the capture stream (allocator warm-up)
                self._fwd_bwd(self._static_in)
            torch.cuda.current_stream(self.device).wait_stream(s)
            self.graph = torch.cuda.CUDAGraph()
            with torch.cuda.graph(self.graph, stream=s):
                self._static_out = self._fwd_bwd(self._static_in)
            self._graph_mask_used = getattr(self.model, 'direct_used', False)
        for k, v in batch.items():
            self._static_in[k].copy_(v, non_blocking=True)
        self.dp.zero_grad()
        self.graph.replay()
        if self._graph_mask_used:
            self.dp.has_grad.copy_(self.model.grad_mask)
        return {k: v.clone() for k, v in self._static_out.items()}

    def train_step(self, batch: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """One synchronous DP optimizer step. Returns device-resident metric tensors (no host sync)."""
        if self._graph_warmup and self.n_steps >= self._graph_warmup:
            metrics = self._graphed_fwd_bwd(batch)
        else:
            metrics = self._fwd_bwd(batch)
        self.dp.sync()
        metrics['grad_norm'] = self.opt.step(self.dp.counts)
        self.n_steps += 1
        return metrics

    # ------------------------------------------------------------------------------------------------
    def state_dict(self):
        return {'optimizer': self.opt.state_dict(), 'n_steps': self.n_steps}

    def load_state_dict(self, d):
        self.opt.load_state_dict(d['optimizer'])
        self.n_steps = d.get('n_steps', 0)

    def after_load_weights(self):
        """Call after ``policy.load_state_dict`` so the flat buffers see the new weights."""
        self.flat.rebind()
        if self.backend == 'fused':
            self.model.refresh()
