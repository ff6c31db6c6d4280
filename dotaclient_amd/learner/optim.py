"""Fused global-norm clip + Adam over the flat parameter buffer.

Replaces the reference's ``clip_grad_norm_(0.5)`` + ``torch.optim.Adam(lr)`` (optimizer.py:281, 680-681) with one
optimizer over :class:`~dotaclient_amd.parallel.dp.FlatParams`:

* global L2 norm of the (already DP-averaged) flat gradient, clip coefficient ``min(1, max_norm / (norm + 1e-6))``
  (torch's ``clip_grad_norm_`` formula);
* Adam with torch's default betas/eps and *per-parameter* step counts;
* parameters whose DP has-grad count is 0 are skipped entirely (no moment decay, no step increment) — the
  sparse-parameter semantics of the reference's DP wrapper (distributed.py:40-42).

On GPU this runs as two HIP kernels (``ops.adam_norm`` partial sums + ``ops.adam_update`` fused update, see
ops/csrc/adam.hip); :meth:`FlatAdam.step_reference` is the torch implementation used on CPU and as the oracle.
"""
from __future__ import annotations

from typing import Optional

import torch

from ..parallel.dp import FlatParams


class FlatAdam:
    def __init__(self, flat: FlatParams, lr: float = 1e-4, betas=(0.9, 0.999), eps: float = 1e-8,
                 max_grad_norm: Optional[float] = 0.5, use_kernels: Optional[bool] = None):
        self.flat = flat
        self.lr, self.betas, self.eps = lr, betas, eps
        self.max_grad_norm = max_grad_norm
        dev = flat.flat.device
        self.exp_avg = torch.zeros_like(flat.flat)
        self.exp_avg_sq = torch.zeros_like(flat.flat)
        self.steps = torch.zeros(len(flat.params), device=dev, dtype=torch.float32)
        self.last_grad_norm = torch.zeros((), device=dev, dtype=torch.float32)
        # sticky device flag: a step was dropped because its gradient norm was not finite (check_nonfinite raises)
        self.nonfinite = torch.zeros(1, device=dev, dtype=torch.float32)
        if use_kernels is None:
            use_kernels = dev.type == 'cuda'
        self.use_kernels = use_kernels
        if use_kernels:
            from .. import ops
            self._ops = ops.require()

    # ------------------------------------------------------------------------------------------------
    def step(self, counts: Optional[torch.Tensor] = None, divide: bool = False,
             skip: Optional[torch.Tensor] = None):
        """``divide``: ``flat.grad`` holds the DP all-reduce SUMS (DataParallel.sync(scale=False)); the has-grad
        average grad / counts[param] is taken inside the optimizer instead of by a separate pass. ``skip``: 1-element
        f32 device flag; nonzero → nothing is applied this step (decided on the device, no host sync)."""
        if counts is None:
            counts = torch.ones(len(self.flat.params), device=self.flat.flat.device)
        if self.use_kernels:
            return self._step_kernels(counts, divide, skip)
        return self.step_reference(counts, divide, skip)

    def _step_kernels(self, counts, divide=False, skip=None):
        b1, b2 = self.betas
        max_norm = self.max_grad_norm if self.max_grad_norm is not None else -1.0
        self._ops.adam_step(self.flat.flat, self.flat.grad, self.exp_avg, self.exp_avg_sq, self.flat.segment_ids,
                            counts, self.steps, self.last_grad_norm, float(self.lr), float(b1), float(b2),
                            float(self.eps), float(max_norm), divide=bool(divide), header=int(self.flat.header),
                            skip=skip, nonfinite=self.nonfinite)
        return self.last_grad_norm

    def check_nonfinite(self):
        """Raise if a step since the last call was dropped for a non-finite gradient (host sync: call at iteration
        boundaries). The reference raises on a NaN loss before optimizer.step() (optimizer.py:674-676); a finite loss
        with Inf / NaN gradients is caught here instead of training on with silently skipped steps."""
        if float(self.nonfinite.item()) != 0.0:
            self.nonfinite.zero_()
            raise FloatingPointError('non-finite gradient norm: the optimizer step was skipped')

    @torch.no_grad()
    def step_reference(self, counts, divide=False, skip=None):
        b1, b2 = self.betas
        g = torch.where(self.flat.segment_ids >= 0, self.flat.grad, torch.zeros_like(self.flat.grad))   # no header
        if divide:
            segc = self.flat.segment_ids.long().clamp_min(0)
            inv = torch.where(counts > 0, 1.0 / counts.clamp_min(1.0), torch.zeros_like(counts))
            g = g * torch.where(self.flat.segment_ids >= 0, inv[segc], torch.zeros_like(g))
        norm = torch.linalg.vector_norm(g)
        self.last_grad_norm.copy_(norm)
        if skip is not None and float(skip.reshape(-1)[0]) != 0.0:
            return norm
        if not bool(torch.isfinite(norm)):
            self.nonfinite.fill_(1.0)       # same as the kernels: nothing applied, step counters unchanged
            return norm
        if self.max_grad_norm is not None:
            coef = (self.max_grad_norm / (norm + 1e-6)).clamp(max=1.0)
            g = g * coef
        active_p = counts > 0
        self.steps += active_p.to(self.steps.dtype)
        seg = self.flat.segment_ids.long()
        valid = seg >= 0
        segc = seg.clamp_min(0)
        active = active_p[segc] & valid
        step = self.steps[segc]
        m = torch.where(active, b1 * self.exp_avg + (1 - b1) * g, self.exp_avg)
        v = torch.where(active, b2 * self.exp_avg_sq + (1 - b2) * g * g, self.exp_avg_sq)
        self.exp_avg.copy_(m)
        self.exp_avg_sq.copy_(v)
        bc1 = 1 - torch.pow(torch.full_like(step, b1), step)
        bc2 = 1 - torch.pow(torch.full_like(step, b2), step)
        denom = (v.sqrt() / bc2.clamp_min(1e-30).sqrt()) + self.eps
        upd = (self.lr / bc1.clamp_min(1e-30)) * m / denom
        self.flat.flat.sub_(torch.where(active, upd, torch.zeros_like(upd)))
        return norm

    # ------------------------------------------------------------------------------------------------
    def layout(self):
        """The flat buffer's layout (header length, per-parameter offsets and sizes): the moments are only meaningful
        against the layout they were written with."""
        return {'header': int(self.flat.header), 'offsets': [int(o) for o in self.flat.offsets],
                'numel': [int(n) for n in self.flat.numel]}

    def state_dict(self):
        return {'exp_avg': self.exp_avg.cpu(), 'exp_avg_sq': self.exp_avg_sq.cpu(), 'steps': self.steps.cpu(),
                'lr': self.lr, 'betas': self.betas, 'eps': self.eps, 'max_grad_norm': self.max_grad_norm,
                'layout': self.layout()}

    def load_state_dict(self, d, keep_hparams: bool = True):
        """Restore the moments and step counts. The hyperparameters this optimizer was built with (from the CLI)
        win over the checkpointed ones unless ``keep_hparams`` is False; a difference is logged. Moments saved
        under another flat layout are remapped parameter by parameter (same parameters, same sizes); a state without
        a recorded layout (written before layouts were versioned) is accepted only if its length matches the
        current buffer exactly, otherwise it is rejected with ValueError."""
        import logging
        log = logging.getLogger(__name__)
        cur = self.layout()
        saved = d.get('layout')
        if saved is None:
            if d['exp_avg'].numel() != self.exp_avg.numel():
                raise ValueError(f'optimizer state of {d["exp_avg"].numel()} elements has no recorded flat layout '
                                 f'and does not match this buffer ({self.exp_avg.numel()} elements): it was '
                                 'written by an older layout; resume the weights only (drop the trainer state)')
            self.exp_avg.copy_(d['exp_avg'])
            self.exp_avg_sq.copy_(d['exp_avg_sq'])
        elif saved == cur:
            self.exp_avg.copy_(d['exp_avg'])
            self.exp_avg_sq.copy_(d['exp_avg_sq'])
        else:
            if saved['numel'] != cur['numel']:
                raise ValueError('optimizer state was written for different parameters (sizes '
                                 f'{saved["numel"]} vs {cur["numel"]})')
            log.info('resume: remapping Adam moments from flat layout (header %d) to (header %d)', saved['header'],
                     cur['header'])
            for key in ('exp_avg', 'exp_avg_sq'):
                src, dst = d[key], getattr(self, key)
                for so, do, n in zip(saved['offsets'], cur['offsets'], cur['numel']):
                    dst[do:do + n].copy_(src[so:so + n])
        self.steps.copy_(d['steps'])
        hp = {'lr': d['lr'], 'betas': tuple(d['betas']), 'eps': d['eps'], 'max_grad_norm': d['max_grad_norm']}
        if not keep_hparams:
            self.lr, self.betas, self.eps, self.max_grad_norm = hp['lr'], hp['betas'], hp['eps'], hp['max_grad_norm']
            return
        mine = {'lr': self.lr, 'betas': tuple(self.betas), 'eps': self.eps, 'max_grad_norm': self.max_grad_norm}
        diff = {k: (hp[k], mine[k]) for k in mine if hp[k] != mine[k]}
        if diff:
            log.warning('resume: keeping the configured optimizer hyperparameters over the checkpointed ones '
                        '(checkpoint, configured): %s', diff)
