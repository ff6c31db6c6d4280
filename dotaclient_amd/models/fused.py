"""MI355X execution of :class:`~dotaclient_amd.models.policy.Policy` on hand-written gfx950 kernels.

Same parameters (it wraps the reference module and reads its ``nn.Parameter``s, which live in the learner's flat
buffer), different execution: the loss and every gradient of a minibatch come from ONE pass of explicit kernels in a
fixed order, no autograd graph (models/pipelined.py ``fused_step_tm``; ``train_direct`` is the learner's
graph-captured hot path, :class:`~dotaclient_amd.models.pipelined.PipelinedPolicyLoss` the autograd face for callers
that backprop themselves):

=================  ======================================================================================
stage              kernels (ops/csrc)
=================  ======================================================================================
entity encoder     ``encoder.hip``: unit MLP + per-type GEMM + max-pool/argmax; backward ∂W_τ / ∂W1 / ∂b1
                   (5v5: ``attn_block.hip`` LayerNorm + self-attention + out-projection, fwd and bwd)
pre-RNN + input    ``dx_chain.hip`` forward chain: relu(x896·W_preᵀ + b) then ·W_ihᵀ (or the reference's linear
projection         fake_rnn layer, policy.py:67-68) in one kernel; backward: the ∂X chain
recurrence         ``lstm_team.hip``: XCD-team persistent LSTM forward / backward
heads + loss       ``dx_chain.hip`` heads GEMM + ``heads_loss.hip`` (pointer logits, 4 masked log-softmaxes,
                   PPO/VPG, entropy, value, ∂L/∂every head input)
weight gradients   ``gemm_tn.hip`` split-K TN GEMM over the B·S rows; ``glue.hip`` small encoder gradients
optimizer          ``adam.hip`` fused global-norm clip + Adam
=================  ======================================================================================

Precision (``FusedPolicy(precision=...)``):

* ``'fp32-exact'`` (the learner default, the reference's fp32 training, optimizer.py:281, policy.py:52-78): every
  product an IEEE fp32 FMA (``v_mfma_f32_16x16x4_f32`` / fp32 VALU), fp32 activations, gradients and accumulation.
* ``'fp32'``: fp32 activations; the hand-written MFMA kernels split each fp32 operand into a hi and a lo bf16 and
  sum hi·hi + lo·hi + hi·lo (≈2⁻¹⁶ relative per product, "bf16x3").
* ``'bf16'`` has no kernel path (:meth:`use_pipeline` is False): the learner runs it on the torch backend under bf16
  autocast (learner/engine.py). The fused step has no vendor-GEMM branch.

The 5v5 entity-attention block runs on the fused block kernels (ops/csrc/attn_block.hip): bf16x3 products at
``'fp32'``, their IEEE-fp32 twins (``v_mfma_f32_16x16x4_f32``) at ``'fp32-exact'``. Configurations the kernels do not
cover (unit / env widths other than 128, bf16) run on the torch backend (learner/engine.py).
"""
from __future__ import annotations

from typing import Dict, List

import torch

from .policy import Policy

LDZ = 160


class FusedPolicy:
    def __init__(self, policy: Policy, loss_cfg=None, precision: str = 'fp32'):
        from .. import ops
        if precision not in ('fp32', 'bf16', 'fp32-exact'):
            raise ValueError(f'precision must be fp32, fp32-exact or bf16, got {precision!r}')
        self.C = ops.require()
        self.policy = policy
        self.cfg = policy.config
        self.loss_cfg = loss_cfg
        self.precision = precision
        self.fp32 = precision in ('fp32', 'fp32-exact')
        # 'fp32-exact': IEEE fp32 products everywhere (no bf16x3 split): the exact-f32 MFMA / VALU twins of every
        # kernel of the step (models/pipelined.py)
        self.exact = precision == 'fp32-exact'
        dev = next(policy.parameters()).device
        self.err = torch.zeros(1, dtype=torch.int32, device=dev)
        self.param_names: List[str] = [n for n, _ in policy.named_parameters()]
        self.params = [p for _, p in policy.named_parameters()]
        self.fully_fused = not self.cfg.entity_attention and self.cfg.unit_dim == 128 and self.cfg.env_dim == 128
        # the 5v5 entity-attention encoder has fused kernels on the pipelined (time-major) step only
        self.attention_fused = (self.cfg.entity_attention and self.cfg.unit_dim == 128 and self.cfg.env_dim == 128
                                and self.cfg.attention_heads == 4 and self.cfg.layout.max_units == 64)

    def wcast(self, t: torch.Tensor) -> torch.Tensor:
        """A detached working copy of a weight in this learner's GEMM operand dtype (fp32 or bf16)."""
        t = t.detach()
        return t if self.fp32 else t.to(torch.bfloat16)

    def apply_direct_grads(self, grads, g, written=(), set_mask: bool = True):
        """Accumulate precomputed gradients straight into the parameters' ``.grad`` (views of the learner's flat
        buffer) with two multi-tensor kernels, instead of returning 30 tensors to autograd (which launches one
        accumulation copy per parameter, ≈1 ms of host-bound launches per step). ``g`` = upstream gradient
        (None = 1). Records which parameters received a gradient in ``grad_mask`` for the DP has-grad counts."""
        gl, views, mask = [], [], []
        for name, p, t in zip(self.param_names, self.params, grads):
            mask.append(t is not None or name in written)
            if t is None:
                continue
            if p.grad is None:
                p.grad = torch.zeros_like(p)
            gl.append((t if t.dtype == torch.float32 else t.float()).contiguous())
            views.append(p.grad)
        # one launch with the tensor table in the kernel arguments — torch's foreach kernels stage their tensor
        # lists through a host buffer, which a replayed hipGraph would read stale
        self.C.multi_axpy(views, gl, None if g is None else g.reshape(1).float().contiguous())
        if set_mask and getattr(self, '_mask_list', None) != mask:
            self._mask_list = mask
            self.grad_mask = torch.tensor(mask, dtype=torch.float32, device=self.err.device)
        self.direct_used = True

    # ---- direct (autograd-free) learner step support ---------------------------------------------
    def attach_flat(self, flat: torch.Tensor):
        """The learner's flat fp32 parameter buffer (every parameter is a view of it): the per-step weight images
        are gathered from it by one kernel (models/pipelined.py:WeightImages)."""
        self.flat_buffer = flat
        self._wimg = None

    def weight_images(self):
        from .pipelined import WeightImages
        with_value = self.loss_cfg is None or self.loss_cfg.vf_coef > 0
        key = (with_value, self.flat_buffer.data_ptr() if getattr(self, 'flat_buffer', None) is not None else None,
               tuple(p.data_ptr() for p in self.params))
        if getattr(self, '_wimg', None) is None or self._wimg_key != key:
            if getattr(self, 'flat_buffer', None) is None:
                raise RuntimeError('FusedPolicy.attach_flat(flat) must be called before the fused LSTM step')
            self._wimg = WeightImages(self, self.flat_buffer, with_value)
            self._wimg_key = key
        return self._wimg

    def scratch(self, name, shape, dtype, device):
        d = self.__dict__.setdefault('_scratch', {})
        t = d.get(name)
        if t is None or tuple(t.shape) != tuple(shape) or t.dtype != dtype or t.device != torch.device(device):
            t = d[name] = torch.zeros(shape, dtype=dtype, device=device)
        return t

    def loss_prep_ws(self, device):
        return self.scratch('loss_prep_ws', (int(self.C.loss_prep_ws_elems()),), torch.int32, device)

    def train_direct(self, batch_tm, B: int, S: int, cfg=None) -> torch.Tensor:
        """Autograd-free step over time-major rows (see models/pipelined.py:train_direct); returns the metrics
        vector. Only for :meth:`use_pipeline` configurations."""
        from .pipelined import train_direct
        if cfg is not None:
            self.loss_cfg = cfg
        self.refresh()
        self.direct_used = False
        return train_direct(self, batch_tm, B, S)

    def forward_logp_value(self, batch_tm, B: int, S: int):
        """(logp, value) per time-major row at the current weights: the forward half of the step, no backward
        (models/pipelined.py :func:`forward_logp_value`)."""
        from .pipelined import forward_logp_value
        self.refresh()
        H = self.cfg.hidden
        dev = batch_tm['units'].device
        h0, c0 = batch_tm.get('h0'), batch_tm.get('c0')
        if h0 is None:
            h0 = c0 = torch.zeros(B, H, device=dev)
        return forward_logp_value(self, batch_tm['units'], batch_tm['env'], batch_tm['actions'], batch_tm['masks'],
                                  h0, c0, B, S, reset_t=batch_tm.get('reset'))

    def side_stream(self):
        if getattr(self, '_side', None) is None:
            # (default priority: either stream at high priority measured 0.7 ms per step slower under graph replay,
            # profiles/r4_stream_priority_ab.txt)
            self._side = torch.cuda.Stream(device=self.err.device)
        return self._side

    def use_pipeline(self) -> bool:
        """Whether the kernels cover this configuration (models/pipelined.py): fp32 / fp32-exact, the LSTM policies or
        the reference's linear fake_rnn layer with its VPG value quirk (the compat preset)."""
        if not (self.fully_fused or self.attention_fused) or not self.fp32:
            return False
        if self.cfg.rnn == 'lstm':
            return self.cfg.hidden % 128 == 0
        return self.cfg.hidden % 128 == 0 and self.cfg.pre_rnn_dim == 256

    # Data-parallel split of the direct step (learner/engine.py): the learner sets ``split_hook`` to a callable
    # that the step calls once, at the point where every gradient of :meth:`early_param_names` is final.
    split_hook = None
    early_applied = frozenset()

    def early_param_names(self) -> frozenset:
        """Parameters whose gradients are final before the encoder backward (pre-RNN, recurrence, heads): a
        contiguous suffix of the registration order, so their flat-buffer range is one all-reduce bucket."""
        pre = ('affine_pre_rnn.', 'rnn.', 'fake_rnn.', 'affine_head_enum.', 'affine_move_', 'affine_unit_attention.',
               'affine_value.')
        return frozenset(n for n in self.param_names if n.startswith(pre))

    @property
    def chunks(self) -> int:
        import os
        # 1 = no time-chunk overlap: measured on MI355X, work running concurrently on the other XCDs slows the
        # L2-bound team recurrence by more than it saves (profiles/r5_half_team.md: 5.45 ms at one chunk, 6.2-6.9 ms
        # chunked)
        return int(os.environ.get('DCA_PIPELINE_CHUNKS', '1'))

    def gate_perm(self, H, device):
        key = (H, str(device))
        if getattr(self, '_perm_key', None) != key:
            from ..ops.lstm import gate_perm
            self._perm, self._perm_key = gate_perm(H, device), key
            self._inv = torch.empty_like(self._perm)
            self._inv[self._perm] = torch.arange(self._perm.numel(), device=self._perm.device)
        return self._perm

    def gate_perm_i32(self, H, device):
        """:meth:`gate_perm` as int32 (the TN GEMM's output row map: unit-major result row m → gate-major row)."""
        key = (H, str(device))
        if getattr(self, '_perm32_key', None) != key:
            self._perm32, self._perm32_key = self.gate_perm(H, device).to(torch.int32).contiguous(), key
        return self._perm32

    def gate_inv(self, H, device):
        """Inverse of :meth:`gate_perm` (unit-major gate rows → PyTorch gate-major rows), cached."""
        self.gate_perm(H, device)
        return self._inv

    def type_segments(self, device):
        """(U, 6) 0/1 matrix mapping unit slots to their unit type (sums pointer gradients per type), cached."""
        key = str(device)
        if getattr(self, '_seg_key', None) != key:
            counts = list(self.cfg.layout.counts)
            seg = torch.zeros(sum(counts), 6, device=device)
            off = 0
            for t, cnt in enumerate(counts):
                seg[off:off + cnt, t] = 1.0
                off += cnt
            self._seg, self._seg_key = seg, key
        return self._seg

    def type_offset_list(self):
        import itertools
        return [0] + list(itertools.accumulate(self.cfg.layout.counts))

    def type_offsets(self, device):
        """(7,) int32 device tensor: first unit slot of each unit type (+ total), cached."""
        key = str(device)
        if getattr(self, '_toff_key', None) != key:
            import itertools
            offs = [0] + list(itertools.accumulate(self.cfg.layout.counts))
            self._toff, self._toff_key = torch.tensor(offs, dtype=torch.int32, device=device), key
        return self._toff

    def unit_types(self, device):
        """(U,) uint8 device tensor: unit slot → unit type index, cached."""
        key = str(device)
        if getattr(self, '_utype_key', None) != key:
            ty = sum([[t] * c for t, c in enumerate(self.cfg.layout.counts)], [])
            self._utype, self._utype_key = torch.tensor(ty, dtype=torch.uint8, device=device), key
        return self._utype

    def refresh(self):
        self.params = [p for _, p in self.policy.named_parameters()]

    # ------------------------------------------------------------------------------------------------
    def head_cat(self, P, differentiable: bool = False):
        """Concatenate the five head Linear layers into one (LDZ, H) matrix: [q | enum | x | y | value | pad].
        ``differentiable`` keeps the autograd link to the parameters (per-stage path); the fully fused Function
        computes the head gradients itself and uses detached copies."""
        H = self.cfg.hidden
        dev = P['affine_value.weight'].device
        d = (lambda t: t) if differentiable else (lambda t: t.detach())
        with_value = self.loss_cfg is None or self.loss_cfg.vf_coef > 0
        wv = d(P['affine_value.weight']) if with_value else torch.zeros(1, H, device=dev)
        bv = d(P['affine_value.bias']) if with_value else torch.zeros(1, device=dev)
        pad = LDZ - 150
        w = torch.cat([d(P['affine_unit_attention.weight']), d(P['affine_head_enum.weight']),
                       d(P['affine_move_x.weight']), d(P['affine_move_y.weight']), wv,
                       torch.zeros(pad, H, device=dev)], 0)
        b = torch.cat([d(P['affine_unit_attention.bias']), d(P['affine_head_enum.bias']),
                       d(P['affine_move_x.bias']), d(P['affine_move_y.bias']), bv,
                       torch.zeros(pad, device=dev)], 0)
        return w, b

    def split_head_grads(self, dW, db, grads):
        spans = [('affine_unit_attention', 0, 128), ('affine_head_enum', 128, 131), ('affine_move_x', 131, 140),
                 ('affine_move_y', 140, 149)]
        if self.loss_cfg is None or self.loss_cfg.vf_coef > 0:
            spans.append(('affine_value', 149, 150))
        for name, lo, hi in spans:
            grads[f'{name}.weight'] = dW[lo:hi]
            grads[f'{name}.bias'] = db[lo:hi]

    # ------------------------------------------------------------------------------------------------
    def loss(self, batch: Dict[str, torch.Tensor], cfg):
        """Loss + metrics of a batch-major minibatch through :class:`PipelinedPolicyLoss` (its backward scales the
        gradients the forward pass already computed)."""
        from ..ops.heads import assemble_loss, batch_norms
        from .pipelined import PipelinedPolicyLoss
        if not self.use_pipeline():
            raise ValueError(f'FusedPolicy: no kernel path for {self.cfg} at {self.precision} (use the torch backend)')
        self.loss_cfg = cfg
        self.direct_used = False
        B, S = batch['env'].shape[:2]
        N = B * S
        dev = batch['env'].device
        actions = batch['actions'].reshape(N, -1).contiguous()
        masks = batch['masks'].reshape(N, -1).contiguous()
        ret = batch['ret'].reshape(N).float().contiguous()
        algo = 0 if cfg.algo == 'ppo' else 1
        norms = batch_norms(actions, ret, cfg.compat_value_bug and algo == 1, S)
        zeros = torch.zeros(N, device=dev)
        adv = batch['adv'].reshape(N).contiguous() if 'adv' in batch else zeros
        lpo = batch['logp_old'].reshape(N).contiguous() if 'logp_old' in batch else zeros
        nret = batch['norm_ret'].reshape(N).contiguous() if 'norm_ret' in batch else zeros
        rst = batch.get('reset')
        H = self.cfg.hidden
        h0 = batch.get('h0')
        c0 = batch.get('c0')
        if h0 is None:
            h0 = torch.zeros(B, H, device=dev)
            c0 = torch.zeros(B, H, device=dev)
        self.refresh()
        vt = batch.get('vt') if getattr(cfg, 'vtrace', False) else None
        part, logp = PipelinedPolicyLoss.apply(self, batch['units'].contiguous(), batch['env'].contiguous(), actions,
                                               masks, adv, ret, lpo, nret, norms, h0.contiguous(), c0.contiguous(),
                                               rst, vt, *self.params)
        loss, metrics = assemble_loss(part, norms, cfg, ret, N, S)
        if getattr(self, 'vtrace_stats', None) is not None:
            st = self.vtrace_stats.sum(0)
            for i, k in enumerate(('offpolicy/rho_mean', 'offpolicy/rho_truncated', 'offpolicy/behaviour_kl')):
                metrics[k] = st[i] / st[3].clamp_min(1.0)
        return loss, metrics

    def check_error(self):
        """Raise if a persistent kernel timed out (host sync — call at iteration boundaries, not per step)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f'persistent kernel error code {e} (recurrence hand-off timed out)')
