"""MI355X execution of :class:`~dotaclient_amd.models.policy.Policy` on hand-written gfx950 kernels.

Same parameters (it wraps the reference module and reads its ``nn.Parameter``s, which live in the learner's flat
buffer), different execution. The whole learner forward *and* backward is ONE ``autograd.Function`` with an explicit,
hand-ordered backward (no per-op autograd graph):

=================  ======================================================================================
stage              forward / backward
=================  ======================================================================================
entity encoder     ``_C.encoder_fwd``: unit MLP + per-type GEMM + max-pool/argmax (MFMA, one kernel) /
                   ``_C.encoder_bwd``: ∂W1 in-kernel, ∂emb/basic as K-blocked images → split-K MFMA GEMM for ∂W_τ
pre-RNN            bf16 GEMM (fp32 out) + ReLU / two GEMMs
LSTM               input-projection GEMM + ONE persistent ``_C.lstm_fwd`` launch /
                   ONE persistent ``_C.lstm_bwd`` launch + weight-gradient GEMMs over all B·S rows
heads + loss       one heads GEMM + ``_C.heads_loss`` (pointer logits, 4 masked log-softmaxes, PPO/VPG,
                   entropy, value, and ∂L/∂(every head input) in the same pass) / two GEMMs
=================  ======================================================================================

Precision (``FusedPolicy(precision=...)``):

* ``'fp32'`` (default; the reference trains in fp32, optimizer.py:281, policy.py:52-78): fp32 activations,
  gradients and accumulation end to end. The hand-written kernels run "bf16x3" — each fp32 MFMA operand split once
  into a hi and a lo bf16, products as hi·hi + lo·hi + hi·lo (≈2⁻¹⁶ relative per product) — and the plain GEMMs
  run on hipBLASLt's fast fp32 mode, the same accuracy class (``DCA_F32_GEMM=exact``: its exact-f32 path). The LSTM
  hidden state is exchanged and stored in fp32.
* ``'bf16'``: bf16 GEMM operands / saved activations, fp32 accumulation, recurrence state and optimizer.

The 5v5 entity-attention block runs on its bf16 kernels (ops/csrc/attn.hip) in the bf16 learner and on its fp32
(bf16x3 split-MFMA) attention core, fp32 LayerNorm / pool kernels and hipBLASLt fp32 GEMMs in the fp32 learner
(``models/pipelined.py:_fused_step_tm``); the rest of the 5v5 step is the same fused pipeline.
"""
from __future__ import annotations

from typing import Dict, List

import torch
import torch.nn.functional as F

from .policy import TYPE_SUFFIX, Policy

from ..ops.lstm import impl as lstm_impl  # noqa: E402
from ..ops.lstm import team_bwd, team_fwd  # noqa: E402

LDZ = 160


def _mm(a, b):
    """fp32-output GEMM: bf16 operands on hipBLASLt's bf16 path, fp32 operands on its exact-f32 path."""
    return a @ b if a.dtype == torch.float32 else torch.mm(a, b, out_dtype=torch.float32)


def _bf(t):
    return t.detach().to(torch.bfloat16)


def tn_splitk(a: torch.Tensor, b: torch.Tensor, chunk: int = 2048) -> torch.Tensor:
    """aᵀ·b for tall-skinny operands (K ≫ M, N: weight gradients reduced over B·S·units rows) as a batched GEMM over
    K-chunks + a sum. A plain GEMM of this shape gets only (M/64)·(N/128) workgroups and no split-K on hipBLASLt
    (measured 25 TF for 128×128×179200); chunking gives K/chunk× more parallelism."""
    K, M = a.shape
    N = b.shape[1]
    nc = K // chunk
    if nc < 2:
        return torch.mm(a.t(), b, out_dtype=torch.float32) if a.dtype == torch.bfloat16 else a.t() @ b
    main = nc * chunk
    if a.dtype == torch.bfloat16:
        part = torch.bmm(a[:main].view(nc, chunk, M).transpose(1, 2), b[:main].view(nc, chunk, N),
                         out_dtype=torch.float32)
    else:
        part = torch.bmm(a[:main].view(nc, chunk, M).transpose(1, 2), b[:main].view(nc, chunk, N))
    out = part.sum(0)
    if main < K:
        out += (torch.mm(a[main:].t(), b[main:], out_dtype=torch.float32) if a.dtype == torch.bfloat16
                else a[main:].t() @ b[main:])
    return out


class _PolicyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fp: 'FusedPolicy', units, env, actions, masks, adv, ret, logp_old, nret, norms, h0, c0, *params):
        C = fp.C
        cfg, lc = fp.cfg, fp.loss_cfg
        P = dict(zip(fp.param_names, params))
        _bf = fp.wcast                        # GEMM operand dtype of this learner: bf16, or fp32 (bf16x3 kernels)
        adt = torch.float32 if fp.fp32 else torch.bfloat16
        B, S, U, _ = units.shape
        N = B * S
        counts = list(cfg.layout.counts)
        units2 = units.reshape(N, U, 10).contiguous()
        env2 = env.reshape(N, 3).contiguous()
        wt16 = torch.stack([_bf(P[f'affine_unit_{s}.weight']) for s in TYPE_SUFFIX])
        bt = torch.stack([P[f'affine_unit_{s}.bias'].detach() for s in TYPE_SUFFIX])
        x896, emb, arg = C.encoder_fwd(units2, env2, P['affine_unit_basic_stats.weight'].detach(),
                                       P['affine_unit_basic_stats.bias'].detach(), wt16, bt,
                                       P['affine_env.weight'].detach(), P['affine_env.bias'].detach(), counts,
                                       bool(cfg.compat_bugs))
        if cfg.compat_bugs:   # reference policy.py:127: enemy-tower pool = enemy-nonhero pool
            x896[:, 768:896] = x896[:, 512:640]
            arg[:, 5] = arg[:, 3]
        wpre16 = _bf(P['affine_pre_rnn.weight'])
        x = torch.relu(_mm(x896, wpre16.t()) + P['affine_pre_rnn.bias'].detach())
        x16 = x.to(adt)
        if cfg.rnn == 'lstm':
            H = cfg.hidden
            wih16, whh16 = _bf(P['rnn.weight_ih_l0']), _bf(P['rnn.weight_hh_l0'])
            bias = P['rnn.bias_ih_l0'].detach() + P['rnn.bias_hh_l0'].detach()
            if lstm_impl() == 'team':
                # unit-major gate order: W_ih rows permuted so x·W_ihᵀ lands directly in the (B,S,H,4) layout
                perm = fp.gate_perm(H, wih16.device)
                wih16 = wih16[perm].contiguous()
                xp4 = (_mm(x16, wih16.t()) + bias[perm]).view(B, S, H, 4)
                hs16, _, cs, gates, _, _ = team_fwd(C, xp4, whh16, h0, c0, fp.err, False)
            else:
                assert not fp.fp32, 'the fp32 learner runs the team recurrence (DCA_LSTM_IMPL=team)'
                perm = None
                xp = (_mm(x16, wih16.t()) + bias).view(B, S, 4 * H)
                hs, cs, gates = [], [], []
                mb = C.lstm_max_batch(H)
                for s0 in range(0, B, mb):
                    s1 = min(B, s0 + mb)
                    o = C.lstm_fwd(xp[s0:s1], whh16, h0[s0:s1].contiguous(), c0[s0:s1].contiguous(), fp.err, False)
                    hs.append(o[0]); cs.append(o[2]); gates.append(o[3])
                cat = (lambda L: torch.cat(L) if len(L) > 1 else L[0])
                hs16, cs, gates = cat(hs), cat(cs), cat(gates)
            xh16 = hs16.view(N, H)
            ctx.perm = perm
            rnn_saved = (hs16, cs, gates, wih16, whh16)
        else:
            wf16 = _bf(P['fake_rnn.weight'])
            xh16 = (_mm(x16, wf16.t()) + P['fake_rnn.bias'].detach()).to(adt)
            rnn_saved = (wf16,)
        wcat, bcat = fp.head_cat(P)
        wcat16 = wcat.to(adt)
        z = _mm(xh16, wcat16.t()) + bcat
        dz, dtl, part, logp = C.heads_loss(z, emb.view(N, U, 128), actions, masks, adv, ret, logp_old, nret, norms,
                                           0 if lc.algo == 'ppo' else 1, bool(lc.compat_value_bug), S, B,
                                           float(lc.clip_eps), float(lc.entropy_coef), float(lc.vf_coef))
        ctx.fp = fp
        ctx.dims = (B, S, U, N)
        ctx.save_for_backward(units2, env2, x896, arg, x, x16, xh16, h0, c0, dz, dtl, z, wt16, wpre16, wcat16,
                              *rnn_saved)
        ctx.mark_non_differentiable(logp)
        return part.sum(0), logp

    @staticmethod
    def backward(ctx, gpart, _glogp):
        fp = ctx.fp
        C, cfg = fp.C, fp.cfg
        B, S, U, N = ctx.dims
        (units2, env2, x896, arg, x, x16, xh16, h0, c0, dz, dtl, z, wt16, wpre16, wcat16, *rnn_saved) = \
            ctx.saved_tensors
        P = {n: p for n, p in zip(fp.param_names, fp.params)}
        g = gpart[15]
        grads: Dict[str, torch.Tensor] = {}
        adt = torch.float32 if fp.fp32 else torch.bfloat16
        # ---- heads
        dZ = dz * g
        dZ16 = dZ.to(adt)
        dWcat = _mm(dZ16.t(), xh16)
        dbcat = dZ.sum(0)
        fp.split_head_grads(dWcat, dbcat, grads)
        dxh = _mm(dZ16, wcat16)
        # ---- recurrence
        if cfg.rnn == 'lstm':
            hs16, cs, gates, wih16, whh16 = rnn_saved
            H = cfg.hidden
            dxh3 = dxh.view(B, S, H)
            perm = ctx.perm
            if perm is not None:
                dgates = team_bwd(C, dxh3, gates, cs, c0, None, None, whh16, fp.err)[0].view(N, 4 * H)
            else:
                dg = []
                mb = C.lstm_max_batch(H)
                for s0 in range(0, B, mb):
                    s1 = min(B, s0 + mb)
                    o = C.lstm_bwd(dxh3[s0:s1], gates[s0:s1], cs[s0:s1], c0[s0:s1].contiguous(), None, None, whh16,
                                   fp.err)
                    dg.append(o[0])
                dgates = (torch.cat(dg) if len(dg) > 1 else dg[0]).view(N, 4 * H)
            dG16 = dgates.to(adt)
            hprev = torch.cat([h0.to(adt).unsqueeze(1), hs16[:, :-1]], dim=1).view(N, H)
            dwhh = _mm(dG16.t(), hprev)
            dwih = _mm(dG16.t(), x16)
            db = dgates.sum(0)
            if perm is not None:           # back to PyTorch's gate-major row order
                inv = torch.empty_like(perm)
                inv[perm] = torch.arange(perm.numel(), device=perm.device)
                dwhh, dwih, db = dwhh[inv], dwih[inv], db[inv]
            grads['rnn.weight_hh_l0'] = dwhh
            grads['rnn.weight_ih_l0'] = dwih
            grads['rnn.bias_ih_l0'] = db
            grads['rnn.bias_hh_l0'] = db
            dx = _mm(dG16, wih16)
        else:
            (wf16,) = rnn_saved
            dxh16 = dxh.to(adt)
            grads['fake_rnn.weight'] = _mm(dxh16.t(), x16)
            grads['fake_rnn.bias'] = dxh.sum(0)
            dx = _mm(dxh16, wf16)
        # ---- pre-RNN
        dpre = dx * (x > 0)
        dpre16 = dpre.to(adt)
        grads['affine_pre_rnn.weight'] = _mm(dpre16.t(), x896)
        grads['affine_pre_rnn.bias'] = dpre.sum(0)
        dx896 = _mm(dpre16, wpre16)
        # ---- entity encoder
        dtl_g = (dtl * g).contiguous()
        wtT16 = wt16.transpose(1, 2).contiguous()
        counts = list(cfg.layout.counts)
        dwt, dw1, db1 = C.encoder_bwd(units2, P['affine_unit_basic_stats.weight'].detach(),
                                              P['affine_unit_basic_stats.bias'].detach(), wtT16, dtl_g, z, dx896, arg,
                                              counts, bool(cfg.compat_bugs))
        grads['affine_unit_basic_stats.weight'] = dw1
        grads['affine_unit_basic_stats.bias'] = db1
        q = z[:, :128]
        # ∂b_τ = Σ_n q[n]·Σ_{u∈τ} dtl[n,u] + Σ_n ∂pool_τ[n]  (each pooled column routes to exactly one unit)
        seg = torch.zeros(U, 6, device=q.device)
        off = 0
        for t, cnt in enumerate(counts):
            seg[off:off + cnt, t] = 1.0
            off += cnt
        dbt = tn_splitk((dtl_g @ seg).contiguous(), q.contiguous())          # (6, 128)
        dpool = dx896[:, 128:].reshape(N, 6, 128).sum(0)
        if cfg.compat_bugs:
            dpool = dpool.clone()
            dpool[3] += dpool[5]
            dpool[5] = 0
        dbt = dbt + dpool
        for t, s in enumerate(TYPE_SUFFIX):
            grads[f'affine_unit_{s}.weight'] = dwt[t]
            grads[f'affine_unit_{s}.bias'] = dbt[t]
        # env embedding (3 → 128): tiny, fp32 torch
        we, be = P['affine_env.weight'].detach(), P['affine_env.bias'].detach()
        de = dx896[:, :128] * ((env2 @ we.t() + be) > 0)
        grads['affine_env.weight'] = de.t() @ env2
        grads['affine_env.bias'] = de.sum(0)
        fp.apply_direct_grads([grads.get(n) for n in fp.param_names], None)
        return (None,) * (12 + len(fp.param_names))


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
        # 'fp32-exact': IEEE fp32 products everywhere (no bf16x3 split): hipBLASLt's exact-f32 GEMMs, the exact-f32
        # MFMA template of the fused ∂X kernel, the exact VALU recurrence and heads/loss kernels, and the encoder /
        # weight-gradient products as exact-f32 torch ops (models/pipelined.py) — the accuracy reference mode
        self.exact = precision == 'fp32-exact'
        if self.exact and policy.config.entity_attention:
            raise ValueError('fp32-exact covers the 1v1 policies (the entity-attention kernels are bf16x3 only)')
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

    def side_stream(self):
        if getattr(self, '_side', None) is None:
            import os
            # DCA_SIDE_PRIORITY=1: the recurrence / weight-gradient side stream at high priority (A/B knob)
            pr = -1 if os.environ.get('DCA_SIDE_PRIORITY', '0') == '1' else 0
            self._side = torch.cuda.Stream(device=self.err.device, priority=pr)
        return self._side

    def use_pipeline(self) -> bool:
        """Time-chunked two-stream step (models/pipelined.py): team LSTM, fully fused LSTM policy, no compat value
        bug (its value loss couples all rows of a sequence). ``DCA_PIPELINE=0`` disables it."""
        import os
        lc = self.loss_cfg
        return ((self.fully_fused or self.attention_fused) and self.cfg.rnn == 'lstm' and lstm_impl() == 'team'
                and not (lc is not None and lc.compat_value_bug) and os.environ.get('DCA_PIPELINE', '1') != '0')

    # Data-parallel split of the direct step (learner/engine.py): the learner sets ``split_hook`` to a callable
    # that the step calls once, at the point where every gradient of :meth:`early_param_names` is final.
    split_hook = None
    early_applied = frozenset()

    def early_param_names(self) -> frozenset:
        """Parameters whose gradients are final before the encoder backward (pre-RNN, recurrence, heads): a
        contiguous suffix of the registration order, so their flat-buffer range is one all-reduce bucket."""
        pre = ('affine_pre_rnn.', 'rnn.', 'affine_head_enum.', 'affine_move_', 'affine_unit_attention.',
               'affine_value.')
        return frozenset(n for n in self.param_names if n.startswith(pre))

    @property
    def chunks(self) -> int:
        import os
        # 1 = no time-chunk overlap: measured on MI355X, GEMMs running concurrently on the other XCDs slow the
        # L2-bound team recurrence by more than they save (bench 10.25 / 10.6 / 11.0 ms at 1 / 2 / 4 chunks)
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
        from ..ops.heads import assemble_loss, batch_norms, heads_loss
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
        if not self.fully_fused and not self.use_pipeline():
            assert rst is None or not bool(rst.any()), 'packed sequences need the pipelined LSTM step'
            xh, emb, _, _ = self.trunk(batch['env'], batch['units'], batch.get('h0'), batch.get('c0'))
            w, b = self.head_cat(dict(zip(self.param_names, self.params)), differentiable=True)
            U = emb.shape[2]
            return heads_loss(xh.reshape(N, -1), w, b, emb.reshape(N, U, -1), batch, cfg, S)[:2]
        H = self.cfg.hidden
        h0 = batch.get('h0')
        c0 = batch.get('c0')
        if h0 is None:
            h0 = torch.zeros(B, H, device=dev)
            c0 = torch.zeros(B, H, device=dev)
        self.refresh()
        if self.use_pipeline():
            from .pipelined import PipelinedPolicyLoss
            part, logp = PipelinedPolicyLoss.apply(self, batch['units'].contiguous(), batch['env'].contiguous(), actions,
                                                   masks, adv, ret, lpo, nret, norms, h0.contiguous(), c0.contiguous(),
                                                   rst, *self.params)
        else:
            assert rst is None or not bool(rst.any()), 'packed sequences need the pipelined LSTM step'
            part, logp = _PolicyLoss.apply(self, batch['units'].contiguous(), batch['env'].contiguous(), actions, masks,
                                           adv, ret, lpo, nret, norms, h0.contiguous(), c0.contiguous(), *self.params)
        loss, metrics = assemble_loss(part, norms, cfg, ret, N, S)
        return loss, metrics

    # ---- per-stage path (entity-attention configs) --------------------------------------------------
    def trunk(self, env, units, h0=None, c0=None):
        p = self.policy
        with torch.autocast('cuda', dtype=torch.bfloat16):
            x, emb = p.encode(env, units)
        x, emb = x.float(), emb.to(torch.bfloat16)
        B, S, _ = x.shape
        if self.cfg.rnn == 'lstm':
            from ..ops.lstm import lstm_sequence
            H = self.cfg.hidden
            if h0 is None:
                h0 = torch.zeros(B, H, device=x.device)
                c0 = torch.zeros(B, H, device=x.device)
            r = p.rnn
            xh, hn, cn, _ = lstm_sequence(x, r.weight_ih_l0, r.weight_hh_l0, r.bias_ih_l0, r.bias_hh_l0,
                                          h0.contiguous(), c0.contiguous(), self.err)
        else:
            xh = F.linear(x, p.fake_rnn.weight, p.fake_rnn.bias)
            hn = cn = None
        return xh, emb, hn, cn

    def check_error(self):
        """Raise if a persistent kernel timed out (host sync — call at iteration boundaries, not per step)."""
        e = int(self.err.item())
        if e:
            raise RuntimeError(f'persistent kernel error code {e} (recurrence hand-off timed out)')
