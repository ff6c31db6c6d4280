"""The fused LSTM learner step: time-major core, weight images, and the autograd-free direct step.

Rows are processed TIME-MAJOR (row = t·B + b) so a time chunk is a contiguous slice of every activation. The
loss and every gradient are computed in ONE forward pass of explicit kernels (no autograd graph); two ways in:

* :class:`PipelinedPolicyLoss` — an ``autograd.Function`` over batch-major inputs (transposed once on entry) whose
  ``backward`` only scales the precomputed gradients by the upstream gradient (used by ``Learner.loss`` callers
  that backprop themselves, and by tests);
* :func:`train_direct` — the learner's hot path: time-major inputs (gathered straight from the HBM replay,
  ``learner.engine.Learner.train_step_replay``), loss normalisers from one kernel (``loss_prep``), the per-step
  working copies of all weights from one gather kernel (``weight_prep``, :class:`WeightImages`), gradients written
  into the flat gradient buffer by one multi-tensor kernel and the loss + metrics by one kernel
  (``loss_assemble``) — about 120 fewer launches per step than the autograd route, and the whole step is
  capturable in one hipGraph.

Time chunks (``DCA_PIPELINE_CHUNKS`` > 1) software-pipeline the step over two streams:

    stream L (recurrence):  F0 F1 F2 F3 ............ B3 B2 B1 B0
    stream A (everything):     H0 H1 H2 H3            G3 G2 G1 G0

``F_c``/``B_c`` = team-LSTM forward/backward over chunk c, ``H_c`` = heads GEMM + heads/loss kernel + heads backward
of chunk c, ``G_c`` = the weight gradients that depend on chunk c. Measured on MI355X it does not pay: work on the
other XCDs slows the L2-bound recurrence more than it saves (round 2: +3.5 % / +7 % per step at 2 / 4 chunks; round 5
with CU-exclusive half teams: 5.45 ms at one chunk against 6.2-6.9 ms chunked, profiles/r5_half_team.md), so the
default is one chunk.

Precisions: ``fp32-exact`` (IEEE fp32 products) and ``fp32`` (fp32 activations, bf16x3-split MFMA operands). Every
product of the step runs in a hand-written kernel — there is no vendor-GEMM branch; a bf16 learner runs on the torch
backend (learner/engine.py).
"""
from __future__ import annotations

import os
from typing import Dict, List, Optional

import torch

from ..ops.lstm import team_bwd, team_fwd
from .policy import TYPE_SUFFIX

LDZ = 160

# parameters whose gradient the direct step accumulates in place (split-K GEMM straight into the flat grad buffer)
DIRECT_GEMM_GRADS = ('rnn.weight_hh_l0', 'rnn.weight_ih_l0', 'affine_pre_rnn.weight', 'affine_pre_rnn.bias')

METRIC_NAMES = ['loss', 'policy_loss', 'entropy_loss', 'advantage_loss', 'entropy', 'advantage', 'approx_kl',
                'clipfrac', 'entropy/enum', 'entropy/x', 'entropy/y', 'entropy/target_unit',
                # in-step V-trace (LossConfig.vtrace): mean truncated importance weight, fraction truncated, and the
                # behaviour KL estimate mean(log μ − log π) of the minibatch
                'offpolicy/rho_mean', 'offpolicy/rho_truncated', 'offpolicy/behaviour_kl']


def _frag_order(w: torch.Tensor) -> torch.Tensor:
    """(R, K) bf16 → MFMA fragment order [R/16][K/32][lane = 16·(k%32 // 8) + r%16][8] (ops/csrc/attn_block.hip)."""
    R, K = w.shape
    return w.view(R // 16, 16, K // 32, 4, 8).permute(0, 2, 3, 1, 4).contiguous()


def _k16_order(w: torch.Tensor) -> torch.Tensor:
    """(R, K) bf16 → 16x16x16 B-fragment order [R/16][K/16][lane = 16·(r%16 // 4) + k%16][4]: element j of lane l is
    w[16·rt + 4·(l>>4) + j][16·ct + (l&15)] (ops/csrc/attn_block.hip gfrag4)."""
    R, K = w.shape
    return w.view(R // 16, 4, 4, K // 16, 16).permute(0, 3, 1, 4, 2).contiguous()


def _acc(a, b):
    """Accumulate a per-chunk gradient: the first chunk's tensor is used as is (no zero fill + add)."""
    return b if a is None else a.add_(b)


def chunk_bounds(S: int, chunks: int):
    c = max(1, min(chunks, S))
    edges = [round(i * S / c) for i in range(c + 1)]
    return [(edges[i], edges[i + 1]) for i in range(c) if edges[i + 1] > edges[i]]


class WeightImages:
    """Per-step working copies of the weights, produced by ONE ``weight_prep`` gather launch from the flat fp32
    parameter buffer (instead of ≈25 cast / stack / permute / cat launches):

    GEMM operands (fp32; the historical ``16`` suffix of the keys is kept): ``wt16`` (6,128,128) type
    weights, ``wtT16`` their transposes, ``wpre16`` (256,896) + ``bpre16``, ``wih16`` (4H,256) rows in unit-major
    gate order, ``whh16`` (4H,H), ``wcat16`` (LDZ,H) = [attention|enum|x|y|value|0-pad];
    always fp32: ``bt`` (6,128), ``bias4`` (4H) = (b_ih + b_hh) in unit-major gate order, ``bcat`` (LDZ).
    The index maps are built once from the parameters' offsets in the flat buffer."""

    def __init__(self, fp, flat: torch.Tensor, with_value: bool):
        cfg = fp.cfg
        H = cfg.hidden
        dev = flat.device
        base = flat.data_ptr()
        P = dict(zip(fp.param_names, fp.params))

        def idx(name):
            p = P[name]
            assert p.is_contiguous() and p.dtype == torch.float32
            off = (p.data_ptr() - base) // 4
            assert 0 <= off and off + p.numel() <= flat.numel(), f'{name} is not a view of the flat buffer'
            return torch.arange(p.numel(), dtype=torch.int64).view(p.shape) + off

        lstm = cfg.rnn == 'lstm'
        perm = fp.gate_perm(H, 'cpu') if lstm else None
        neg = lambda *shape: torch.full(shape, -1, dtype=torch.int64)  # noqa: E731
        # the recurrent layer's input weight — W_ih (rows in unit-major gate order) or the reference's linear fake_rnn
        # W_f (policy.py:67-68, 143-145) — keeps the keys wih16 / wihT16 / ih_s / dx1_s for both
        w_in = idx('rnn.weight_ih_l0')[perm] if lstm else idx('fake_rnn.weight')
        wt = torch.stack([idx(f'affine_unit_{s}.weight') for s in TYPE_SUFFIX])
        head_rows = [idx('affine_unit_attention.weight'), idx('affine_head_enum.weight'),
                     idx('affine_move_x.weight'), idx('affine_move_y.weight'),
                     idx('affine_value.weight') if with_value else neg(1, H)]
        wcat = torch.cat(head_rows + [neg(LDZ - 150, H)], 0)
        parts16 = {'wt16': wt, 'wtT16': wt.transpose(1, 2).contiguous(), 'wpre16': idx('affine_pre_rnn.weight'),
                   'bpre16': idx('affine_pre_rnn.bias'), 'wih16': w_in, 'wcat16': wcat,
                   # (in, 4H) copy for ∂pre = ∂G·W_ih: the ∂X chain's operand K-contiguous per column
                   'wihT16': w_in.t().contiguous()}
        if lstm:
            parts16['whh16'] = idx('rnn.weight_hh_l0')
        if getattr(fp, 'fp32', False):
            # (out, in)-transposed pre-RNN weight: the fused ∂X chain's second operand, K-contiguous per column
            parts16['wpreT'] = idx('affine_pre_rnn.weight').t().contiguous()
        head_b = [idx('affine_unit_attention.bias'), idx('affine_head_enum.bias'), idx('affine_move_x.bias'),
                  idx('affine_move_y.bias'), idx('affine_value.bias') if with_value else neg(1)]
        bcat = torch.cat(head_b + [neg(LDZ - 150)])
        parts32 = {'bt': (torch.stack([idx(f'affine_unit_{s}.bias') for s in TYPE_SUFFIX]), None),
                   'bias4': ((idx('rnn.bias_ih_l0')[perm], idx('rnn.bias_hh_l0')[perm]) if lstm
                             else (idx('fake_rnn.bias'), None)),
                   'bcat': (bcat, None)}
        if cfg.entity_attention and getattr(fp, 'fp32', False):
            # fp32 5v5: the encoder adds b_τ + b_out as well (E0' = E0 + b_out; LayerNorm subtracts it again and the
            # out-projection then accumulates onto E0' in place: no residual copy, no bias pass)
            bo = idx('entity_attn.out.bias')
            parts32['bt'] = (parts32['bt'][0], bo.unsqueeze(0).expand(6, -1))
            parts32['bout'] = (bo, None)
        partsS = {}
        if getattr(fp, 'fp32', False):
            # fp32 learner: the GEMM operand images are fp32 gathers too (the HIP kernels split them into bf16 hi/lo
            # pairs themselves)
            parts32.update({k: (v, None) for k, v in parts16.items()})
            parts16 = {}
            # bf16 hi / lo SLAB-MAJOR images [K/32][rows][32] of the chain kernels' weights (ops/csrc/dx_chain.hip):
            # forward W_pre (256, 896) and W_ih (4H, 256, unit-major rows); ∂X W_ihᵀ (256, 4H) and W_preᵀ (896, 256)
            def slab(t):
                return t.reshape(t.shape[0], t.shape[1] // 32, 32).permute(1, 0, 2).contiguous()
            wpre_i = idx('affine_pre_rnn.weight')
            wih_i = w_in
            if getattr(fp, 'exact', False):
                # IEEE-fp32 learner: the chain kernels take fp32 weights as they are (no hi / lo images); the heads
                # GEMM's W_cat zero-padded to 256 rows and its transpose (the ∂h product's operand)
                if H % 128 == 0:
                    wcat_p = torch.cat([wcat, neg(256 - LDZ, H)], 0)
                    parts32['wcat256'] = (wcat_p, None)
                    parts32['wcatT256'] = (wcat_p.t().contiguous(), None)
                    parts32['bcat256'] = (torch.cat([bcat, neg(256 - LDZ)]), None)
            elif wpre_i.shape[1] % 128 == 0 and wih_i.shape[0] % 128 == 0:
                partsS = {'pre_s': slab(wpre_i), 'ih_s': slab(wih_i), 'dx1_s': slab(wih_i.t()),
                          'dx2_s': slab(wpre_i.t())}
            if H % 128 == 0 and not getattr(fp, 'exact', False):
                # heads GEMM and its ∂X product on the chain kernel's stages: W_cat zero-padded to 256 rows
                wcat_p = torch.cat([wcat, neg(256 - LDZ, H)], 0)
                partsS['wcat_s'] = slab(wcat_p)
                partsS['wcatT_s'] = slab(wcat_p.t())
                parts32['bcat256'] = (torch.cat([bcat, neg(256 - LDZ)]), None)
            if cfg.entity_attention and getattr(fp, 'exact', False):
                # the IEEE-fp32 attention block's fp32 weight images, in the fragment orders of its forward (W_qkv,
                # W_out) and backward (W_outᵀ, W_qkv k16) — gathered here, no per-step split or permute launches
                wq_i, wo_i = idx('entity_attn.qkv.weight'), idx('entity_attn.out.weight')
                parts32['wq_x'] = (_frag_order(wq_i), None)
                parts32['wo_x'] = (_frag_order(wo_i), None)
                parts32['wot_x'] = (_frag_order(wo_i.t().contiguous()), None)
                parts32['wq4_x'] = (_k16_order(wq_i), None)
            elif cfg.entity_attention:
                # the fused attention block's W_qkv / W_out hi / lo images in MFMA fragment order (attn_block.hip),
                # from this same gather instead of two split + two permute-copy launches before the block
                partsS['wq_f'] = _frag_order(idx('entity_attn.qkv.weight'))
                partsS['wo_f'] = _frag_order(idx('entity_attn.out.weight'))
        self.shapes16 = {k: tuple(v.shape) for k, v in parts16.items()}
        self.shapes32 = {k: tuple(v[0].shape) for k, v in parts32.items()}
        m16 = torch.cat([v.reshape(-1) for v in parts16.values()]) if parts16 else torch.zeros(0, dtype=torch.int64)
        m32 = torch.cat([torch.stack([a.reshape(-1), (b.reshape(-1) if b is not None else neg(a.numel()))], 1)
                         for a, b in parts32.values()])
        # (expand() above is a broadcast view; reshape copies it)
        self.map16 = m16.to(torch.int32).to(dev)
        self.map32 = m32.to(torch.int32).contiguous().to(dev)
        self.buf16 = torch.empty(m16.numel(), dtype=torch.bfloat16, device=dev)
        self.buf32 = torch.empty(m32.shape[0], dtype=torch.float32, device=dev)
        self.views: Dict[str, torch.Tensor] = {}
        self.mapS = self.bufH = self.bufL = None
        if partsS:
            self.mapS = torch.cat([v.reshape(-1) for v in partsS.values()]).to(torch.int32).to(dev)
            self.bufH = torch.empty(self.mapS.numel(), dtype=torch.bfloat16, device=dev)
            self.bufL = torch.empty_like(self.bufH)
            o = 0
            for k, v in partsS.items():
                self.views[k] = (self.bufH[o:o + v.numel()].view(v.shape), self.bufL[o:o + v.numel()].view(v.shape))
                o += v.numel()
        o = 0
        for k, shp in self.shapes16.items():
            n = 1
            for d in shp:
                n *= d
            self.views[k] = self.buf16[o:o + n].view(shp)
            o += n
        o = 0
        for k, shp in self.shapes32.items():
            n = 1
            for d in shp:
                n *= d
            self.views[k] = self.buf32[o:o + n].view(shp)
            o += n
        self.flat = flat

    def refresh(self, C) -> Dict[str, torch.Tensor]:
        if self.mapS is not None:
            C.weight_prep(self.flat, self.map16, self.buf16, self.map32, self.buf32, self.mapS, self.bufH, self.bufL)
        else:
            C.weight_prep(self.flat, self.map16, self.buf16, self.map32, self.buf32)
        return self.views


# Fixed choices of the step, each measured against its alternative in earlier rounds (the alternatives were removed):
# * the weight-gradient GEMMs of the recurrence and pre-RNN layer run on the (then idle) recurrence stream, beside the
#   ∂X chain of the main stream; in the exact learner ∂W_pre / ∂b_pre go to the main stream after the encoder
#   backward instead (5.514 vs 5.560 ms per step; the bf16x3 learner keeps them on the side stream: 4.911 vs 4.921);
# * the fp32 forward chain relu(x896·W_preᵀ + b)·W_ihᵀ, the heads GEMM and its ∂X product, and the ∂X chain
#   (∂G·W_ih)⊙[x>0]·W_pre are hand-written kernels (ops/csrc/dx_chain.hip), not vendor GEMMs;
# * the fp32 5v5 attention block forward and backward are one kernel each (ops/csrc/attn_block.hip; the five-launch
#   backward took 1858 vs 1660 µs), ∂W_out / ∂W_qkv on the side stream after the encoder backward (8.10 vs 8.13 ms);
#   fp32-exact runs their IEEE-fp32 twins (the same kernels templated on the operand precision);
# * the exact recurrence's gate activations use the hardware exp / reciprocal: products-exact, the same worst
#   tensor errors against float64 as libm expf / tanhf (PPO 2.50e-6 both), 0.5 ms per step faster.


# 5v5: ∂W_out on the main stream after the encoder backward, ∂W_qkv alone on the recurrence stream (A/B knob, round 6:
# both GEMMs serial on the recurrence stream left ∂W_qkv exposed at the step's end, profiles/r5_5v5_exact_timeline.txt)
# (A third stream for ∂W_out, concurrent with both, measured 0.27 ms slower: profiles/r6_gemm_map_and_5v5_streams.md.)
_WG_BALANCE = os.environ.get('DCA_5V5_WG_BALANCE', '1')


def fused_step_tm(fp, *args, **kw):
    """:func:`_fused_step_tm`: every product on a hand-written kernel (no torch GEMM, so no matmul mode to pin)."""
    return _fused_step_tm(fp, *args, **kw)


def _fused_step_tm(fp, W: Dict[str, torch.Tensor], P: Dict[str, torch.Tensor], units_t, env_t, act_t, msk_t, adv_t,
                   ret_t, lpo_t, nret_t, norms, h0, c0, B: int, S: int, gout: Optional[Dict[str, torch.Tensor]] = None,
                   reset_t: Optional[torch.Tensor] = None, vt_t: Optional[torch.Tensor] = None):
    """Loss partials and all parameter gradients of one minibatch, from TIME-MAJOR rows (row = t·B + b).

    ``W`` = :class:`WeightImages` views, ``P`` = fp32 parameters (for the small fp32 weights used directly).
    ``gout`` (direct mode): parameter name → gradient tensor (a view of the flat gradient buffer); the big
    weight-gradient GEMMs (W_hh, W_ih, pre-RNN) ACCUMULATE straight into those and are left out of ``grads``.
    Returns (partials (R,16) f32, logp (N) f32 time-major, grads {param name → tensor})."""
    from ..ops.gemm import gemm_tn as _gemm_tn
    exact = bool(getattr(fp, 'exact', False))
    lin = fp.cfg.rnn != 'lstm'          # the reference's linear fake_rnn layer (compat preset): no recurrence
    if exact and B > 32 and not lin:
        # lstm_team.hip plan(): the sequences run as chains of ≤ 4 rows (one XCD team each) on the exact fp32 VALU
        # recurrence; more than 4 rows per chain take the bf16x3 MFMA team kernel — not IEEE fp32
        raise ValueError(f'fp32-exact: at most 32 sequences per step and GPU (got {B}); use precision fp32')

    def gemm_tn(*a, **k):
        # weight gradients: split-K MFMA; IEEE-fp32 learner: exact v_mfma_f32_16x16x4_f32 (ops/csrc/gemm_tn.hip)
        return _gemm_tn(*a, exact=exact, **k)
    C = fp.C
    cfg, lc = fp.cfg, fp.loss_cfg
    N = B * S
    U = units_t.shape[1]
    H = cfg.hidden
    dev = units_t.device
    counts = list(cfg.layout.counts)
    main = torch.cuda.current_stream(dev)
    sL = fp.side_stream()
    w1, b1 = P['affine_unit_basic_stats.weight'].detach(), P['affine_unit_basic_stats.bias'].detach()
    we, be = P['affine_env.weight'].detach(), P['affine_env.bias'].detach()
    wt16, wtT16, wpre16 = W['wt16'], W['wtT16'], W['wpre16']
    wih16, whh16 = W['wih16'], W.get('whh16')
    bt, bias_p = W['bt'], W['bias4']
    # ---- encoder, pre-RNN, input projection over all rows (row-parallel, fast)
    attn = cfg.entity_attention
    assert getattr(fp, 'fp32', False), 'the fused step runs at fp32 / fp32-exact (bf16: torch backend)'
    adt = torch.float32         # fp32 activations; bf16x3 MFMA operands (fp32) or IEEE-fp32 products (fp32-exact)
    # (exact: the IEEE-fp32 encoder variant, ops/csrc/encoder.hip encoder_fwd_x_kernel)
    # time chunks with the 1v1 fp32 policies: the encoder and the forward chain run chunk by chunk, each chunk's
    # recurrence launched as soon as its input projection is ready (the next chunk's encoder runs beside it)
    front = len(chunk_bounds(S, fp.chunks)) > 1 and not attn and not lin and reset_t is None
    enc_done: List[torch.cuda.Event] = []
    if front:
        x896 = torch.empty(N, 896, device=dev)
        emb = torch.empty(N, U, 128, device=dev)
        arg = torch.empty(N, 6, 128, dtype=torch.uint8, device=dev)
        x16 = torch.empty(N, 256, device=dev)
        xp = torch.empty(N, 4 * H, device=dev)
        if exact:
            nil = wpre16.new_empty(0)
            cw = (wpre16, nil, wih16, nil)
        else:
            cw = (W['pre_s'][0], W['pre_s'][1], W['ih_s'][0], W['ih_s'][1])
        for t0, t1 in chunk_bounds(S, fp.chunks):
            r0, r1 = t0 * B, t1 * B
            C.encoder_fwd(units_t[r0:r1], env_t[r0:r1], w1, b1, wt16, bt, we, be, counts, bool(cfg.compat_bugs),
                          exact=exact, x896_out=x896[r0:r1], emb_out=emb[r0:r1], arg_out=arg[r0:r1])
            if cfg.compat_bugs:   # reference policy.py:127: enemy-tower pool = enemy-nonhero pool
                x896[r0:r1, 768:896] = x896[r0:r1, 512:640]
                arg[r0:r1, 5] = arg[r0:r1, 3]
            C.pre_rnn_chain(x896[r0:r1], cw[0], cw[1], W['bpre16'], cw[2], cw[3], x_out=x16[r0:r1],
                            xp_out=xp[r0:r1])
            e = torch.cuda.Event()
            e.record(main)
            enc_done.append(e)
        xp4 = xp.view(S, B, H, 4)
    else:
        x896, emb, arg = C.encoder_fwd(units_t, env_t, w1, b1, wt16, bt, we, be, counts, bool(cfg.compat_bugs), exact=exact)
        if attn:
            # 5v5 entity attention, ONE kernel (ops/csrc/attn_block.hip attn_block_fwd_f32_kernel): LayerNorm → QKV
            # (bias added in the kernel) → 4-head self-attention → out-projection onto E0' = E0 + b_out (bias folded into
            # bt) → pools / argmax of the attended embeddings; bf16x3 operands, or the IEEE-fp32 twin at fp32-exact
            toff = fp.type_offset_list()
            bqkv = P['entity_attn.qkv.bias'].detach()
            # one kernel per step; E0' stays untouched (the LayerNorm backward's input), E1 is a new tensor
            E0p = emb.view(N * U, 128)
            if exact:                          # fp32 fragment images: the IEEE-fp32 block kernel
                nil = E0p.new_empty(0)
                wq, wo = (W['wq_x'], nil), (W['wo_x'], nil)
            elif 'wq_f' in W:                  # hi / lo fragment images from the step's weight_prep launch
                wq, wo = W['wq_f'], W['wo_f']
            else:
                wq = [_frag_order(t) for t in C.split_bf16x2(P['entity_attn.qkv.weight'].detach())]
                wo = [_frag_order(t) for t in C.split_bf16x2(P['entity_attn.out.weight'].detach())]
            arg = torch.empty(N, 6, 128, dtype=torch.uint8, device=dev)
            Xn, ln_mu, ln_rs, QKV, Oat, lse, E1 = C.attn_block_fwd(
                E0p, W['bout'], P['entity_attn.ln.weight'].detach(), P['entity_attn.ln.bias'].detach(), wq[0], wq[1],
                bqkv, wo[0], wo[1], toff, x896, arg, bool(cfg.compat_bugs), 1e-5)
            emb = E1.view(N, U, 128)
        elif cfg.compat_bugs:   # reference policy.py:127: enemy-tower pool = enemy-nonhero pool
            x896[:, 768:896] = x896[:, 512:640]
            arg[:, 5] = arg[:, 3]
        # the forward chain relu(x896·W_preᵀ + b)·W_ihᵀ in ONE kernel (ops/csrc/dx_chain.hip; x16 > 0 ⟺ x > 0)
        if exact:
            # IEEE-fp32 forward chain: the same kernel on v_mfma_f32_16x16x4_f32 with the fp32 weights as they are
            nil = wpre16.new_empty(0)
            x16, xp = C.pre_rnn_chain(x896, wpre16, nil, W['bpre16'], wih16, nil)
            xp4 = xp.view(S, B, H, 4) if not lin else None
        else:
            if 'pre_s' in W:                 # hi / lo images from the step's weight_prep launch
                fw1, fw2 = W['pre_s'], W['ih_s']
            else:
                fw1, fw2 = C.split_bf16x2(wpre16, True), C.split_bf16x2(wih16, True)   # slab-major bf16 hi / lo images
            x16, xp = C.pre_rnn_chain(x896, fw1[0], fw1[1], W['bpre16'], fw2[0], fw2[1])
            xp4 = xp.view(S, B, H, 4) if not lin else None
    if lin:
        # fake_rnn: h = pre·W_fᵀ + b_f (the chain kernel's second product) — no activation, no recurrence
        hs16 = xp.add_(bias_p).view(S, B, H)
        cs = gates4 = None
    else:
        hs16 = torch.empty(S, B, H, dtype=adt, device=dev)
        cs = torch.empty(S, B, H, device=dev)
        gates4 = torch.empty(S, B, H, 4, device=dev)
    spans = chunk_bounds(S, 1 if lin else fp.chunks)
    one = len(spans) == 1            # single chunk: outputs are used as produced (no staging copies)
    # sequence packing (learner/ingest.py): per-(step, row) episode-start flags, time-major (S, B) u8 — the team
    # recurrence zeroes h, c before a flagged step (forward) and stops the gradient there (backward)
    rst = reset_t.reshape(S, B) if reset_t is not None else None
    assert rst is None or one, 'packed sequences run as one time chunk'
    assert one or not attn, "the entity-attention step runs as one time chunk"
    if not one:
        dxh = torch.empty(S, B, H, device=dev)
        z = torch.empty(N, 256, device=dev)
        dtl = torch.empty(N, U, device=dev)
        logp = torch.empty(N, device=dev)
    dWcat = dbcat = None
    heads_wg = None
    parts: List[torch.Tensor] = []
    # heads_loss algo: 0 = PPO clipped surrogate, 1 = VPG (reference), 2 = PPO's truncated-IS off-policy term
    algo = (2 if getattr(lc, 'offpolicy', 'clip') == 'tis' else 0) if lc.algo == 'ppo' else 1
    # ---- forward recurrence on stream L, heads (+ heads backward) per chunk on the main stream
    ready = torch.cuda.Event()
    ready.record(main)
    if not front:
        sL.wait_event(ready)
    # every recurrence chunk is enqueued up front (the host must never hold the recurrence stream back while it
    # is busy launching the per-chunk work of the main stream)
    h_c, c_c = h0.contiguous(), c0.contiguous()
    fwd_done = []
    with torch.cuda.stream(sL):
        for i, (t0, t1) in enumerate([] if lin else spans):
            if front:
                sL.wait_event(enc_done[i])
            o = team_fwd(C, xp4[t0:t1], whh16, h_c, c_c, fp.err, False, time_major=True,
                         hs_out=hs16[t0:t1], cs_out=cs[t0:t1], gates_out=gates4[t0:t1], bias4=bias_p,
                         reset=rst)
            h_c, c_c = o[4], o[5]
            e = torch.cuda.Event()
            e.record(sL)
            fwd_done.append(e)
    if lin:
        fwd_done.append(ready)
    # weight operands of the fused ∂X kernel: bf16 hi/lo images from the step's weight_prep (exact: fp32 as is)
    if exact:
        dx_w = (W['wihT16'], W['wihT16'].new_empty(0), W['wpreT'], W['wpreT'].new_empty(0))
    elif 'dx1_s' in W:
        dx_w = tuple(W['dx1_s']) + tuple(W['dx2_s'])
    else:
        dx_w = tuple(C.split_bf16x2(W['wihT16'], True)) + tuple(C.split_bf16x2(W['wpreT'], True))
    # heads GEMM + its ∂X product on the chain kernel's stages (bf16x3 images, or exact: fp32 W_cat padded to 256)
    if exact:
        nil = W['wcat256'].new_empty(0)
        hw = ((W['wcat256'], nil), (W['wcatT256'], nil), W['bcat256'])
    else:
        hw = (W['wcat_s'], W['wcatT_s'], W['bcat256'])
    fp.vtrace_stats = None
    for (t0, t1), done in zip(spans, fwd_done):
        main.wait_event(done)
        r0, r1 = t0 * B, t1 * B
        xh = hs16[t0:t1].view(-1, H)
        zc = C.rowmm_out256(xh, hw[0][0], hw[0][1], hw[2])   # (n, 256), padding columns 0
        if vt_t is not None:
            # V-trace INSIDE the step (LossConfig.vtrace): this step's own values (z column 149) and log-probs of the
            # recorded actions (a first, forward-only pass of the heads kernel) against the actor's behaviour
            # log-probs (lpo_t) give the advantages and value targets — for fresh and replayed experience alike,
            # at the weights being trained (ops/csrc/scan.hip vtrace_step_kernel), then normalised over the valid rows
            from ..constants import EPS
            from ..ops.scan import vtrace_step
            assert one, 'in-step V-trace runs as one time chunk'
            zero = fp.scratch('vt_zero', (N,), torch.float32, dev)
            _, _, _, lp_a = C.heads_loss(zc, emb, act_t, msk_t, zero, zero, zero, zero, norms, 0, False, S, B,
                                         float(lc.clip_eps), 0.0, 0.0, dz_bf16=False, precise=exact)
            adv_v, ret_t, vstats = vtrace_step(None, lp_a, lpo_t, vt_t, B, S, lc.gamma, lc.gae_lambda,
                                               getattr(lc, 'vtrace_rho_bar', 1.0), getattr(lc, 'vtrace_c_bar', 1.0),
                                               z=zc, vcol=149)
            adv_t = torch.empty_like(adv_v)
            C.adv_normalize(adv_v, vt_t[:, 2].contiguous(), adv_t, float(EPS))
            fp.vtrace_stats = vstats
        dz16, dtl_c, part, lp = C.heads_loss(zc, emb[r0:r1], act_t[r0:r1], msk_t[r0:r1], adv_t[r0:r1],
                                             ret_t[r0:r1], lpo_t[r0:r1], nret_t[r0:r1], norms, algo,
                                             bool(lc.compat_value_bug), S, B, float(lc.clip_eps),
                                             float(lc.entropy_coef), float(lc.vf_coef), dz_bf16=False,
                                             precise=exact)
        parts.append(part)
        first = dWcat is None
        if first:
            dbcat = torch.empty(LDZ, device=dev)
        dzw = dz16[:, :LDZ]                              # (the heads' columns of the 256-wide ∂z)
        if one:
            # single chunk: the heads' weight gradient waits on the recurrence stream behind the backward
            # recurrence (off the path between the two recurrences; joined with the other weight gradients)
            dWcat = torch.empty(LDZ, H, device=dev)
            heads_wg = (dzw, xh)
        else:
            dWcat = gemm_tn(dzw, xh, out=dWcat, accumulate=not first, colsum=dbcat)
        if one:
            z, dtl, logp = zc, dtl_c, lp
            dxh = C.rowmm_in256(dz16, hw[1][0], hw[1][1]).view(S, B, H)
        else:
            z[r0:r1].copy_(zc)
            dtl[r0:r1].copy_(dtl_c)
            logp[r0:r1].copy_(lp)
            dxh[t0:t1].copy_(C.rowmm_in256(dz16, hw[1][0], hw[1][1]).view(t1 - t0, B, H))
    heads_done = torch.cuda.Event()
    heads_done.record(main)
    # ---- backward recurrence on stream L (reverse chunks), weight gradients per chunk on the main stream
    grads: Dict[str, torch.Tensor] = {}
    fp.split_head_grads(dWcat, dbcat, grads)
    # data-parallel split (direct mode, single chunk): see the split point in the backward loop below
    split = fp.split_hook if (gout is not None and one) else None
    early_names = fp.early_param_names() if split is not None else frozenset()
    fp.early_applied = frozenset()
    dgates16 = None if lin else torch.empty(S, B, H, 4, dtype=adt, device=dev)   # ∂gates straight from the kernel
    db = dw1 = db1 = dWt = dbt = dWe = dbe = None
    dgam = dbet = None
    side_after: List = []                # side-stream work enqueued after the encoder backward (5v5 fused path)
    after_enc: List = []                 # main-stream work enqueued after the encoder backward (exact ∂W_pre)
    if attn:
        dWout = torch.empty(128, 128, device=dev)
        dbout = torch.empty(128, device=dev)
        dWqkv = torch.empty(384, 128, device=dev)
        dbqkv = torch.empty(384, device=dev)
    gperm = fp.gate_perm_i32(H, dev)
    # weight-gradient GEMMs: split-K MFMA over the B·S rows (ops/csrc/gemm_tn.hip), written in PyTorch's gate-major
    # row order through the gate permutation; in direct mode accumulated straight into the flat gradient buffer
    direct = gout is not None
    if lin:
        dWhh = None
        dWih = grads['fake_rnn.weight'] = torch.empty(H, x16.shape[1], device=dev)
        dbf = grads['fake_rnn.bias'] = torch.empty(H, device=dev)
    else:
        dWhh = gout['rnn.weight_hh_l0'] if direct else torch.zeros(4 * H, H, device=dev)
        dWih = gout['rnn.weight_ih_l0'] if direct else torch.zeros(4 * H, x16.shape[1], device=dev)
    dWpre = gout['affine_pre_rnn.weight'] if direct else torch.zeros(wpre16.shape[0], wpre16.shape[1], device=dev)
    dbpre = gout['affine_pre_rnn.bias'] if direct else torch.zeros(wpre16.shape[0], device=dev)
    h016 = h0.to(adt).contiguous()
    sL.wait_event(heads_done)
    dh_n = dc_n = None
    bwd_done = []
    with torch.cuda.stream(sL):
        for t0, t1 in ([] if lin else reversed(spans)):
            cinit = c0.contiguous() if t0 == 0 else cs[t0 - 1]
            o = team_bwd(C, dxh[t0:t1], gates4[t0:t1], cs[t0:t1], cinit, dh_n, dc_n, whh16, fp.err,
                         time_major=True, dg_out=dgates16[t0:t1], dg_bf16=False,
                         want_dbias=True, reset=rst)
            dh_n, dc_n = o[1], o[2]
            db = _acc(db, o[3])
            e = torch.cuda.Event()
            e.record(sL)
            bwd_done.append(e)
        if lin:
            bwd_done.append(heads_done)
        if heads_wg is not None:
            gemm_tn(heads_wg[0], heads_wg[1], out=dWcat, colsum=dbcat)
    # single chunk: the recurrence stream (idle once the backward recurrence is done) takes the weight-gradient GEMMs
    # of W_hh, W_ih and the pre-RNN layer, off the critical ∂X chain (∂pre → ∂x896 → encoder backward) on the main
    # stream; the main stream joins it before the DP split point and before returning
    wg_side = one
    wg_done = None
    for (t0, t1), done in zip(reversed(spans), bwd_done):
        main.wait_event(done)
        r0, r1 = t0 * B, t1 * B
        n = r1 - r0
        dG16 = dxh.view(n, H) if lin else dgates16[t0:t1].view(n, 4 * H)
        with torch.cuda.stream(sL if wg_side else main):
            if lin:
                pass                                   # ∂W_f, ∂b_f: below (no recurrent weight)
            elif rst is not None:
                # packed: the h_{t-1} operand is zero where an episode starts at t (the forward never used it)
                hprev = torch.cat([h016.unsqueeze(0), hs16[:S - 1]], 0).masked_fill_(rst.bool().unsqueeze(2), 0.0)
                gemm_tn(dG16, hprev.view(n, H), out=dWhh, perm=gperm, accumulate=True)
            elif t0 > 0:
                gemm_tn(dG16, hs16[t0 - 1:t1 - 1].view(n, H), out=dWhh, perm=gperm, accumulate=True)
            else:       # h_{t-1} rows: h0 for t = 0, then hs[0 : t1-1] — no concatenation materialised
                gemm_tn(dG16, hs16[0:t1 - 1].view(n - B, H), out=dWhh, perm=gperm, accumulate=True, b0=h016)
            if lin:
                gemm_tn(dG16, x16[r0:r1], out=dWih, colsum=dbf)
            else:
                gemm_tn(dG16, x16[r0:r1], out=dWih, perm=gperm, accumulate=True)
        # ∂pre = (∂G·W_ih)⊙[x16 > 0] and ∂x896 = ∂pre·W_pre in one launch (the ∂pre tile stays in LDS)
        dpre16, dx896 = C.dpre_dx(dG16, dx_w[0], dx_w[1], x16[r0:r1], dx_w[2], dx_w[3])
        pre_main = wg_side and split is None and exact
        if pre_main:
            with torch.cuda.stream(sL):       # the side stream ends with ∂W_ih
                wg_done = torch.cuda.Event()
                wg_done.record(sL)
            after_enc.append(lambda d=dpre16, xr=x896[r0:r1]: gemm_tn(d, xr, out=dWpre, accumulate=True,
                                                                      colsum=dbpre))
        elif wg_side:
            sL.wait_stream(main)
            with torch.cuda.stream(sL):
                gemm_tn(dpre16, x896[r0:r1], out=dWpre, accumulate=True, colsum=dbpre)
                wg_done = torch.cuda.Event()
                wg_done.record(sL)
        else:
            gemm_tn(dpre16, x896[r0:r1], out=dWpre, accumulate=True, colsum=dbpre)
        if split is not None:
            if wg_done is not None:
                main.wait_event(wg_done)
                wg_done = None
            # DP split point: every gradient of the recurrence, pre-RNN and heads is final here (the big ones are
            # already in the flat buffer); apply the small ones and let the learner all-reduce those buckets while
            # the encoder backward below runs (see Learner._replay_split)
            if not lin:
                grads['rnn.bias_ih_l0'] = db         # (gate-major already: the kernel writes PyTorch's order)
                grads['rnn.bias_hh_l0'] = db
            early = [grads.pop(nm, None) if nm in early_names else None for nm in fp.param_names]
            fp.apply_direct_grads(early, None, set_mask=False)    # the final call records the full mask
            fp.early_applied = early_names
            split()
            split = None
        demb_in = None
        if attn:
            # one kernel from ∂x896 / the pointer gradient to ∂E0; the two weight-gradient GEMMs over the N·U unit
            # rows (∂W_out = ∂E1ᵀ·O, ∂W_qkv = ∂QKVᵀ·Xn, with their bias column sums) go to the recurrence stream
            if exact:
                nil = E0p.new_empty(0)
                wot, wq4 = (W['wot_x'], nil), (W['wq4_x'], nil)
            else:
                wot = [_frag_order(t) for t in C.split_bf16x2(P['entity_attn.out.weight'].detach().t().contiguous())]
                wq4 = [_k16_order(t) for t in C.split_bf16x2(P['entity_attn.qkv.weight'].detach())]
            dE1, dQKV, demb_in, lnsum = C.attn_block_bwd(
                dtl, z, dx896, arg, toff, bool(cfg.compat_bugs), Oat, QKV, bqkv, lse, E0p, W['bout'], ln_mu, ln_rs,
                P['entity_attn.ln.weight'].detach(), wot[0], wot[1], wq4[0], wq4[1], None)
            dgam, dbet, dbt_attn = lnsum[:128], lnsum[128:256], lnsum[256:].view(6, 128)
            dbout = torch.empty(128, device=dev)
            dbqkv = torch.empty(384, device=dev)
            if wg_side and _WG_BALANCE == '1':
                # ∂W_qkv (the larger: 384 × 128 over the N·U rows) alone on the recurrence stream from the attention
                # backward on; ∂W_out on the main stream after the encoder backward — the two streams' tails balance
                sL.wait_stream(main)
                side_after.append(lambda: gemm_tn(dQKV, Xn, out=dWqkv, colsum=dbqkv))
                after_enc.append(lambda: gemm_tn(dE1, Oat, out=dWout, colsum=dbout))
            elif wg_side:
                # enqueued AFTER the encoder backward below (side_after): issued here, the graph ran the two GEMMs
                # (156 + 401 µs) and then the encoder backward strictly one after the other
                sL.wait_stream(main)
                side_after.append(lambda: (gemm_tn(dE1, Oat, out=dWout, colsum=dbout),
                                           gemm_tn(dQKV, Xn, out=dWqkv, colsum=dbqkv)))
            else:
                dWout = gemm_tn(dE1, Oat, colsum=dbout)
                dWqkv = gemm_tn(dQKV, Xn, colsum=dbqkv)
        # ∂b_τ, ∂W_env, ∂b_env: one pass over the rows (ops/csrc/glue.hip enc_small_grads); single chunk: on the
        # recurrence stream, concurrent with the encoder backward
        def small_grads():
            return C.enc_small_grads(z[r0:r1], dtl[r0:r1], fp.type_offsets(dev), dx896, env_t[r0:r1], we, be,
                                     bool(cfg.compat_bugs))
        small = None
        if wg_side and not side_after:
            sL.wait_stream(main)
            with torch.cuda.stream(sL):
                small = small_grads()
                wg_done = torch.cuda.Event()
                wg_done.record(sL)
        dwt_c, dw1_c, db1_c = C.encoder_bwd(units_t[r0:r1], w1, b1, wtT16, dtl[r0:r1], z[r0:r1],
                                            dx896, arg[r0:r1], counts, bool(cfg.compat_bugs), demb_in=demb_in,
                                            exact=exact)
        for fn in after_enc:
            fn()
        after_enc.clear()
        if side_after:
            # the side stream already waits on the attention backward (not on the encoder backward just issued)
            with torch.cuda.stream(sL):
                for fn in side_after:
                    fn()
                small = small_grads()
                wg_done = torch.cuda.Event()
                wg_done.record(sL)
            side_after.clear()
        dw1 = _acc(dw1, dw1_c)
        db1 = _acc(db1, db1_c)
        dWt = _acc(dWt, dwt_c)
        dbt_c, dWe_c, dbe_c = small if small is not None else small_grads()
        dbt = _acc(dbt, dbt_attn if attn else dbt_c)
        dWe = _acc(dWe, dWe_c)
        dbe = _acc(dbe, dbe_c)
    if wg_done is not None:
        main.wait_event(wg_done)
    if not direct:
        if not lin:
            grads['rnn.weight_hh_l0'] = dWhh
            grads['rnn.weight_ih_l0'] = dWih
        grads['affine_pre_rnn.weight'] = dWpre
        grads['affine_pre_rnn.bias'] = dbpre
    if not lin and 'rnn.bias_ih_l0' not in fp.early_applied:
        grads['rnn.bias_ih_l0'] = db
        grads['rnn.bias_hh_l0'] = db
    grads['affine_unit_basic_stats.weight'] = dw1
    grads['affine_unit_basic_stats.bias'] = db1
    for t, s in enumerate(TYPE_SUFFIX):
        grads[f'affine_unit_{s}.weight'] = dWt[t]
        grads[f'affine_unit_{s}.bias'] = dbt[t]
    grads['affine_env.weight'] = dWe
    grads['affine_env.bias'] = dbe
    if attn:
        grads['entity_attn.ln.weight'] = dgam
        grads['entity_attn.ln.bias'] = dbet
        grads['entity_attn.qkv.weight'] = dWqkv
        grads['entity_attn.qkv.bias'] = dbqkv
        grads['entity_attn.out.weight'] = dWout
        grads['entity_attn.out.bias'] = dbout
    part = parts[0] if len(parts) == 1 else torch.cat(parts, 0)
    return part, logp, grads


class PipelinedPolicyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fp, units, env, actions, masks, adv, ret, logp_old, nret, norms, h0, c0, reset, vt, *params):
        P = dict(zip(fp.param_names, params))
        B, S, U, _ = units.shape
        N = B * S
        tm = (lambda x: x.reshape(B, S, *x.shape[1:]).transpose(0, 1).reshape(N, *x.shape[1:]).contiguous())
        units_t = units.transpose(0, 1).reshape(N, U, 10).contiguous()
        env_t = env.transpose(0, 1).reshape(N, 3).contiguous()
        W = fp.weight_images().refresh(fp.C)
        rst_t = reset.reshape(B, S).transpose(0, 1).reshape(N).contiguous() if reset is not None else None
        part, logp, grads = fused_step_tm(fp, W, P, units_t, env_t, tm(actions), tm(masks), tm(adv), tm(ret),
                                          tm(logp_old), tm(nret), norms, h0, c0, B, S, reset_t=rst_t,
                                          vt_t=tm(vt.reshape(N, 4)) if vt is not None else None)
        ctx.grads = [grads.get(nm) for nm in fp.param_names]
        ctx.fp = fp
        logp_b = logp.view(S, B).t().reshape(N)        # back to batch-major (B·S) row order
        ctx.mark_non_differentiable(logp_b)
        return part.sum(0), logp_b

    @staticmethod
    def backward(ctx, gpart, _glogp):
        ctx.fp.apply_direct_grads(ctx.grads, gpart[15])
        ctx.grads = None
        return (None,) * (14 + len(ctx.fp.param_names))


def train_direct(fp, batch_tm: Dict[str, torch.Tensor], B: int, S: int) -> torch.Tensor:
    """One learner step without autograd: gradients are ADDED into the parameters' ``.grad`` (views of the flat
    gradient buffer), ``fp.grad_mask`` marks which parameters got one. ``batch_tm`` holds time-major rows
    (``units (N,U,10)``, ``env (N,3)``, ``actions``/``masks (N,A)`` u8, ``adv``/``ret``/``logp_old``/``norm_ret``
    (N,)) plus ``h0``/``c0 (B,H)``. Returns the metrics vector (16,) laid out as :data:`METRIC_NAMES`."""
    C = fp.C
    lc = fp.loss_cfg
    N = B * S
    dev = batch_tm['units'].device
    norms = fp.scratch('norms', (8,), torch.float32, dev)
    # the loss normalisers only feed the heads/loss kernel (after the forward recurrence, which runs on the side
    # stream and is waited for by the main stream): computed on that stream, beside the encoder and pre-RNN chain
    main = torch.cuda.current_stream(dev)
    sL = fp.side_stream()
    sL.wait_stream(main)
    with torch.cuda.stream(sL):
        C.loss_prep(batch_tm['actions'], fp.loss_prep_ws(dev), norms)
        if lc.compat_value_bug and lc.vf_coef > 0:
            # the reference's value target is the LAST sequence's returns broadcast over the batch (optimizer.py:603,
            # SURVEY §2.10-2): Σ G_last and Σ G_last² of row b = B-1 for the heads kernel and the loss assembly
            g_last = batch_tm['ret'].view(S, B)[:, B - 1]
            norms[6:8] = torch.stack([g_last.sum(), (g_last * g_last).sum()])
    W = fp.weight_images().refresh(C)
    P = dict(zip(fp.param_names, fp.params))
    H = fp.cfg.hidden
    h0 = batch_tm.get('h0')
    c0 = batch_tm.get('c0')
    if h0 is None:
        h0 = torch.zeros(B, H, device=dev)
        c0 = torch.zeros(B, H, device=dev)
    gout = {nm: P[nm].grad for nm in DIRECT_GEMM_GRADS if nm in P}
    vt = batch_tm.get('vt') if getattr(lc, 'vtrace', False) else None
    if getattr(lc, 'vtrace', False) and vt is None:
        raise ValueError('LossConfig.vtrace needs the per-row vt field (learner/optimizer.py advantages="vtrace-step")')
    part, _, grads = fused_step_tm(fp, W, P, batch_tm['units'], batch_tm['env'], batch_tm['actions'],
                                   batch_tm['masks'], batch_tm['adv'], batch_tm['ret'], batch_tm['logp_old'],
                                   batch_tm['norm_ret'], norms, h0, c0, B, S, gout=gout,
                                   reset_t=batch_tm.get('reset'), vt_t=vt)
    fp.apply_direct_grads([grads.get(nm) for nm in fp.param_names], None,
                          written=set(gout) | set(fp.early_applied))
    out = torch.empty(16, device=dev)
    C.loss_assemble(part, norms, N, 0 if lc.algo == 'ppo' else 1, float(lc.entropy_coef), float(lc.vf_coef), out,
                    S=S, compat_value_bug=bool(lc.compat_value_bug))
    if fp.vtrace_stats is not None:
        st = fp.vtrace_stats.sum(0)
        out[12:15] = st[:3] / st[3].clamp_min(1.0)
    return out


def forward_logp_value(fp, units_t, env_t, act_t, msk_t, h0, c0, B: int, S: int,
                       reset_t: Optional[torch.Tensor] = None):
    """The policy's log-prob of the sampled actions and its value, per time-major row (row = t·B + b), at the weights
    in the flat buffer NOW (in stream order) — the forward half of :func:`fused_step_tm` on the same kernels and at
    the same precision (entity encoder [+ attention block] → forward chain → recurrence → heads GEMM → heads kernel),
    no backward. The learner's ``policy_old`` (reference optimizer.py:279, 474): once per iteration, before its
    minibatches, the iteration's experience is evaluated at the iteration's starting weights
    (learner/optimizer.py ``old_logp='learner'``). Returns (logp (N,) f32, value (N,) f32)."""
    C = fp.C
    cfg = fp.cfg
    exact = bool(getattr(fp, 'exact', False))
    lin = cfg.rnn != 'lstm'
    N = B * S
    U = units_t.shape[1]
    H = cfg.hidden
    dev = units_t.device
    W = fp.weight_images().refresh(C)
    P = dict(zip(fp.param_names, fp.params))
    w1, b1 = P['affine_unit_basic_stats.weight'].detach(), P['affine_unit_basic_stats.bias'].detach()
    we, be = P['affine_env.weight'].detach(), P['affine_env.bias'].detach()
    x896, emb, arg = C.encoder_fwd(units_t, env_t, w1, b1, W['wt16'], W['bt'], we, be, list(cfg.layout.counts),
                                   bool(cfg.compat_bugs), exact=exact)
    if cfg.entity_attention:
        E0p = emb.view(N * U, 128)
        if exact:
            nil = E0p.new_empty(0)
            wq, wo = (W['wq_x'], nil), (W['wo_x'], nil)
        else:
            wq, wo = W['wq_f'], W['wo_f']
        arg = torch.empty(N, 6, 128, dtype=torch.uint8, device=dev)
        out = C.attn_block_fwd(E0p, W['bout'], P['entity_attn.ln.weight'].detach(), P['entity_attn.ln.bias'].detach(),
                               wq[0], wq[1], P['entity_attn.qkv.bias'].detach(), wo[0], wo[1],
                               fp.type_offset_list(), x896, arg, bool(cfg.compat_bugs), 1e-5)
        emb = out[6].view(N, U, 128)
    elif cfg.compat_bugs:   # reference policy.py:127: enemy-tower pool = enemy-nonhero pool
        x896[:, 768:896] = x896[:, 512:640]
    if exact:
        nil = W['wpre16'].new_empty(0)
        x16, xp = C.pre_rnn_chain(x896, W['wpre16'], nil, W['bpre16'], W['wih16'], nil)
        hw = ((W['wcat256'], nil), W['bcat256'])
    else:
        x16, xp = C.pre_rnn_chain(x896, W['pre_s'][0], W['pre_s'][1], W['bpre16'], W['ih_s'][0], W['ih_s'][1])
        hw = (W['wcat_s'], W['bcat256'])
    if lin:
        hs = xp.add_(W['bias4']).view(S, B, H)
    else:
        rst = reset_t.reshape(S, B) if reset_t is not None else None
        hs = torch.empty(S, B, H, device=dev)
        o = team_fwd(C, xp.view(S, B, H, 4), W['whh16'], h0.contiguous(), c0.contiguous(), fp.err, False,
                     time_major=True, hs_out=hs, cs_out=torch.empty(S, B, H, device=dev),
                     gates_out=torch.empty(S, B, H, 4, device=dev), bias4=W['bias4'], reset=rst)
        hs = o[0]
    z = C.rowmm_out256(hs.reshape(N, H), hw[0][0], hw[0][1], hw[1])          # (N, 256): heads logits | value
    zero = fp.scratch('fwd_zero', (N,), torch.float32, dev)
    norms = fp.scratch('fwd_norms', (8,), torch.float32, dev)
    # the heads kernel's selected-action log-prob (its loss partials / gradients are not used here)
    _, _, _, lp = C.heads_loss(z, emb, act_t, msk_t, zero, zero, zero, zero, norms, 0, False, S, B, 0.1, 0.0, 0.0,
                               dz_bf16=False, precise=exact)
    return lp, z[:, 149].contiguous()
