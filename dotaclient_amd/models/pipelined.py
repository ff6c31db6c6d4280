"""Time-chunked, two-stream learner step: everything that is not the LSTM recurrence runs UNDER it.

With the XCD-team recurrence (ops/csrc/lstm_team.hip) a batch of 8 sequences occupies one XCD (32 of 256 CUs)
for the whole forward and backward recurrence — ≈8 ms of a ≈12 ms step — while every other stage (heads GEMMs and
the fused heads+loss kernel, the weight-gradient GEMMs, the pre-RNN backward, the entity-encoder backward) waits
for it. Those stages are all row-parallel, so the sequence is cut into ``C`` time chunks and software-pipelined:

    stream L (recurrence):  F0 F1 F2 F3 ............ B3 B2 B1 B0
    stream A (everything):     H0 H1 H2 H3            G3 G2 G1 G0

* ``F_c`` = team-LSTM forward over chunk c (carrying h, c between chunks); ``H_c`` = heads GEMM + heads/loss kernel
  + the heads backward GEMMs of chunk c (produces ∂L/∂h for chunk c) — overlapped with ``F_{c+1}``;
* ``B_c`` = team-LSTM backward over chunk c (carrying ∂h, ∂c backwards); ``G_c`` = all weight gradients that
  depend on chunk c's ∂gates (W_hh, W_ih, biases, pre-RNN, entity encoder incl. ∂W_τ) — overlapped with
  ``B_{c-1}``.

Measured: overlapping does not pay on MI355X today — GEMMs running on the other XCDs slow the L2-bound team
recurrence more than they save (10.25 / 10.6 / 11.0 ms per bench step at 1 / 2 / 4 chunks), so the default is one
chunk; what this Function buys in that setting is a step with NO work in the autograd backward, which is what makes
the whole forward+backward capturable in one hipGraph (Learner.enable_graph).

Rows are processed TIME-MAJOR (row = t·B + b) so a chunk is a contiguous slice of every activation; the inputs
are transposed once on entry. The loss and every gradient are computed in the Function's forward (for an upstream
gradient of 1); ``backward`` only scales them by the actual upstream gradient — the math is identical to
:class:`~dotaclient_amd.models.fused._PolicyLoss` up to summation order.
"""
from __future__ import annotations

from typing import Dict

import torch

from ..ops.lstm import team_bwd, team_fwd
from .policy import TYPE_SUFFIX

LDZ = 160


def _mm(a, b):
    return torch.mm(a, b, out_dtype=torch.float32)


def _bf(t):
    return t.detach().to(torch.bfloat16)


def _acc(a, b):
    """Accumulate a per-chunk gradient: the first chunk's tensor is used as is (no zero fill + add)."""
    return b if a is None else a.add_(b)


def chunk_bounds(S: int, chunks: int):
    c = max(1, min(chunks, S))
    edges = [round(i * S / c) for i in range(c + 1)]
    return [(edges[i], edges[i + 1]) for i in range(c) if edges[i + 1] > edges[i]]


class PipelinedPolicyLoss(torch.autograd.Function):
    @staticmethod
    def forward(ctx, fp, units, env, actions, masks, adv, ret, logp_old, nret, norms, h0, c0, *params):
        from .fused import tn_splitk
        C = fp.C
        cfg, lc = fp.cfg, fp.loss_cfg
        P = dict(zip(fp.param_names, params))
        B, S, U, _ = units.shape
        N = B * S
        H = cfg.hidden
        dev = units.device
        counts = list(cfg.layout.counts)
        main = torch.cuda.current_stream(dev)
        sL = fp.side_stream()
        tm = (lambda x: x.reshape(B, S, *x.shape[1:]).transpose(0, 1).reshape(N, *x.shape[1:]).contiguous())
        # ---- time-major inputs
        units_t = units.transpose(0, 1).reshape(N, U, 10).contiguous()
        env_t = env.transpose(0, 1).reshape(N, 3).contiguous()
        act_t, msk_t = tm(actions), tm(masks)
        adv_t, ret_t, lpo_t, nret_t = tm(adv), tm(ret), tm(logp_old), tm(nret)
        # ---- weights
        w1, b1 = P['affine_unit_basic_stats.weight'].detach(), P['affine_unit_basic_stats.bias'].detach()
        wt16 = torch.stack([_bf(P[f'affine_unit_{s}.weight']) for s in TYPE_SUFFIX])
        bt = torch.stack([P[f'affine_unit_{s}.bias'].detach() for s in TYPE_SUFFIX])
        we, be = P['affine_env.weight'].detach(), P['affine_env.bias'].detach()
        wpre16 = _bf(P['affine_pre_rnn.weight'])
        perm = fp.gate_perm(H, dev)
        wih16 = _bf(P['rnn.weight_ih_l0'])[perm].contiguous()
        whh16 = _bf(P['rnn.weight_hh_l0'])
        bias_p = (P['rnn.bias_ih_l0'].detach() + P['rnn.bias_hh_l0'].detach())[perm].contiguous()
        wcat, bcat = fp.head_cat(P)
        wcat16 = wcat.to(torch.bfloat16)
        # ---- encoder, pre-RNN, input projection over all rows (row-parallel, fast)
        x896, emb, arg = C.encoder_fwd(units_t, env_t, w1, b1, wt16, bt, we, be, counts, bool(cfg.compat_bugs))
        x = torch.relu(_mm(x896, wpre16.t()) + P['affine_pre_rnn.bias'].detach())
        x16 = x.to(torch.bfloat16)
        xp4 = _mm(x16, wih16.t()).view(S, B, H, 4)          # the recurrence kernel adds the bias (bias4)
        hs16 = torch.empty(S, B, H, dtype=torch.bfloat16, device=dev)
        cs = torch.empty(S, B, H, device=dev)
        gates4 = torch.empty(S, B, H, 4, device=dev)
        spans = chunk_bounds(S, fp.chunks)
        one = len(spans) == 1            # single chunk: outputs are used as produced (no staging copies)
        if not one:
            dxh = torch.empty(S, B, H, device=dev)
            z = torch.empty(N, LDZ, device=dev)
            dtl = torch.empty(N, U, device=dev)
            logp = torch.empty(N, device=dev)
        dWcat = dbcat = None
        parts = []
        algo = 0 if lc.algo == 'ppo' else 1
        # ---- forward recurrence on stream L, heads (+ heads backward) per chunk on the main stream
        ready = torch.cuda.Event()
        ready.record(main)
        sL.wait_event(ready)
        # every recurrence chunk is enqueued up front (the host must never hold the recurrence stream back while it
        # is busy launching the per-chunk work of the main stream)
        h_c, c_c = h0.contiguous(), c0.contiguous()
        fwd_done = []
        with torch.cuda.stream(sL):
            for t0, t1 in spans:
                o = team_fwd(C, xp4[t0:t1], whh16, h_c, c_c, fp.err, False, time_major=True,
                             hs_out=hs16[t0:t1], cs_out=cs[t0:t1], gates_out=gates4[t0:t1], bias4=bias_p)
                h_c, c_c = o[4], o[5]
                e = torch.cuda.Event()
                e.record(sL)
                fwd_done.append(e)
        for (t0, t1), done in zip(spans, fwd_done):
            main.wait_event(done)
            r0, r1 = t0 * B, t1 * B
            xh = hs16[t0:t1].view(-1, H)
            zc = _mm(xh, wcat16.t()) + bcat
            dz, dtl_c, part, lp = C.heads_loss(zc, emb[r0:r1], act_t[r0:r1], msk_t[r0:r1], adv_t[r0:r1],
                                               ret_t[r0:r1], lpo_t[r0:r1], nret_t[r0:r1], norms, algo, False,
                                               S, B, float(lc.clip_eps), float(lc.entropy_coef), float(lc.vf_coef))
            parts.append(part.sum(0))
            dz16 = dz.to(torch.bfloat16)
            dWcat = _acc(dWcat, _mm(dz16.t(), xh))
            dbcat = _acc(dbcat, dz.sum(0))
            if one:
                z, dtl, logp = zc, dtl_c, lp
                dxh = _mm(dz16, wcat16).view(S, B, H)
            else:
                z[r0:r1].copy_(zc)
                dtl[r0:r1].copy_(dtl_c)
                logp[r0:r1].copy_(lp)
                dxh[t0:t1].copy_(_mm(dz16, wcat16).view(t1 - t0, B, H))
        heads_done = torch.cuda.Event()
        heads_done.record(main)
        # ---- backward recurrence on stream L (reverse chunks), weight gradients per chunk on the main stream
        grads: Dict[str, torch.Tensor] = {}
        fp.split_head_grads(dWcat, dbcat, grads)
        dgates16 = torch.empty(S, B, H, 4, dtype=torch.bfloat16, device=dev)   # ∂gates straight from the kernel
        dWhh = dWih = db = dWpre = dbpre = dw1 = db1 = dWt = dbt = dWe = dbe = None
        wtT16 = wt16.transpose(1, 2).contiguous()
        seg = fp.type_segments(dev)
        h016 = h0.to(torch.bfloat16)
        sL.wait_event(heads_done)
        dh_n = dc_n = None
        bwd_done = []
        with torch.cuda.stream(sL):
            for t0, t1 in reversed(spans):
                cinit = c0.contiguous() if t0 == 0 else cs[t0 - 1]
                o = team_bwd(C, dxh[t0:t1], gates4[t0:t1], cs[t0:t1], cinit, dh_n, dc_n, whh16, fp.err,
                             time_major=True, dg_out=dgates16[t0:t1], dg_bf16=True, want_dbias=True)
                dh_n, dc_n = o[1], o[2]
                db = _acc(db, o[3])
                e = torch.cuda.Event()
                e.record(sL)
                bwd_done.append(e)
        for (t0, t1), done in zip(reversed(spans), bwd_done):
            main.wait_event(done)
            r0, r1 = t0 * B, t1 * B
            n = r1 - r0
            dG16 = dgates16[t0:t1].view(n, 4 * H)
            hprev = hs16[t0 - 1:t1 - 1].view(n, H) if t0 > 0 else torch.cat(
                [h016.unsqueeze(0), hs16[0:t1 - 1]], 0).view(n, H)
            dWhh = _acc(dWhh, _mm(dG16.t(), hprev))
            dWih = _acc(dWih, _mm(dG16.t(), x16[r0:r1]))
            dpre = _mm(dG16, wih16) * (x[r0:r1] > 0)
            dpre16 = dpre.to(torch.bfloat16)
            dWpre = _acc(dWpre, _mm(dpre16.t(), x896[r0:r1]))
            dbpre = _acc(dbpre, dpre.sum(0))
            dx896 = _mm(dpre16, wpre16)
            q = z[r0:r1, :128]
            dwt_c, dw1_c, db1_c = C.encoder_bwd(units_t[r0:r1], w1, b1, wtT16, dtl[r0:r1], z[r0:r1],
                                                      dx896, arg[r0:r1], counts, bool(cfg.compat_bugs))
            dw1 = _acc(dw1, dw1_c)
            db1 = _acc(db1, db1_c)
            dbt = _acc(dbt, tn_splitk((dtl[r0:r1] @ seg).contiguous(), q.contiguous())
                       + dx896[:, 128:].reshape(n, 6, 128).sum(0))
            dWt = _acc(dWt, dwt_c)
            env_c = env_t[r0:r1]
            de = dx896[:, :128] * ((env_c @ we.t() + be) > 0)
            dWe = _acc(dWe, de.t() @ env_c)
            dbe = _acc(dbe, de.sum(0))
        inv = fp.gate_inv(H, dev)
        grads['rnn.weight_hh_l0'] = dWhh[inv]
        grads['rnn.weight_ih_l0'] = dWih[inv]
        grads['rnn.bias_ih_l0'] = db[inv]
        grads['rnn.bias_hh_l0'] = grads['rnn.bias_ih_l0']
        grads['affine_pre_rnn.weight'] = dWpre
        grads['affine_pre_rnn.bias'] = dbpre
        grads['affine_unit_basic_stats.weight'] = dw1
        grads['affine_unit_basic_stats.bias'] = db1
        for t, s in enumerate(TYPE_SUFFIX):
            grads[f'affine_unit_{s}.weight'] = dWt[t]
            grads[f'affine_unit_{s}.bias'] = dbt[t]
        grads['affine_env.weight'] = dWe
        grads['affine_env.bias'] = dbe
        ctx.grads = [grads.get(nm) for nm in fp.param_names]
        ctx.fp = fp
        # logp back to batch-major (B·S) row order
        logp_b = logp.view(S, B).t().reshape(N)
        ctx.mark_non_differentiable(logp_b)
        return torch.stack(parts).sum(0), logp_b

    @staticmethod
    def backward(ctx, gpart, _glogp):
        ctx.fp.apply_direct_grads(ctx.grads, gpart[15])
        ctx.grads = None
        return (None,) * (12 + len(ctx.fp.param_names))
