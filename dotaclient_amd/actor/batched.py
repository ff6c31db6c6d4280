"""GPU-resident batched actor inference: one hipGraph replay steps thousands of players at once.

The reference actor runs one player per process on the CPU: featurize → ``policy.single`` → ``select_actions`` →
``action_to_pb`` every 200 ms of game time (agent.py:641-660, policy.py:171-283). Here the per-player state (LSTM
h/c) lives on the GPU in fixed slots and one step of *all* slots is a captured graph:

    H2D(env, units, handles, keep)           pinned → static device buffers (one copy each)
    encoder_fwd                              fused entity encoder kernel (shared with the learner)
    [5v5: attn_block_fwd                     LayerNorm + QKV + attention + out-projection + pools, one kernel]
    actor_core                               ONE kernel (ops/csrc/actor_core.hip): episode resets (h, c *= keep),
                                             relu(x896·W_preᵀ + b), gates = [x | h]·[W_ih | W_hh]ᵀ + b + LSTM cell
                                             (or the fake_rnn Linear), z = h·W_headsᵀ + b for all 5 heads
    sample_actions                           fused masked log-softmax + Gumbel-max + hierarchical selection
    D2H(idx, logp, value[, act, msk])

No vendor GEMM in any actor step: bf16 operands (:class:`GpuActorPolicy`, the default), IEEE fp32 on the f32 MFMA
(:class:`F32ActorPolicy` — the reference actor's precision, agent.py:641-660 → policy.py:80-84) or e4m3
(:class:`Fp8ActorPolicy`).

so the host only featurizes (native C++, :mod:`dotaclient_amd.native`) and turns indices into protobuf actions.
Sampling uses a counter-based hash RNG (seed, step counter, row, head, entry) kept in device memory, so replays
draw fresh noise without re-capture.
"""
from __future__ import annotations

import os
import time
from typing import Dict, Optional

import numpy as np
import torch

from ..models.policy import TYPE_SUFFIX, Policy

LDZ = 160


class _Pack:
    """Named regions of ONE pinned host buffer and ONE device buffer with the same byte layout (256-B aligned
    regions in declaration order), so any contiguous run of regions moves in a single copy."""

    def __init__(self, fields, device):
        self.off, self.size, off = {}, {}, 0
        for name, shape, dt in fields:
            nb = int(np.prod(shape)) * torch.empty((), dtype=dt).element_size()
            self.off[name], self.size[name] = off, nb
            off = (off + nb + 255) // 256 * 256
        self.host_bytes = torch.zeros(off, dtype=torch.uint8, pin_memory=True)
        self.dev_bytes = torch.zeros(off, dtype=torch.uint8, device=device)
        self.host, self.dev = {}, {}
        for name, shape, dt in fields:
            o, nb = self.off[name], self.size[name]
            self.host[name] = self.host_bytes[o:o + nb].view(dt).view(shape)
            self.dev[name] = self.dev_bytes[o:o + nb].view(dt).view(shape)

    def copy_range(self, first: str, last: str, to_host: bool = False):
        a, b = self.off[first], self.off[last] + self.size[last]
        if to_host:
            self.host_bytes[a:b].copy_(self.dev_bytes[a:b], non_blocking=True)
        else:
            self.dev_bytes[a:b].copy_(self.host_bytes[a:b], non_blocking=True)


def frag_weight(w: torch.Tensor, mode: int) -> torch.Tensor:
    """(N, K) fp32 weight → the MFMA fragment order of ops/csrc/actor_core.hip: mode 0 (fp32) [N/16][K/16][lane][4]
    with element j of lane l = w[16·t + (l & 15)][16·g + 4·(l >> 4) + j]; mode 1 (bf16) [N/16][K/32][lane][8] with
    w[16·t + (l & 15)][32·g + 8·(l >> 4) + j]. One wave's k-group load is 1 KB contiguous."""
    N, K = w.shape
    kg, e = (16, 4) if mode == 0 else (32, 8)
    if N % 16 or K % kg:
        raise ValueError(f'frag_weight: ({N}, {K}) must be multiples of (16, {kg})')
    src = w.float() if mode == 0 else w.to(torch.bfloat16)
    return src.reshape(N // 16, 16, K // kg, 4, e).permute(0, 2, 3, 1, 4).contiguous().view(-1)


class GpuActorPolicy:
    """Fixed-slot batched policy step on one GPU: LSTM / linear-RNN policies, 1v1 or 5v5 (entity attention), bf16
    operands on hand-written MFMA kernels (``CORE_MODE`` 1; :class:`F32ActorPolicy` is the IEEE-fp32 twin)."""

    CORE_MODE = 1        # ops/csrc/actor_core.hip: 0 = IEEE fp32 (f32 MFMA), 1 = bf16 operands

    def __init__(self, policy: Policy, n_slots: int, device='cuda', seed: int = 0, use_graph: bool = True,
                 record: bool = True, inputs_from: Optional['GpuActorPolicy'] = None, raw: bool = False):
        from .. import ops
        self.C = ops.require()
        # raw: observations staged as compact raw unit records (features/raw.py, 32 B per unit slot + a 16 B hero
        # record per slot instead of 40 B of features + an 8 B handle) and featurized by the step's first kernel
        # (ops/csrc/featurize.hip); the host's native engine then skips the per-unit feature arithmetic
        self.raw = bool(raw)
        cfg = policy.config
        if cfg.unit_dim != 128 or cfg.env_dim != 128:
            raise ValueError('GpuActorPolicy needs 128-wide unit / env embeddings (the fused encoder kernel)')
        if cfg.entity_attention and (cfg.layout.max_units != 64 or cfg.attention_heads != 4):
            raise ValueError('GpuActorPolicy: the attention kernels cover 64 unit slots × 4 heads (the 5v5 preset)')
        self.cfg = cfg
        self.device = torch.device(device)
        self.n = n_slots
        self.U = cfg.layout.max_units
        self.A = 21 + self.U
        self.seed = int(seed)
        self.use_graph = use_graph
        self.record = record
        self.policy = policy
        import itertools
        self.toff = [0] + list(itertools.accumulate(cfg.layout.counts))     # first slot of each unit type
        self._alloc(inputs_from)
        self.load_weights(policy)
        self.graph: Optional[torch.cuda.CUDAGraph] = None

    # ------------------------------------------------------------------------------------------------
    # staged input dtypes (Fp8ActorPolicy stages compact fp16 features / int32 handles); words per staged raw record
    # (Fp8ActorPolicy: the 16-byte form, features/raw.py pack_raw16)
    UNITS_DTYPE, HANDLES_DTYPE = torch.float32, torch.long
    RAW_WORDS = 8

    def _alloc(self, inputs_from=None):
        if self.raw:
            self._alloc_raw(inputs_from)
        else:
            self._alloc_features(inputs_from)
        self.h_keep, self.h_active = self.in_pack.host['keep'], self.in_pack.host['active']
        self.h_keep.fill_(1.0)
        self.h_active.fill_(1.0)
        self.d_env = self.in_pack.dev['env']
        self.d_keep = self.in_pack.dev['keep']
        self.d_active = self.in_pack.dev['active']     # 0 → slot not stepped: LSTM state left untouched
        self._alloc_state()

    def _alloc_raw(self, inputs_from):
        n, U, dev = self.n, self.U, self.device
        self.in_pack = _Pack([('env', (n, 3), torch.float32), ('hero', (n, 4), torch.float32),
                              ('raw', (n, U, self.RAW_WORDS), torch.int32), ('keep', (n, 1), torch.float32),
                              ('active', (n,), torch.float32)], dev)
        if inputs_from is not None:
            if (inputs_from.n, inputs_from.U) != (n, U) or not inputs_from.raw:
                raise ValueError('inputs_from: slot count / layout / staging mismatch')
            self.h_env, self.h_hero, self.h_raw = inputs_from.h_env, inputs_from.h_hero, inputs_from.h_raw
        else:
            self.h_env, self.h_hero, self.h_raw = (self.in_pack.host[k] for k in ('env', 'hero', 'raw'))
        self._shared_inputs = inputs_from is not None
        self.h_units = self.h_handles = None
        self.d_hero, self.d_raw = self.in_pack.dev['hero'], self.in_pack.dev['raw']
        # the featurize kernel's outputs: device-only, in the dtypes the step's kernels read
        self.d_units = torch.zeros(n, U, 10, dtype=self.UNITS_DTYPE, device=dev)
        self.d_handles = torch.full((n, U), -1, dtype=self.HANDLES_DTYPE, device=dev)

    def _alloc_features(self, inputs_from):
        n, U, dev = self.n, self.U, self.device
        ud, hd = self.UNITS_DTYPE, self.HANDLES_DTYPE
        # ONE packed pinned staging buffer and ONE device mirror per direction: a step's inputs cross PCIe in one copy
        # and its outputs come back in one (each separate copy was a DMA dispatch of its own inside the graph)
        self.in_pack = _Pack([('env', (n, 3), torch.float32), ('units', (n, U, 10), ud), ('handles', (n, U), hd),
                              ('keep', (n, 1), torch.float32), ('active', (n,), torch.float32)], dev)
        if inputs_from is not None:
            # a second policy over the same observations (league opponents): share the staged inputs; keep/active
            # stay per policy (its own pack's env / units / handles regions are unused)
            if (inputs_from.n, inputs_from.U) != (n, U):
                raise ValueError('inputs_from: slot count / layout mismatch')
            self.h_env, self.h_units, self.h_handles = inputs_from.h_env, inputs_from.h_units, inputs_from.h_handles
        else:
            self.h_env, self.h_units, self.h_handles = (self.in_pack.host[k] for k in ('env', 'units', 'handles'))
            self.h_handles.fill_(-1)
        self._shared_inputs = inputs_from is not None
        # the kernels read the staged dtypes as they are (fp8 step: fp16 features, int32 handles)
        self.d_units = self.in_pack.dev['units']
        self.d_handles = self.in_pack.dev['handles']

    def _alloc_state(self):
        n, A, dev = self.n, self.A, self.device
        H = self.cfg.hidden
        pin = dict(pin_memory=True)
        self.h = torch.zeros(n, H, device=dev)
        self.c = torch.zeros(n, H, device=dev)
        self.z = torch.zeros(n, LDZ, device=dev)                 # head logits [q | enum | x | y | value | pad]
        self.ctr = torch.zeros(1, dtype=torch.long, device=dev)
        # outputs: [idx | logp | value] first (the part every step returns), then [act | msk] (recorded steps)
        self.out_pack = _Pack([('idx', (n, 4), torch.int32), ('logp', (n,), torch.float32),
                               ('value', (n,), torch.float32), ('act', (n, A), torch.uint8),
                               ('msk', (n, A), torch.uint8)], dev)
        d, o = self.out_pack.dev, self.out_pack.host
        self.idx, self.logp, self.value, self.act, self.msk = d['idx'], d['logp'], d['value'], d['act'], d['msk']
        self.o_idx, self.o_logp, self.o_value, self.o_act, self.o_msk = (o['idx'], o['logp'], o['value'], o['act'],
                                                                         o['msk'])
        # LSTM state snapshots (h, c before the step, after resets) of selected rows — trajectory hidden states
        self.h_rows = torch.zeros(n, dtype=torch.long, **pin)
        self.d_rows = torch.zeros(n, dtype=torch.long, device=dev)
        self.d_snap = torch.zeros(n, 2, H, device=dev)
        self.o_snap = torch.zeros(n, 2, H, **pin)
        self._snap_n = 0
        # the actor's step stream at the DEFAULT priority. (High priority, round 4: +2-3 % in the then actor-bound node
        # loop; round 5: no difference in the GPU-bound loop, scripts/gpu_r5_ff.sh — and with a league's opponent
        # policies adding more high-priority work beside the learner's persistent recurrence, the recurrence stalled
        # for seconds: profiles/r5_replay_timeout.md, scripts/gpu_r5_bisect.sh.)
        self.stream = torch.cuda.Stream(device=dev)

    @torch.no_grad()
    def load_weights(self, policy_or_state):
        """(Re)load weights in place — buffers keep their addresses, so a captured graph stays valid. The copies
        run on the step stream, so they are ordered after the previous replay and before the next one."""
        if hasattr(self, 'stream'):
            with torch.cuda.stream(self.stream):
                return self._load_weights(policy_or_state)
        return self._load_weights(policy_or_state)

    @torch.no_grad()
    def weight_dict(self, policy_or_state):
        """(operand set, ready event): the kernels' operands of these weights (casts, fragment images, fp8
        quantisation), built on the step stream — for :meth:`load_weight_dict` of other policies of the same shape
        (one build per weight version instead of one per policy)."""
        sd = policy_or_state.state_dict() if isinstance(policy_or_state, torch.nn.Module) else policy_or_state
        with torch.cuda.stream(self.stream):
            w = self._weight_dict(sd)
            ev = torch.cuda.Event()
            ev.record(self.stream)
        return w, ev

    @torch.no_grad()
    def load_weight_dict(self, w: Dict[str, torch.Tensor], ready: Optional[torch.cuda.Event] = None,
                         producer: Optional[torch.cuda.Stream] = None):
        """Copy a :meth:`weight_dict` operand set (built on ``producer``, complete at ``ready``) into this policy's
        buffers, ordered on its step stream."""
        other = producer is not None and producer != self.stream
        with torch.cuda.stream(self.stream):
            if ready is not None:
                self.stream.wait_event(ready)
            for k, v in w.items():
                if isinstance(v, torch.Tensor):
                    if other:
                        v.record_stream(self.stream)   # the producer's allocator must not reuse it before this copy
                    self.w[k].copy_(v)

    def _load_weights(self, policy_or_state):
        sd = policy_or_state.state_dict() if isinstance(policy_or_state, torch.nn.Module) else policy_or_state
        w = self._weight_dict(sd)
        if not hasattr(self, 'w'):
            self.w = w
        else:
            for k, v in w.items():
                if isinstance(v, torch.Tensor):
                    self.w[k].copy_(v)

    def _weight_dict(self, sd) -> Dict[str, torch.Tensor]:
        dev, mode, cfg = self.device, self.CORE_MODE, self.cfg
        g = (lambda k: sd[k].detach().to(dev, torch.float32))
        bf = (lambda k: sd[k].detach().to(dev, torch.bfloat16))
        attn32 = cfg.entity_attention or mode == 0       # fp32 encoder output (bf16x3 / exact encoder variants)
        wt = torch.stack([g(f'affine_unit_{s}.weight') for s in TYPE_SUFFIX]).contiguous()
        w = {
            'w1': g('affine_unit_basic_stats.weight').contiguous(), 'b1': g('affine_unit_basic_stats.bias'),
            # (entity attention: the encoder adds b_τ + b_out — the residual's bias folded into E0, as the learner)
            'wt': wt if attn32 else wt.to(torch.bfloat16),
            'bt': torch.stack([g(f'affine_unit_{s}.bias') for s in TYPE_SUFFIX]).contiguous(),
            'we': g('affine_env.weight').contiguous(), 'be': g('affine_env.bias'),
            'cpre': frag_weight(g('affine_pre_rnn.weight'), mode), 'bpre': g('affine_pre_rnn.bias').contiguous(),
        }
        if cfg.entity_attention:
            from ..models.pipelined import _frag_order
            w['bt'] = (w['bt'] + g('entity_attn.out.bias')[None]).contiguous()
            w['bout'] = g('entity_attn.out.bias').contiguous()
            w['ln_g'] = g('entity_attn.ln.weight').contiguous()
            w['ln_b'] = g('entity_attn.ln.bias').contiguous()
            w['bqkv'] = g('entity_attn.qkv.bias').contiguous()
            # W_qkv / W_out in MFMA fragment order (ops/csrc/attn_block.hip, as the learner): hi / lo bf16 images
            # (bf16x3 block), or — the IEEE-fp32 actor, mode 0 — the fp32 image and an empty lo (the exact block
            # kernel attn_block_fwd_f32_kernel<true>, the fp32-exact learner's forward)
            for key, name in (('wq', 'entity_attn.qkv.weight'), ('wo', 'entity_attn.out.weight')):
                if mode == 0:
                    w[key + '_h'], w[key + '_l'] = _frag_order(g(name).contiguous()), g(name).new_empty(0)
                else:
                    hi, lo = self.C.split_bf16x2(g(name).contiguous())
                    w[key + '_h'], w[key + '_l'] = _frag_order(hi), _frag_order(lo)
        H = cfg.hidden
        if cfg.rnn == 'lstm':
            from ..ops.lstm import gate_perm
            perm = gate_perm(H, dev)                   # unit-major gate rows: a unit's i, f, g, o in 4 columns
            wcat = torch.cat([g('rnn.weight_ih_l0'), g('rnn.weight_hh_l0')], 1)[perm]
            w['cg'] = frag_weight(wcat.contiguous(), mode)
            w['bg'] = (g('rnn.bias_ih_l0') + g('rnn.bias_hh_l0'))[perm].contiguous()
        else:
            w['cg'] = frag_weight(g('fake_rnn.weight'), mode)
            w['bg'] = g('fake_rnn.bias').contiguous()
        heads = ['affine_unit_attention', 'affine_head_enum', 'affine_move_x', 'affine_move_y', 'affine_value']
        wh = torch.cat([g(f'{k}.weight') for k in heads] + [torch.zeros(LDZ - 150, H, device=dev)], 0)
        bh = torch.cat([g(f'{k}.bias') for k in heads] + [torch.zeros(LDZ - 150, device=dev)], 0)
        w['ch'] = frag_weight(wh, mode)
        w['bh'] = bh.contiguous()
        w['wh32'] = wh.contiguous()
        return w

    # ------------------------------------------------------------------------------------------------
    def _forward(self):
        """The captured body: reads d_* / h / c, writes idx/act/msk/logp/value and the new h / c.

        3 launches (5v5: 4), none a vendor GEMM: encoder kernel [→ attention block] → ``actor_core`` (episode
        resets, pre-RNN layer, gates + LSTM cell or the linear layer, heads; bumps the sampler's RNG counter) →
        sampling kernel."""
        C, w, cfg = self.C, self.w, self.cfg
        if self.raw:
            C.featurize_raw(self.d_raw, self.d_hero, self.d_units, self.d_handles)
        x896, emb, arg = C.encoder_fwd(self.d_units, self.d_env, w['w1'], w['b1'], w['wt'], w['bt'], w['we'],
                                       w['be'], list(cfg.layout.counts), bool(cfg.compat_bugs),
                                       exact=self.CORE_MODE == 0)
        if cfg.entity_attention:
            # 5v5 pre-LN self-attention over the 64 unit slots + pools of the attended embeddings, ONE kernel
            # (ops/csrc/attn_block.hip, the learner's forward); E1 is the pointer head's unit embedding
            out = C.attn_block_fwd(emb.view(self.n * self.U, 128), w['bout'], w['ln_g'], w['ln_b'], w['wq_h'],
                                   w['wq_l'], w['bqkv'], w['wo_h'], w['wo_l'], self.toff, x896, arg,
                                   bool(cfg.compat_bugs), 1e-5)
            emb = out[6].view(self.n, self.U, 128)
        elif cfg.compat_bugs:
            x896[:, 768:896] = x896[:, 512:640]
        C.actor_core(x896, w['cpre'], w['bpre'], w['cg'], w['bg'], w['ch'], w['bh'], self.h, self.c,
                     self.d_keep.view(-1), self.z, self.CORE_MODE, cfg.rnn != 'lstm', active=self.d_active,
                     bump=self.ctr)
        C.sample_actions(self.z, emb, self.d_handles, self.seed, self.ctr, self.idx, self.act, self.msk, self.logp,
                         self.value)

    def _h2d(self):
        if self._shared_inputs:
            # observations staged by the policy this one shares them with: its pinned views, our device regions
            ip = self.in_pack.dev
            ip['env'].copy_(self.h_env, non_blocking=True)
            if self.raw:
                ip['hero'].copy_(self.h_hero, non_blocking=True)
                ip['raw'].copy_(self.h_raw, non_blocking=True)
            else:
                ip['units'].copy_(self.h_units, non_blocking=True)
                ip['handles'].copy_(self.h_handles, non_blocking=True)
            self.in_pack.copy_range('keep', 'active')
        else:
            self.in_pack.copy_range('env', 'active')          # one H2D copy of the whole staged step

    def _d2h(self):
        self.out_pack.copy_range('idx', 'msk' if self.record else 'value', to_host=True)

    # The step's input / output copies run OUTSIDE the captured graph, as plain async copies on the step stream: from
    # pinned memory those go to the SDMA copy engines. Captured, they became blit kernels (__amd_rocclr_copyBuffer) on
    # the shader cores — 155 µs of CU time per 4 096-slot step, 36-58 % of the actor step, running beside the
    # learner's latency-bound recurrence in the node loop (profiles/r5_actor_*_summary.md). DCA_ACTOR_GRAPH_COPIES=1
    # captures them again (A/B).
    GRAPH_COPIES = os.environ.get('DCA_ACTOR_GRAPH_COPIES', '0') == '1'

    def capture(self):
        """Warm up (allocator) on a side stream and capture the policy step in one hipGraph: a step is one launch
        (plus the two SDMA copies around it, or — ``GRAPH_COPIES`` — with the copies inside the graph)."""
        s = self.stream
        s.wait_stream(torch.cuda.current_stream(self.device))
        ctr0 = self.ctr.clone()
        with torch.cuda.stream(s):
            for _ in range(3):
                self._h2d()
                self._forward()
                self._d2h()
        torch.cuda.current_stream(self.device).wait_stream(s)
        g = torch.cuda.CUDAGraph()
        with torch.cuda.graph(g, stream=s, capture_error_mode='thread_local'):
            if self.GRAPH_COPIES:
                self._h2d()
            self._forward()
            if self.GRAPH_COPIES:
                self._d2h()
        torch.cuda.synchronize(self.device)
        # warm-up steps advanced the recurrent state and the RNG counter: start from a clean slate
        self.ctr.copy_(ctr0)
        self.h.zero_(); self.c.zero_()
        self.graph = g

    # ------------------------------------------------------------------------------------------------
    def _snapshot(self, rows: np.ndarray):
        """Gather the selected rows' (h, c) as they ENTER this step (before its resets, which the host applies from
        the staged keep flags in :meth:`wait`), on the step stream ahead of the step."""
        k = len(rows)
        self.h_rows.numpy()[:k] = rows
        self._snap_keep = self.h_keep.numpy()[rows, 0].copy()
        d = self.d_rows[:k]
        d.copy_(self.h_rows[:k], non_blocking=True)
        torch.index_select(self.h, 0, d, out=self.d_snap[:k, 0])
        torch.index_select(self.c, 0, d, out=self.d_snap[:k, 1])
        self.o_snap[:k].copy_(self.d_snap[:k], non_blocking=True)
        self._snap_n = k

    def step_async(self, snapshot_rows: Optional[np.ndarray] = None):
        """Launch one step for all slots using the host staging buffers; call :meth:`wait` for the outputs.
        ``snapshot_rows``: slots whose LSTM state *entering* this step (after resets) :meth:`wait` returns as
        ``out['hidden']`` (k, 2, H) — the trajectory's stored states (codec ``hiddens``)."""
        if self.use_graph and self.graph is None:
            self.capture()
        with torch.cuda.stream(self.stream):
            self._snap_n = 0
            if snapshot_rows is not None and len(snapshot_rows) and self.cfg.rnn == 'lstm':
                self._snapshot(np.asarray(snapshot_rows))
            if self.graph is not None:
                if not self.GRAPH_COPIES:
                    self._h2d()
                self.graph.replay()
                if not self.GRAPH_COPIES:
                    self._d2h()
            else:
                self._h2d()
                self._forward()
                self._d2h()
            self._done = torch.cuda.Event()
            self._done.record(self.stream)

    def wait(self) -> Dict[str, np.ndarray]:
        self._done.synchronize()
        self.h_keep.fill_(1.0)
        out = {'idx': self.o_idx.numpy(), 'logp': self.o_logp.numpy(), 'value': self.o_value.numpy()}
        if self.record:
            out['actions'] = self.o_act.numpy()
            out['masks'] = self.o_msk.numpy()
        if self._snap_n:
            hid = self.o_snap.numpy()[:self._snap_n]
            hid *= self._snap_keep[:, None, None]        # resets of this step (keep = 0) → zero state
            out['hidden'] = hid
        return out

    def step(self, env: np.ndarray, units: np.ndarray, handles: np.ndarray, reset: Optional[np.ndarray] = None,
             active: Optional[np.ndarray] = None):
        """Synchronous step: (n,3), (n,U,10), (n,U) arrays for all slots; ``reset`` (n,) bool zeroes h/c first;
        ``active`` (n,) bool: only these slots advance their LSTM state (outputs of the others are don't-care)."""
        self.stage(env, units, handles)
        if reset is not None:
            self.h_keep.numpy()[:, 0] = 1.0 - np.asarray(reset, dtype=np.float32)
        self.h_active.numpy()[:] = 1.0 if active is None else np.asarray(active, dtype=np.float32)
        self.step_async()
        return self.wait()

    def step_raw(self, env: np.ndarray, hero: np.ndarray, raw: np.ndarray, reset: Optional[np.ndarray] = None,
                 active: Optional[np.ndarray] = None):
        """:meth:`step` from raw unit records (a ``raw=True`` policy): (n,3) env, (n,4) hero, (n,U,8) int32 raw."""
        self.stage_raw(env, hero, raw)
        if reset is not None:
            self.h_keep.numpy()[:, 0] = 1.0 - np.asarray(reset, dtype=np.float32)
        self.h_active.numpy()[:] = 1.0 if active is None else np.asarray(active, dtype=np.float32)
        self.step_async()
        return self.wait()

    def stage(self, env: np.ndarray, units: np.ndarray, handles: np.ndarray):
        """Copy (n,3), (n,U,10), (n,U) host arrays into the pinned staging buffers (torch's vectorised casts: the
        fp8 step stages fp16 / int32, and numpy's fp32→fp16 cast is several times slower)."""
        if self.raw:
            raise RuntimeError('stage: this policy stages raw unit records (stage_raw)')
        self.h_env.copy_(torch.from_numpy(np.ascontiguousarray(env)))
        self.h_units.copy_(torch.from_numpy(np.ascontiguousarray(units)))
        self.h_handles.copy_(torch.from_numpy(np.ascontiguousarray(handles)))

    def stage_raw(self, env: np.ndarray, hero: np.ndarray, raw: np.ndarray):
        """Copy (n,3) env, (n,4) hero and (n,U,8) int32 raw unit records (features/raw.py) into the staging buffers
        (a 16-byte-record policy also takes (n,U,4) records as they are)."""
        if not self.raw:
            raise RuntimeError('stage_raw: this policy stages features (stage)')
        if self.RAW_WORDS == 4 and raw.shape[-1] == 8:
            from ..features.raw import pack_raw16
            raw = pack_raw16(raw)
        self.h_env.copy_(torch.from_numpy(np.ascontiguousarray(env)))
        self.h_hero.copy_(torch.from_numpy(np.ascontiguousarray(hero)))
        self.h_raw.copy_(torch.from_numpy(np.ascontiguousarray(raw)))

    def hidden(self):
        return self.h, self.c


class F32ActorPolicy(GpuActorPolicy):
    """:class:`GpuActorPolicy` at the reference actor's precision (agent.py:641-660 → policy.py:80-84, torch fp32):
    the IEEE-fp32 entity encoder (``encoder_fwd`` exact: the learner's ``encoder_fwd_x_kernel``), for the 5v5 policy
    the IEEE-fp32 attention block (``attn_block_fwd`` with fp32 fragment images: the fp32-exact learner's block
    forward), and the fp32 ``actor_core`` (every product an fp32 FMA on ``v_mfma_f32_16x16x4_f32``), fp32 unit
    embeddings into the sampler. LSTM-128 / LSTM-512 / 5v5, or the compat linear layer."""

    CORE_MODE = 0




def fp8_weight(w: torch.Tensor):
    """(N, K) fp32 weight → (e4m3fn bytes in MFMA fragment order, (N,) fp32 per-channel dequant scales) for
    ops/csrc/actor_fp8.hip: each output channel's max |w| maps to 448 (the largest finite e4m3fn); byte order
    [N/16 column tile][K/128 k-step][lane = 16·(k%128 // 32) + n%16][k % 32] — the 32-byte operand of a lane of the
    16x16x128 f8f6f4 MFMA; one tile's k-step is one coalesced 2 KB load of a wave."""
    N, K = w.shape
    if N % 16 or K % 128:
        raise ValueError(f'fp8_weight: ({N}, {K}) must be multiples of (16, 128)')
    amax = w.abs().amax(1)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    q = (w / s[:, None]).clamp(-448.0, 448.0).to(torch.float8_e4m3fn).view(torch.uint8)
    frag = q.view(N // 16, 16, K // 128, 4, 32).permute(0, 2, 3, 1, 4).contiguous()
    return frag.view(-1), s.float().contiguous()


class Fp8ActorPolicy(GpuActorPolicy):
    """:class:`GpuActorPolicy` with the policy's GEMMs on hand-written e4m3 MFMA kernels (ops/csrc/actor_fp8.hip;
    BASELINE config 5, fp8 actor inference): the entity encoder's unit-type GEMMs (``encoder_fp8``, one 16x16x128
    f8f6f4 MFMA per output tile) and, in one more launch, the pre-RNN layer, the LSTM step and the heads
    (``actor_fp8``). Weights are quantised per output channel at (hot-)load time, activations per row (per (row, unit)
    in the encoder) inside the kernels. The sampling kernel is shared with the bf16 step.

    Compact staging: unit features cross PCIe as fp16 and unit handles as int32 (3.3 + 0.7 MB per 4096-slot step
    instead of 6.6 + 1.3 MB — the copies were 57 % of the bf16 step), read by the kernels as they are (the encoder
    converts the fp16 features in LDS, the sampler tests int32 handles).
    The host-side buffers keep the :class:`GpuActorPolicy` API (``h_units`` / ``h_handles`` numpy views assign with
    a cast). ``compact=False`` keeps fp32 / int64 host buffers. ``raw=True`` (VecActor's default): 16-byte raw unit
    records — position, height, facing and the health ratio as binary16, flags, handle; 16 B per unit slot against
    32 B for the fp32 / bf16 steps' records — featurized to fp16 by the step's first kernel (``featurize_raw16_kernel``);
    the engine keeps the full records for the learner.
    1v1 LSTM policies with hidden 512 / pre-RNN 256 (the kernel's shape)."""

    def __init__(self, policy: Policy, n_slots: int, device='cuda', compact: bool = True, **kw):
        cfg = policy.config
        if cfg.rnn != 'lstm' or cfg.hidden != 512 or cfg.pre_rnn_dim != 256 or cfg.entity_attention:
            raise ValueError('Fp8ActorPolicy: 1v1 LSTM policy with hidden 512, pre-RNN 256')
        self.compact = bool(compact)
        super().__init__(policy, n_slots, device=device, **kw)

    RAW_WORDS = 4            # raw staging: the 16-byte records (binary16 fields; the step's features are fp16)

    def _alloc(self, inputs_from=None):
        if self.compact or self.raw:
            self.UNITS_DTYPE, self.HANDLES_DTYPE = torch.float16, torch.int32
        super()._alloc(inputs_from)
        if inputs_from is not None and not self.raw and inputs_from.h_units.dtype != self.UNITS_DTYPE:
            raise ValueError('Fp8ActorPolicy: inputs_from must stage the same feature dtype')

    def _weight_dict(self, sd):
        w = super()._weight_dict(sd)
        dev = self.device
        g = (lambda k: sd[k].detach().to(dev, torch.float32))
        from ..ops.lstm import gate_perm
        perm = gate_perm(self.cfg.hidden, dev)
        w['wpre8'], w['spre'] = fp8_weight(g('affine_pre_rnn.weight'))
        w['bpre32'] = g('affine_pre_rnn.bias').contiguous()
        wcat = torch.cat([g('rnn.weight_ih_l0'), g('rnn.weight_hh_l0')], 1)[perm]
        w['wg8'], w['sg'] = fp8_weight(wcat.contiguous())
        w['bg'] = (g('rnn.bias_ih_l0') + g('rnn.bias_hh_l0'))[perm].contiguous()
        w['wh8'], w['sh8'] = fp8_weight(w['wh32'])
        # the encoder's six unit-type weights (128 out × 128 in each), per-channel e4m3 in fragment order
        wt = [fp8_weight(g(f'affine_unit_{s}.weight')) for s in TYPE_SUFFIX]
        w['wt8'] = torch.cat([q for q, _ in wt]).contiguous()
        w['st8'] = torch.stack([s_ for _, s_ in wt]).contiguous()
        for k in ('cpre', 'cg', 'ch', 'wt'):       # the bf16 core's operands are not used here
            w.pop(k, None)
        return w

    def _forward(self):
        """Captured body, 3 launches: fp8 encoder → fp8 core (pre-RNN, gates + cell, heads; bumps the sampler's RNG
        counter) → sampling."""
        C, w, cfg = self.C, self.w, self.cfg
        if self.raw:
            C.featurize_raw(self.d_raw, self.d_hero, self.d_units, self.d_handles)
        x896, emb = C.encoder_fp8(self.d_units, self.d_env, w['w1'], w['b1'], w['wt8'], w['st8'], w['bt'], w['we'],
                                  w['be'], list(cfg.layout.counts))
        if cfg.compat_bugs:
            x896[:, 768:896] = x896[:, 512:640]
        C.actor_fp8(x896, w['wpre8'], w['spre'], w['bpre32'], w['wg8'], w['sg'], w['bg'], w['wh8'], w['sh8'],
                    w['bh'], self.h, self.c, self.d_keep.view(-1), self.z, self.d_active, self.ctr)
        C.sample_actions(self.z, emb, self.d_handles, self.seed, self.ctr, self.idx, self.act, self.msk, self.logp,
                         self.value)


class TorchSlotPolicy:
    """:class:`GpuActorPolicy`'s host interface (staged ``h_*`` inputs, per-slot LSTM state, ``keep``/``active``,
    :meth:`step_async`/:meth:`wait`, hidden snapshots) over the eager torch policy on any device — the CPU actor
    (BASELINE config 1: no GPU) and policies the fused graph does not cover (5v5 entity attention)."""

    def __init__(self, policy: Policy, n_slots: int, device='cpu', seed: int = 0, record: bool = True,
                 inputs_from: Optional['TorchSlotPolicy'] = None, **_):
        from .runner import PolicyRunner
        self.cfg = policy.config
        self.n = n_slots
        self.U = self.cfg.layout.max_units
        self.A = 21 + self.U
        self.device = torch.device(device)
        self.policy = type(policy)(self.cfg).to(self.device).eval()
        self.load_weights(policy)
        self.runner = PolicyRunner(self.policy, device=self.device, seed=seed)
        n, U = n_slots, self.U
        if inputs_from is not None:
            if (inputs_from.n, inputs_from.U) != (n, U):
                raise ValueError('inputs_from: slot count / layout mismatch')
            self.h_env, self.h_units, self.h_handles = inputs_from.h_env, inputs_from.h_units, inputs_from.h_handles
        else:
            self.h_env = torch.zeros(n, 3)
            self.h_units = torch.zeros(n, U, 10)
            self.h_handles = torch.full((n, U), -1, dtype=torch.long)
        self.h_keep = torch.ones(n, 1)
        self.h_active = torch.ones(n)
        H = self.cfg.hidden
        self.recurrent = self.cfg.rnn == 'lstm'
        self.h = np.zeros((n, H), np.float32)
        self.c = np.zeros((n, H), np.float32)
        self._out = None

    @torch.no_grad()
    def load_weights(self, policy_or_state):
        sd = policy_or_state.state_dict() if isinstance(policy_or_state, torch.nn.Module) else policy_or_state
        self.policy.load_state_dict({k: v.detach().to(self.device) for k, v in sd.items()}, strict=True)

    def step_async(self, snapshot_rows: Optional[np.ndarray] = None):
        keep = self.h_keep.numpy()
        self.h *= keep
        self.c *= keep
        out = {}
        if snapshot_rows is not None and len(snapshot_rows) and self.recurrent:
            rows = np.asarray(snapshot_rows)
            out['hidden'] = np.stack([self.h[rows], self.c[rows]], 1)
        act = np.flatnonzero(self.h_active.numpy() > 0)
        n, A = self.n, self.A
        out.update(idx=np.zeros((n, 4), np.int32), logp=np.zeros(n, np.float32), value=np.zeros(n, np.float32),
                   actions=np.zeros((n, A), np.uint8), masks=np.zeros((n, A), np.uint8))
        if len(act):
            hid = (self.h[act], self.c[act]) if self.recurrent else None
            o, nh = self.runner.step(self.h_env.numpy()[act], self.h_units.numpy()[act], self.h_handles.numpy()[act],
                                     hid)
            out['idx'][act] = np.stack([o.enum, o.x, o.y, o.target], 1)
            out['logp'][act], out['value'][act] = o.logp, o.value
            out['actions'][act], out['masks'][act] = o.actions, o.masks
            if nh is not None:
                self.h[act], self.c[act] = nh
        self._out = out

    def wait(self) -> Dict[str, np.ndarray]:
        self.h_keep.fill_(1.0)
        return self._out


ACTOR_PRECISIONS = ('bf16', 'fp32', 'fp8')


def slot_policy_class(policy: Policy, device='cuda', precision: str = 'bf16'):
    """The class :func:`make_slot_policy` builds: the fused graph-captured :class:`GpuActorPolicy` where it applies
    (``precision='fp32'``: :class:`F32ActorPolicy`, ``'fp8'``: :class:`Fp8ActorPolicy`), else :class:`TorchSlotPolicy`."""
    dev = torch.device(device)
    cfg = policy.config
    if precision not in ACTOR_PRECISIONS:
        raise ValueError(f'actor precision must be one of {ACTOR_PRECISIONS}, got {precision!r}')
    if precision == 'fp8':
        return Fp8ActorPolicy
    fused = dev.type == 'cuda' and cfg.unit_dim == 128 and cfg.env_dim == 128 and (
        not cfg.entity_attention or (cfg.layout.max_units == 64 and cfg.attention_heads == 4))
    if fused:
        return F32ActorPolicy if precision == 'fp32' else GpuActorPolicy
    return TorchSlotPolicy


def make_slot_policy(policy: Policy, n_slots: int, device='cuda', precision: str = 'bf16', **kw):
    """A :func:`slot_policy_class` policy over ``n_slots`` slots (``raw=True``: raw unit-record staging with the
    features computed on the GPU — the fused policies only)."""
    cls = slot_policy_class(policy, device, precision)
    if cls is TorchSlotPolicy:
        if kw.pop('raw', False):
            raise ValueError('raw unit-record staging needs a fused GPU actor policy')
        kw.pop('use_graph', None)
    return cls(policy, n_slots, device=torch.device(device), **kw)


# ----------------------------------------------------------------------------------------------------
def _synthetic_states(n_states: int, seed: int = 0):
    """Serialized CMsgBotWorldState snapshots from the synthetic engine (both teams' views, varied game times)."""
    from ..env import SyntheticDotaService
    from ..env.configs import get_1v1_selfplay_config
    from ..features.actions import action_to_pb
    from ..features.featurizer import get_unit
    from ..protos import pb
    svc = SyntheticDotaService(seed=seed)
    svc.reset_sync(get_1v1_selfplay_config())
    rng = np.random.default_rng(seed)
    states = []
    t = 0
    while len(states) < n_states:
        t += 1
        for team, pid in ((2, 0), (3, 5)):
            ws = svc.observe_sync(pb.ObserveConfig(team_id=team)).world_state
            if t > 100 and t % 3 == 0:   # skip the pre-horn start; decorrelate a little
                states.append(ws.SerializeToString())
            hero = get_unit(ws, player_id=pid)
            if hero is None:
                act = action_to_pb({'enum': 0}, None, None, pid)
            else:
                act = action_to_pb({'enum': 1, 'x': int(rng.integers(9)), 'y': int(rng.integers(9))},
                                   hero.location, None, pid)
            svc.act_sync(pb.Actions(actions=pb.CMsgBotWorldState.Actions(actions=[act]), team_id=team))
    return states[:n_states]


def measure_actor_throughput(policy: Policy, device='cuda', n_games: int = 2048, steps: int = 50,
                             warmup: int = 5, featurize: bool = True, threads: int = 8,
                             precision: str = 'bf16', raw: bool = True) -> Dict[str, float]:
    """Actor steps/s (player-observations → sampled actions per second) of one GPU-resident batched actor.

    ``n_games`` 1v1 games = 2·n_games player slots stepped per launch. With ``featurize`` the host side decodes
    and featurizes serialized world states through the native featurizer every step (the reference actor's
    per-step work, agent.py:611-660) overlapped with the previous GPU step; otherwise only the GPU step + copies
    are timed. ``precision='fp8'``: :class:`Fp8ActorPolicy`, ``'fp32'``: :class:`F32ActorPolicy`. Returns ``{'steps_per_s', 'gpu_steps_per_s',
    'ms_per_step', 'slots'}`` (``gpu_steps_per_s``: copy → step → copy, one step at a time). ``raw``
    (default, the runtime's path): raw unit records staged and featurized on the GPU (ops/csrc/featurize.hip);
    otherwise host features.
    """
    n = 2 * n_games
    dev = torch.device(device)
    layout = policy.config.layout
    cls = {'fp8': Fp8ActorPolicy, 'fp32': F32ActorPolicy}.get(precision, GpuActorPolicy)
    gp = cls(policy, n, device=dev, seed=1234, record=True, raw=raw)
    feat = None
    if featurize:
        from .. import native
        if not native.AVAILABLE:
            featurize = False
        else:
            pool = _synthetic_states(256)
            pids = [0 if i % 2 == 0 else 5 for i in range(n)]
            teams = [2 if i % 2 == 0 else 3 for i in range(n)]
            batch = [pool[i % len(pool)] for i in range(n)]
            counts = list(layout.counts)

            def feat():
                if raw:
                    return native.featurize_batch_raw(batch, pids, teams, counts, threads)[:3]
                return native.featurize_batch(batch, pids, teams, counts, threads)
    if not featurize:
        rng = np.random.default_rng(0)
        env = rng.standard_normal((n, 3)).astype(np.float32)
        units = rng.standard_normal((n, layout.max_units, 10)).astype(np.float32)
        handles = np.where(rng.random((n, layout.max_units)) < 0.5, rng.integers(1, 1000, (n, layout.max_units)),
                           -1).astype(np.int64)

        if raw:
            from ..features.raw import F_PRESENT
            hero = np.zeros((n, 4), np.float32)
            hero[:, :2] = rng.uniform(-7000, 7000, (n, 2))
            hero[:, 2] = 600.0
            rawb = np.zeros((n, layout.max_units, 8), np.int32)
            rawb.view(np.float32)[..., :5] = rng.uniform(-1000, 1000, (n, layout.max_units, 5))
            rawb[..., 5] = handles
            rawb[..., 6] = np.where(rng.random((n, layout.max_units)) < 0.6, F_PRESENT, 0)

        def feat():
            return (env, hero, rawb) if raw else (env, units, handles, None)

    def fill(f):
        if raw:
            gp.stage_raw(f[0], f[1], f[2])
        else:
            gp.stage(f[0], f[1], f[2])

    fill(feat())
    gp.step_async(); gp.wait()
    for _ in range(warmup):
        gp.step_async()
        f = feat()
        gp.wait()
        fill(f)
    # GPU-only rate (no featurize in the loop)
    torch.cuda.synchronize(dev)
    t0 = time.perf_counter()
    for _ in range(steps):
        gp.step_async()
        gp.wait()
    gpu_dt = (time.perf_counter() - t0) / steps
    # pipelined: featurize step t+1 on the host while the GPU runs step t
    t0 = time.perf_counter()
    for _ in range(steps):
        gp.step_async()
        f = feat()
        gp.wait()
        fill(f)
    dt = (time.perf_counter() - t0) / steps
    return {'steps_per_s': n / dt, 'gpu_steps_per_s': n / gpu_dt, 'ms_per_step': dt * 1e3, 'slots': n}
