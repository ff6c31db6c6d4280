"""Data-parallel gradient synchronisation over one flat gradient buffer.

Capability parity with the reference's ``DistributedDataParallelSparseParamCPU`` (reference distributed.py:16-79):

* parameters are broadcast from rank 0 when the wrapper is built (distributed.py:71-74);
* after backward every gradient is SUM-all-reduced and divided by the number of ranks that actually produced a
  gradient for that parameter ("has-grad count", distributed.py:29-57);
* parameters outside the loss graph on *every* rank (count 0) are neither reduced-into nor stepped by the optimizer
  (e.g. ``affine_value`` when ``vf_coef == 0``).

Re-designed for MI355X / RCCL over xGMI rather than translated:

* all parameters live as views of ONE flat fp32 buffer and all gradients as views of ONE flat gradient buffer,
  so the reference's 60 sequential per-parameter gloo calls become a handful of large bucketed collectives (a
  ring all-reduce over xGMI is per-link bandwidth bound; few large messages amortise RCCL launch latency);
* the per-parameter has-grad counts — and the persistent kernels' error flag — travel in a header segment at the
  START of the flat gradient buffer, inside the last bucket (which always holds the first-registered parameters):
  one contiguous all-reduce, no separate collective and no per-step concatenation / copy;
* with ``overlap=True`` a bucket's all-reduce is issued on a dedicated comm stream from a post-accumulate-grad hook
  as soon as every parameter in it has its gradient, so communication overlaps the rest of backward (buckets are
  formed in reverse registration order ≈ backward order);
* every rank ends with the identical reduced gradient (fixes reference quirk §2.10-8).
"""
from __future__ import annotations

import time

from typing import Dict, List, Optional, Sequence

import torch
import torch.distributed as dist
import torch.nn as nn

from .dist import get_world_size, is_distributed


class FlatParams:
    """Re-home a module's trainable parameters (and their ``.grad``) into two contiguous flat buffers.

    ``flat[offsets[i]:offsets[i]+numel[i]]`` is parameter i; autograd accumulates in place into the matching
    view of ``grad`` because ``.grad`` is pre-set (zero it with :meth:`zero_grad`, never set it to None).
    Offsets are 64-element aligned so each parameter starts on a 256-B boundary (16-B vector loads in kernels).
    The first ``header`` elements (``n_params + 1`` rounded up to 64) hold no parameter: in ``grad`` they carry the
    DP has-grad flags / counts and the kernel-error flag (:class:`DataParallel`); segment id -1, never stepped.
    """

    ALIGN = 64

    def __init__(self, module: nn.Module, device=None, dtype=torch.float32):
        self.names: List[str] = []
        self.params: List[nn.Parameter] = []
        for n, p in module.named_parameters():
            if p.requires_grad:
                self.names.append(n)
                self.params.append(p)
        device = torch.device(device) if device is not None else self.params[0].device
        self.numel = [p.numel() for p in self.params]
        self.header = (len(self.params) + 1 + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.offsets = []
        off = self.header
        for n in self.numel:
            self.offsets.append(off)
            off += (n + self.ALIGN - 1) // self.ALIGN * self.ALIGN
        self.total = off
        self.flat = torch.zeros(self.total, device=device, dtype=dtype)
        self.grad = torch.zeros(self.total, device=device, dtype=dtype)
        # per-element segment id (int32) — used by fused kernels to find a parameter's has-grad count.
        seg = torch.full((self.total,), -1, dtype=torch.int32)
        for i, (o, n) in enumerate(zip(self.offsets, self.numel)):
            seg[o:o + n] = i
        self.segment_ids = seg.to(device)
        with torch.no_grad():
            for p, o, n in zip(self.params, self.offsets, self.numel):
                self.flat[o:o + n].copy_(p.data.reshape(-1))
                p.data = self.flat[o:o + n].view_as(p)
                p.grad = self.grad[o:o + n].view_as(p)

    def view(self, i: int, buf: Optional[torch.Tensor] = None) -> torch.Tensor:
        buf = self.flat if buf is None else buf
        return buf[self.offsets[i]:self.offsets[i] + self.numel[i]].view_as(self.params[i])

    def zero_grad(self):
        self.grad.zero_()

    def rebind(self):
        """Re-attach .data/.grad views (after load_state_dict replaced tensors, for example)."""
        with torch.no_grad():
            for i, p in enumerate(self.params):
                v = self.view(i)
                if p.data.data_ptr() != v.data_ptr():
                    v.copy_(p.data)
                    p.data = v
                p.grad = self.view(i, self.grad)


class DataParallel:
    """Bucketed flat-buffer gradient all-reduce with has-grad-count semantics (see module docstring)."""

    def __init__(self, module: nn.Module, flat: Optional[FlatParams] = None, process_group=None,
                 bucket_cap_mb: float = 8.0, overlap: bool = True, broadcast: bool = True):
        self.module = module
        self.flat = flat if flat is not None else FlatParams(module)
        self.group = process_group
        self.world = get_world_size() if is_distributed() else 1
        self.enabled = self.world > 1
        self.n_params = len(self.flat.params)
        dev = self.flat.grad.device
        # has-grad flags, one float per parameter (1 = this rank produced a gradient this step), and the error flag
        # of the persistent kernels: views of the gradient buffer's header, all-reduced with the last bucket —
        # afterwards the same memory holds the has-grad COUNTS and the number of ranks whose step failed
        self.has_grad = self.flat.grad[:self.n_params]
        self.err_flag = self.flat.grad[self.n_params:self.n_params + 1]
        self.counts = self.has_grad
        self.overlap = overlap and self.enabled and dev.type == 'cuda'
        self._build_buckets(bucket_cap_mb)
        self._comm_stream = torch.cuda.Stream(device=dev) if self.overlap else None
        self._works = []
        self._pending: Dict[int, int] = {}
        self._next = 0
        self._hooks = []
        # per-step communication timing (enable_timing): the early buckets' all-reduce on the comm stream against the
        # step's second compute phase (graph 2), and the count-carrying last bucket after it — a ring of the last
        # records, read without a host sync by comm_stats() (only completed records count)
        self.timing = False
        self._trec: List[dict] = []
        self._cur: Optional[dict] = None
        for i, p in enumerate(self.flat.params):
            self._hooks.append(p.register_post_accumulate_grad_hook(self._make_hook(i)))
        if broadcast and self.enabled:
            dist.broadcast(self.flat.flat, 0, group=self.group)

    # ------------------------------------------------------------------------------------------------
    def _build_buckets(self, cap_mb: float):
        cap = max(1, int(cap_mb * 1024 * 1024 / self.flat.grad.element_size()))
        order = list(range(self.n_params))[::-1]            # reverse registration ≈ backward order
        buckets, cur = [], []
        size = 0
        for i in order:
            n = self.flat.numel[i]
            if cur and size + n > cap:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += n
        if cur:
            buckets.append(cur)
        self.buckets: List[List[int]] = buckets
        self.param_bucket = {}
        for b, idxs in enumerate(buckets):
            for i in idxs:
                self.param_bucket[i] = b
        # contiguous [lo, hi) element range of each bucket in the flat buffer
        self.bucket_ranges = []
        for idxs in buckets:
            lo = min(self.flat.offsets[i] for i in idxs)
            hi = max(self.flat.offsets[i] + self.flat.numel[i] for i in idxs)
            self.bucket_ranges.append((lo, hi))
        self._extend_last()

    def _extend_last(self):
        """The last bucket holds parameter 0, so its range starts right after the header: extend it over the header
        (has-grad flags + error flag ride along in the same all-reduce)."""
        lo, hi = self.bucket_ranges[-1]
        assert 0 in self.buckets[-1] and lo == self.flat.header, 'the count-carrying bucket must hold parameter 0'
        self.bucket_ranges[-1] = (0, hi)

    def split_buckets(self, early: Sequence[int], cap_mb: float = 8.0) -> bool:
        """Bucket layout for a step whose gradients finish in two phases (the learner's direct step): the EARLY
        parameters (a contiguous index range) get their own buckets, launched by :meth:`launch_early` while the
        second phase still runs; the rest form the last bucket, which carries the has-grad counts. Returns False
        (layout unchanged) if ``early`` is not a contiguous proper sub-range."""
        early = sorted(set(early))
        if not early or len(early) >= self.n_params or early != list(range(early[0], early[-1] + 1)):
            return False
        if early[-1] != self.n_params - 1:
            return False                     # early must be a suffix: the late bucket then starts at the header
        late = [i for i in range(self.n_params) if i not in set(early)]
        cap = max(1, int(cap_mb * 1024 * 1024 / self.flat.grad.element_size()))
        buckets, cur, size = [], [], 0
        for i in early[::-1]:
            if cur and size + self.flat.numel[i] > cap:
                buckets.append(cur)
                cur, size = [], 0
            cur.append(i)
            size += self.flat.numel[i]
        buckets.append(cur)
        buckets.append(late[::-1])
        self.buckets = buckets
        self.param_bucket = {i: b for b, idxs in enumerate(buckets) for i in idxs}
        self.bucket_ranges = [(min(self.flat.offsets[i] for i in idxs),
                               max(self.flat.offsets[i] + self.flat.numel[i] for i in idxs)) for idxs in buckets]
        self._extend_last()
        return True

    def _mark(self, name: str, stream=None):
        """Timing mark of the current step's record: a timing event on ``stream`` (GPU) or the wall clock (CPU)."""
        if not self.timing:
            return
        if self._cur is None:
            self._cur = {}
        if self.overlap:
            ev = torch.cuda.Event(enable_timing=True)
            ev.record(stream)
            self._cur[name] = ev
        else:
            self._cur[name] = time.perf_counter()

    def launch_early(self):
        """All-reduce every bucket but the last (the early-phase gradients) now, asynchronously on the comm
        stream, overlapping whatever the current stream runs next; :meth:`sync` finishes the step."""
        if not self.enabled:
            return
        if self.timing and self._next < len(self.buckets) - 1:
            cur = torch.cuda.current_stream(self.flat.grad.device) if self.overlap else None
            self._mark('phase2_start', cur)                     # graph 2 starts behind this point
            if self.overlap:
                self._comm_stream.wait_stream(cur)
            self._mark('early_start', self._comm_stream)
        for b in range(self._next, len(self.buckets) - 1):
            self._launch(b)
        if self.timing and 'early_start' in (self._cur or {}):
            self._mark('early_end', self._comm_stream)
        self._next = len(self.buckets) - 1

    def _make_hook(self, i: int):
        def hook(p):
            self.has_grad[i:i + 1].fill_(1.0)          # kernel fill (capturable), no host→device scalar copy
            if self.overlap and not torch.cuda.is_current_stream_capturing():
                b = self.param_bucket[i]
                self._pending[b] = self._pending.get(b, 0) + 1
                # Launch strictly in bucket-index order so every rank issues the same collective sequence
                # even if some parameter lacks a gradient on some rank.
                while (self._next < len(self.buckets) - 1
                       and self._pending.get(self._next, 0) == len(self.buckets[self._next])):
                    self._launch(self._next)
                    self._next += 1
        return hook

    def _launch(self, b: int):
        lo, hi = self.bucket_ranges[b]
        buf = self.flat.grad[lo:hi]
        if self.overlap:
            cur = torch.cuda.current_stream(buf.device)
            self._comm_stream.wait_stream(cur)
            with torch.cuda.stream(self._comm_stream):
                self._works.append(dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group, async_op=True))
        else:
            dist.all_reduce(buf, op=dist.ReduceOp.SUM, group=self.group)
        self._pending[b] = -1   # launched

    # ------------------------------------------------------------------------------------------------
    def zero_grad(self):
        self.flat.zero_grad()
        self.has_grad.zero_()
        self._pending = {}
        self._next = 0
        self._works = []

    def sync(self, scale: bool = True):
        """Finish the gradient reduction. Afterwards ``flat.grad`` holds the has-grad-averaged gradient and
        ``counts`` the number of ranks that had a gradient for each parameter. ``scale=False`` leaves the SUMS in
        ``flat.grad`` for an optimizer that divides by the counts itself (FlatAdam.step(divide=True))."""
        if not self.enabled:                  # counts IS has_grad (same header view)
            return
        # Launch whatever the hooks did not (params without grad on this rank, the count-carrying last bucket).
        rest = range(self._next, len(self.buckets) - 1)
        if self.timing and len(rest) and 'early_start' not in (self._cur or {}):
            cur = torch.cuda.current_stream(self.flat.grad.device) if self.overlap else None
            if self.overlap:
                self._comm_stream.wait_stream(cur)
            self._mark('early_start', self._comm_stream if self.overlap else None)
        for b in rest:
            self._launch(b)
        if self.timing and len(rest) and 'early_end' not in (self._cur or {}):
            self._mark('early_end', self._comm_stream if self.overlap else None)
        # The last bucket starts at 0: header (has-grad flags, error flag) + the first parameters, one view.
        lo, hi = self.bucket_ranges[-1]
        last = self.flat.grad[lo:hi]
        if self.overlap:
            cur = torch.cuda.current_stream(last.device)
            self._mark('compute_end', cur)                      # the step's compute is queued up to here
            self._comm_stream.wait_stream(cur)
            self._mark('late_start', self._comm_stream)
            with torch.cuda.stream(self._comm_stream):
                dist.all_reduce(last, op=dist.ReduceOp.SUM, group=self.group)
            self._mark('late_end', self._comm_stream)
            for w in self._works:
                w.wait()
            cur.wait_stream(self._comm_stream)
        else:
            self._mark('compute_end')
            self._mark('late_start')
            dist.all_reduce(last, op=dist.ReduceOp.SUM, group=self.group)
            self._mark('late_end')
        if self.timing and self._cur is not None:
            self._trec.append(self._cur)
            del self._trec[:-64]
        self._cur = None
        self._works = []
        self._pending = {}
        self._next = 0
        if not scale:
            return
        # grad /= count  (count 0 → gradient stays 0 and the optimizer skips the parameter); the header keeps the counts
        h = self.flat.header
        inv = torch.where(self.counts > 0, 1.0 / self.counts.clamp_min(1.0), torch.zeros_like(self.counts))
        seg = self.flat.segment_ids[h:]
        scale = torch.where(seg >= 0, inv[seg.clamp_min(0).long()], torch.zeros_like(self.flat.grad[h:]))
        self.flat.grad[h:].mul_(scale)

    def comm_stats(self) -> Optional[Dict[str, float]]:
        """Mean per-step communication timing over the recorded steps (``timing`` on), None without records:
        ``allreduce_ms`` (early + last bucket on the comm stream), ``early_ms`` / ``late_ms``, ``overlap_frac`` — the
        share of the early buckets' all-reduce that ran while the step's second compute phase (graph 2: the encoder
        backward) was still running — and ``exposed_ms``, the comm time after the compute ended (the step waits for
        it). GPU records are timing events read once complete (``query()``, no host sync); CPU (gloo) records the
        wall clock of the synchronous calls (no overlap)."""
        recs = []
        for r in self._trec:
            if 'late_end' not in r:
                continue
            if self.overlap:
                if not all(e.query() for e in r.values()):
                    continue
                t = lambda a, b: r[a].elapsed_time(r[b])  # noqa: E731
            else:
                t = lambda a, b: 1e3 * (r[b] - r[a])       # noqa: E731
            late = t('late_start', 'late_end')
            early = ov = 0.0
            if 'early_end' in r:
                early = t('early_start', 'early_end')
                if 'phase2_start' in r:
                    # [early_start, early_end] ∩ [phase2_start, compute_end] on the comm / compute timelines
                    ov = max(0.0, min(early, t('early_start', 'compute_end')) -
                             max(0.0, t('early_start', 'phase2_start')))
            exposed = max(0.0, t('compute_end', 'late_end'))
            recs.append((early + late, early, late, ov / early if early > 0 else 0.0, exposed))
        if not recs:
            return None
        n = len(recs)
        keys = ('allreduce_ms', 'early_ms', 'late_ms', 'overlap_frac', 'exposed_ms')
        out = {k: sum(r[i] for r in recs) / n for i, k in enumerate(keys)}
        out['steps'] = n
        out['buckets'] = len(self.buckets)
        out['bucket_mb'] = [round((hi - lo) * self.flat.grad.element_size() / 2 ** 20, 3)
                            for lo, hi in self.bucket_ranges]
        return out

    def remove_hooks(self):
        for h in self._hooks:
            h.remove()
        self._hooks = []
