"""Pipelined device ingest: an iteration's rollouts are staged and uploaded while the previous iteration trains.

The reference ingests synchronously: pop rollouts, pad each to a multiple of ``seq_len``, compute returns, slice
into sequences, then train (optimizer.py:428-471). On the GPU learner that host work used to sit in series with the
training of every iteration (decode → pad into pinned buffers → H2D of the padded rows → scan → train). Here:

* a stager thread consumes and decodes experience messages (as the decode-ahead thread did), groups them into the
  next iteration's rollout set (≥ ``seq_per_epoch`` sequences, the reference's gather loop, optimizer.py:441-453),
  packs ONLY THE VALID ROWS of every field into one pinned slot (double-buffered), and issues one H2D copy on a copy
  stream of its own — so decode, packing and the upload of iteration k+1 overlap the training of iteration k;
* the learner thread takes a staged iteration, makes its stream wait for the copy's event, and expands the packed
  rows into the padded ``(n_seq · seq_len, …)`` layout on the device (zero fill + one ``index_copy_`` per field:
  padding never crosses PCIe — with the deploy's ≈550-step games in 1400-step sequences that is ≈60 % of the
  bytes), then runs the return / GAE scan exactly as before.

Slot reuse is event-ordered: the host waits for a slot's previous upload to finish before repacking it, and the copy
stream waits for the learner stream's "consumed" event before overwriting the slot's device bytes.

Sequence packing (``pack=True``, non-compat): instead of padding every rollout to a multiple of ``seq_len`` (the
reference, optimizer.py:355-378 — with ≈560-step games in 1400-step sequences 60 % of the trained rows are padding),
whole rollouts that start from a zero recurrent state are placed first-fit into the free tail of an open sequence.
The row where such a rollout starts carries a ``reset`` flag: the recurrence treats h, c as zero before that step
(forward and backward, ops/csrc/lstm_team.hip), so each episode sees exactly the state it would have seen at the start
of its own padded sequence. Rollouts longer than a sequence, or starting from a stored non-zero state, keep the
padded layout (aligned at a sequence start, the stored chunk states as h0 / c0); their last sequence's free tail is
packed like any other. The return / GAE scan segments are the rollouts in row order.
"""
from __future__ import annotations

import os
import queue
import threading
import time
from dataclasses import dataclass, field
from typing import Callable, Dict, List, Optional

import numpy as np
import torch

from ..transport.codec import Rollout

_ALIGN = 64


_STAGE_PROF = os.environ.get('DCA_STAGE_PROF') == '1'


def _round(n: int) -> int:
    return (n + _ALIGN - 1) // _ALIGN * _ALIGN


def _load_native_copy():
    try:
        from ..native import _native
        return _native.copy_jobs
    except (ImportError, AttributeError):
        return None


_native_copy = _load_native_copy()


def _ops():
    """The HIP extension (raises when it is not built: a GPU learner never falls back silently)."""
    from .. import ops
    return ops.require()


def _load_native_pack():
    try:
        from ..native import _native
        return _native.pack_rows
    except (ImportError, AttributeError):
        return None


_native_pack = _load_native_pack()


def _release_all(rollouts):
    """Give the ring regions of dropped ring-resident rollouts back (learner/optimizer.py zero-copy consumption)."""
    for r in rollouts:
        rel = getattr(r, 'release', None)
        if rel is not None:
            r.release = None
            rel()


class _Stopped(Exception):
    pass


class _ClaimsAbandoned(Exception):
    """stage(): a ring-resident rollout's claim was abandoned by the ring while it was being copied."""


def _claim_ok(r: Rollout) -> bool:
    """Whether a rollout's bytes are still its own: True for heap rollouts, else the ring's verdict on its claim."""
    rel = getattr(r, 'release', None)
    valid = getattr(rel, 'valid', None)
    return True if valid is None else bool(valid())


def _zero_start(r: Rollout) -> bool:
    """A rollout whose recurrent state at its first step is zero (a game start): it may begin mid-sequence."""
    h = r.hiddens
    return h is None or len(h) == 0 or not np.any(np.asarray(h[0]))


class SequencePacker:
    """First-fit placement of rollouts into ``S``-row sequences (see the module docstring). ``add`` places one
    rollout; ``fits`` tells whether it would go into an open sequence without opening a new one."""

    def __init__(self, S: int, pack: bool = True):
        self.S, self.pack = int(S), bool(pack)
        self.n_seq = 0
        self.open: List[List[int]] = []          # [sequence index, rows used] of sequences with a free tail
        self.starts: List[int] = []              # first padded row of every added rollout
        self.seq_src: List[Optional[tuple]] = []  # per sequence: (rollout index, chunk) starting at its row 0
        self.resets: List[int] = []              # rows where a packed rollout starts mid-sequence

    def fits(self, r: Rollout) -> bool:
        T = r.length
        return self.pack and T <= self.S and _zero_start(r) and any(self.S - u >= T for _, u in self.open)

    def add(self, r: Rollout) -> int:
        S, T, i = self.S, r.length, len(self.starts)
        if self.pack and T <= S and _zero_start(r):
            for slot in self.open:
                if S - slot[1] >= T:
                    start = slot[0] * S + slot[1]
                    slot[1] += T
                    self.starts.append(start)
                    if start % S:
                        self.resets.append(start)
                    return start
        k = -(-T // S)
        start = self.n_seq * S
        for c in range(k):
            self.seq_src.append((i, c))
        tail = T - (k - 1) * S
        if self.pack and tail < S:
            self.open.append([self.n_seq + k - 1, tail])
        self.n_seq += k
        self.starts.append(start)
        return start


@dataclass
class StagedIteration:
    rollouts: List[Rollout]                 # decoded rollouts (metrics / canvas / reward stats on the host)
    lens: List[int]
    off: np.ndarray                         # padded row offset of every rollout (len + 1)
    n_seq: int
    L: int                                  # padded rows
    Lv: int                                 # valid rows
    gae_mode: bool
    views: Dict[str, torch.Tensor] = field(default_factory=dict)   # device views of the packed slot
    ready: Optional[torch.cuda.Event] = None
    slot: int = 0
    stage_s: float = 0.0                    # host packing + upload issue time (stager thread)
    gather_s: float = 0.0                   # stager time waiting for the iteration's decoded rollouts
    wait_s: float = 0.0                     # part of stage_s spent waiting for a free slot (the learner behind)
    copy_s: float = 0.0                     # part of stage_s in the field copies into the pinned slot
    release_s: float = 0.0                  # part of stage_s giving ring-resident rollouts back
    raw: bool = False                       # units staged as raw records (featurized on the device in expand)


class _Slot:
    def __init__(self):
        self.host: Optional[torch.Tensor] = None       # pinned bytes
        self.dev: Optional[torch.Tensor] = None        # device bytes
        self.uploaded: Optional[torch.cuda.Event] = None
        self.consumed: Optional[torch.cuda.Event] = None
        self.free = threading.Semaphore(1)             # released by the learner once it has issued the expand


class IngestPipeline:
    """Stager thread + double-buffered pinned/device slots (see module docstring)."""

    def __init__(self, fetch: Optional[Callable], seq_len: int, seq_per_epoch: int, algo: str, hidden: int, device,
                 depth: int = 1, pack: bool = False):
        """``fetch=None``: no stager thread — the learner calls :meth:`stage` and :meth:`expand` inline."""
        self.fetch = fetch                      # fetch(stop_event) -> Rollout | None
        self.pack = bool(pack)
        self._carry: Optional[Rollout] = None   # packing: fetched rollout that did not fit the previous iteration
        self.S = int(seq_len)
        self.need = int(seq_per_epoch)
        self.algo = algo
        self.H = int(hidden)
        self.device = torch.device(device)
        self.cuda = self.device.type == 'cuda'          # CPU learner: the slot IS the device buffer, no events
        self.copy_stream = torch.cuda.Stream(device=self.device) if self.cuda else None
        self.slots = [_Slot(), _Slot()]
        self.q: 'queue.Queue[StagedIteration]' = queue.Queue(maxsize=max(1, depth))
        self.err: Optional[BaseException] = None
        self.stop = threading.Event()
        self.lost = 0
        self.abandoned_iterations = 0          # iterations dropped because a zero-copy claim was abandoned mid-copy
        self._k = 0
        self.th = None
        if fetch is not None:
            self.th = threading.Thread(target=self._run, name='xp-stager', daemon=True)
            self.th.start()

    # ---- stager thread -----------------------------------------------------------------------------
    def _gather(self) -> Optional[List[Rollout]]:
        if not self.pack:
            rollouts, n_seq = [], 0
            while n_seq < self.need:
                r = self.fetch(self.stop)
                if r is None:
                    self.lost += len(rollouts)
                    _release_all(rollouts)
                    return None
                rollouts.append(r)
                n_seq += -(-r.length // self.S)
            return rollouts
        # packing: at least ``need`` sequences, then keep filling their free tails until a rollout does not fit
        # (it is carried over to the next iteration) or every open tail is nearly full
        pk, rollouts = SequencePacker(self.S), []
        while True:
            r, self._carry = self._carry, None
            if r is None:
                r = self.fetch(self.stop)
            if r is None:
                self.lost += len(rollouts)
                _release_all(rollouts)
                return None
            if pk.n_seq >= self.need and not pk.fits(r):
                self._carry = r
                return rollouts
            pk.add(r)
            rollouts.append(r)
            if pk.n_seq >= self.need and all(self.S - u < 32 for _, u in pk.open):
                return rollouts

    def _run(self):
        import contextlib
        try:
            with (torch.cuda.device(self.device) if self.cuda else contextlib.nullcontext()):
                while not self.stop.is_set():
                    tg = time.perf_counter()
                    rollouts = self._gather()
                    if rollouts is None:
                        break
                    tg = time.perf_counter() - tg
                    try:
                        st = self.stage(rollouts)
                        st.gather_s = tg
                    except _ClaimsAbandoned:
                        # (stage() gave every region back): the iteration is dropped, the stager gathers anew
                        self.lost += len(rollouts)
                        self.abandoned_iterations += 1
                        continue
                    except _Stopped:
                        self.lost += len(rollouts)
                        _release_all(rollouts)
                        break
                    while True:
                        try:
                            self.q.put(st, timeout=0.1)
                            break
                        except queue.Full:
                            if self.stop.is_set():
                                self.lost += len(st.rollouts)
                                return
        except BaseException as e:       # surfaced on the learner thread
            self.err = e

    def stage(self, rollouts: List[Rollout]) -> StagedIteration:
        """Pack the valid rows of every field into the next pinned slot and issue its upload (any thread)."""
        t0 = time.perf_counter()
        S = self.S
        marks = self._marks = [('start', t0, time.thread_time())] if _STAGE_PROF else None

        def mk(label):
            if marks is not None:
                marks.append((label, time.perf_counter(), time.thread_time()))
        pk = SequencePacker(S, self.pack)
        for r in rollouts:
            pk.add(r)
        # rollouts in row order: the scan's segments are [start_s, start_{s+1}) (a rollout plus the free tail that
        # follows it in its sequence)
        order = sorted(range(len(rollouts)), key=lambda i: pk.starts[i])
        rank = {i: k for k, i in enumerate(order)}
        seq_src = [None if src is None else (rank[src[0]], src[1]) for src in pk.seq_src]
        rollouts = [rollouts[i] for i in order]
        starts = [pk.starts[i] for i in order]
        lens = [r.length for r in rollouts]
        n_seq = pk.n_seq
        L, Lv = n_seq * S, int(sum(lens))
        off = np.asarray(starts + [L], np.int64)
        resets = np.asarray(pk.resets, np.int64)
        r0 = rollouts[0]
        # raw rollouts (an actor with GPU featurization, features/raw.py): the compact unit records are uploaded and
        # featurized on the device in expand(); an iteration that mixes them with featurized rollouts converts the
        # raw ones on the host (exact: the numpy oracle of the kernel)
        raw = all(r.units is None and r.units_raw is not None for r in rollouts)
        if not raw:
            for r in rollouts:
                r.ensure_units()
        U = (r0.units_raw if raw else r0.units).shape[1]
        A, K = r0.actions.shape[1], r0.rewards.shape[1]
        gae_mode = self.algo == 'ppo' and all(r.values is not None for r in rollouts)
        unit_fields = ([('units_raw', torch.int32, (U, 8)), ('hero', torch.float32, (4,))] if raw else
                       [('units', torch.float32, (U, 10))])
        fields = [('rows', torch.int64, ()), ('env', torch.float32, (3,))] + unit_fields + [
                  ('actions', torch.uint8, (A,)), ('masks', torch.uint8, (A,)), ('logp', torch.float32, ()),
                  ('rewards', torch.float32, (K,))]
        if gae_mode:
            fields.append(('values', torch.float32, ()))
        layout, nbytes = [], 0
        for name, dt, tail in fields:
            n = Lv * int(np.prod(tail, dtype=np.int64)) * torch.empty((), dtype=dt).element_size()
            layout.append((name, dt, tail, nbytes, n))
            nbytes += _round(n)
        hid_off = None
        if self.H:
            hid_off = nbytes
            nbytes += _round(n_seq * 2 * self.H * 4)
        rst_off = None
        if self.pack:
            rst_off = nbytes                     # (L,) u8 episode-start flags in the padded layout
            nbytes += _round(L)
        inv_off = nbytes                         # (L,) i32: the valid row each padded row takes, −1 for padding
        nbytes += _round(4 * L)
        mk('pack')
        slot_i = self._k % 2
        slot = self.slots[slot_i]
        tw = time.perf_counter()
        while not slot.free.acquire(timeout=0.1):      # the learner has not expanded this slot's last contents yet
            if self.stop.is_set():
                raise _Stopped()
        self._k += 1
        if slot.uploaded is not None:
            slot.uploaded.synchronize()               # the slot's previous upload has left the pinned buffer
        tw = time.perf_counter() - tw
        if slot.host is None or slot.host.numel() < nbytes:
            cap = max(nbytes, 2 * (slot.host.numel() if slot.host is not None else 0), 1 << 20)
            if slot.consumed is not None:
                # (rare) growth: the learner has expanded this slot's last contents (its upload was waited for
                # above), so nothing reads the old buffers any more. An event wait, not a device synchronise: the
                # learner may be capturing its step graph right now, and a device-wide sync from this thread would
                # invalidate that capture
                slot.consumed.synchronize()
            # pinned / device allocations are serialised against the learner's graph captures (learner/engine.py)
            from .engine import CAPTURE_LOCK
            with CAPTURE_LOCK:
                slot.host = torch.empty(cap, dtype=torch.uint8, pin_memory=self.cuda)
                if self.cuda:
                    with torch.cuda.stream(self.copy_stream):
                        slot.dev = torch.empty(cap, dtype=torch.uint8, device=self.device)
                else:
                    slot.dev = slot.host
            slot.consumed = None
        hb = slot.host.numpy()
        mk('slot')

        def hview(o, n, dt, shape):
            return hb[o:o + n].view(np.dtype(str(dt).replace('torch.', ''))).reshape(shape)
        views_h = {name: hview(o, n, dt, (Lv,) + tail) for name, dt, tail, o, n in layout}
        pos = 0
        rows = views_h['rows']
        jobs = []
        direct = (('env',) + tuple(f[0] for f in unit_fields) + ('actions', 'masks', 'logp')
                  + (('values',) if gae_mode else ()))
        tc = 0.0
        if _native_pack is not None:
            # every field of every rollout in ONE native call (memcpy / f64 → f32 rewards / zero fill, GIL released);
            # the rows (padded-layout index of every valid row) vectorised
            vpos = np.zeros(len(rollouts) + 1, np.int64)
            np.cumsum(lens, out=vpos[1:])
            rows[:] = np.arange(Lv, dtype=np.int64) + np.repeat(off[:-1] - vpos[:-1], lens)
            mk('loop')
            tc = time.perf_counter()
            try:
                _native_pack([(views_h[name], [getattr(r, name) for r in rollouts])
                              for name in direct + ('rewards',)], vpos, 4)
                rollouts_loop = ()
            except ValueError:          # a field of another dtype (e.g. a reference agent's pickle): numpy converts
                rollouts_loop = zip(rollouts, lens, off[:-1])
            tc = time.perf_counter() - tc
        else:
            rollouts_loop = zip(rollouts, lens, off[:-1])
        # fallback without the native module: the same-dtype fields go to the native parallel copy as one job list
        # when that exists, rows, the f64 → f32 rewards and missing fields stay numpy
        for r, T, a in rollouts_loop:
            sl = slice(pos, pos + T)
            rows[sl] = np.arange(a, a + T)
            for name in direct:
                src, dst = getattr(r, name), views_h[name][sl]
                if src is None:
                    dst[...] = 0
                elif _native_copy is not None and src.dtype == dst.dtype and src.flags.c_contiguous \
                        and src.shape == dst.shape:
                    jobs.append((dst.ctypes.data, src.ctypes.data, dst.nbytes))
                else:
                    dst[...] = src
            np.copyto(views_h['rewards'][sl], r.rewards, casting='same_kind')
            pos += T
        if jobs:
            mk('loop')
            tc = time.perf_counter()
            _native_copy(np.asarray(jobs, dtype=np.int64), 4)
            tc = time.perf_counter() - tc
        mk('copy')
        if self.H:
            hid = hview(hid_off, n_seq * 2 * self.H * 4, 'float32', (n_seq, 2, self.H))
            for i, src in enumerate(seq_src):
                # the state at the sequence's first row: the stored state of the rollout chunk that starts there
                # (zero for a game start, and for packed sequences — their rollouts start from zero)
                hid[i] = 0.0
                if src is not None:
                    r = rollouts[src[0]]
                    a = src[1] * S
                    if r.hiddens is not None and r.hidden_stride and a % r.hidden_stride == 0 \
                            and a // r.hidden_stride < len(r.hiddens):
                        hid[i] = r.hiddens[a // r.hidden_stride]
        iv = hview(inv_off, 4 * L, 'int32', (L,))
        iv[:] = -1
        iv[rows] = np.arange(Lv, dtype=np.int32)
        if self.pack:
            rv = hview(rst_off, L, 'uint8', (L,))
            rv[:] = 0
            rv[resets] = 1
        # ring-resident rollouts (zero-copy consumption, learner/optimizer.py): everything the upload needs is in the
        # pinned slot now — give their ring regions back (the canvas of the last one is kept for the logs)
        mk('hid+reset')
        tr = time.perf_counter()
        # a zero-copy claim held past the ring's abandonment deadline (native/core.h claim_abandon_s_, 60 s: a learner
        # stalled that long while producers needed the space) may have been reclaimed and overwritten WHILE it was
        # copied above — its CRC was checked at claim time, so nothing else would notice: drop the whole iteration
        gone = sum(1 for r in rollouts if not _claim_ok(r))
        if gone:
            _release_all(rollouts)              # (the abandoned tokens' releases are ignored by the ring)
            self._k -= 1                        # the slot was not used: the next stage takes it again
            slot.free.release()
            raise _ClaimsAbandoned(gone)
        rels = [rel for i, r in enumerate(rollouts)
                if (rel := r.detach_shared(keep_canvas=i == len(rollouts) - 1, release=False)) is not None]
        if rels:
            batch = getattr(type(rels[0]), 'release_all', None)      # (learner/optimizer.py _RingClaim: one lock)
            if batch is not None:
                batch(rels)
            else:
                for rel in rels:
                    rel()
        tr = time.perf_counter() - tr
        mk('release')
        ev = None
        if self.cuda:
            # blocking events: the stager waits on them (slot reuse) for up to an iteration, and a spinning wait
            # burned a host core that the node's actor process needs
            ev = torch.cuda.Event(blocking=True)
            with torch.cuda.stream(self.copy_stream):
                if slot.consumed is not None:
                    self.copy_stream.wait_event(slot.consumed)    # the learner has expanded the slot's last contents
                slot.dev[:nbytes].copy_(slot.host[:nbytes], non_blocking=True)
                ev.record(self.copy_stream)
        slot.uploaded = ev
        mk('upload')
        views = {}
        for name, dt, tail, o, n in layout:
            views[name] = slot.dev[o:o + n].view(dt).view((Lv,) + tail)
        if self.H:
            views['hid'] = slot.dev[hid_off:hid_off + n_seq * 2 * self.H * 4].view(torch.float32).view(n_seq, 2,
                                                                                                       self.H)
        if self.pack:
            views['reset'] = slot.dev[rst_off:rst_off + L]
        views['inv'] = slot.dev[inv_off:inv_off + 4 * L].view(torch.int32)
        mk('views')
        self._prof_done()
        return StagedIteration(rollouts=rollouts, lens=lens, off=off, n_seq=n_seq, L=L, Lv=Lv, gae_mode=gae_mode,
                               views=views, ready=ev, slot=slot_i, stage_s=time.perf_counter() - t0, wait_s=tw,
                               copy_s=tc, release_s=tr, raw=raw)

    def _prof_done(self):
        """DCA_STAGE_PROF=1: accumulate the stage() sections and print their means every 200 iterations (stderr)."""
        m = getattr(self, '_marks', None)
        if not m:
            return
        acc = self.__dict__.setdefault('_prof', {})
        for (_, a, ca), (lab, b, cb) in zip(m, m[1:]):
            w, c = acc.get(lab, (0.0, 0.0))
            acc[lab] = (w + (b - a), c + (cb - ca))
        self._prof_n = getattr(self, '_prof_n', 0) + 1
        if self._prof_n % 100 == 0:
            import sys
            n = self._prof_n
            print('[stage prof] ms/iteration wall/cpu ' + ' '.join(f'{k}={1e3 * w / n:.2f}/{1e3 * c / n:.2f}'
                                                                for k, (w, c) in acc.items()),
                  file=sys.stderr, flush=True)

    # ---- learner thread ----------------------------------------------------------------------------
    def get(self) -> StagedIteration:
        while True:
            try:
                return self.q.get(timeout=0.05)
            except queue.Empty:
                if self.err is not None:
                    raise self.err
                if not self.th.is_alive():
                    raise RuntimeError('experience stager thread exited')

    def expand(self, st: StagedIteration, pad: Dict[str, torch.Tensor]) -> Dict[str, torch.Tensor]:
        """On the current (learner) stream: wait for the upload, scatter the packed valid rows into zeroed padded
        buffers, mark the slot consumed. ``pad`` caches the padded device buffers across iterations."""
        cur = torch.cuda.current_stream(self.device) if self.cuda else None
        if cur is not None:
            cur.wait_event(st.ready)
        v = st.views
        rows = v['rows']
        out = {}
        units = ('units_raw', 'hero') if st.raw else ('units',)
        names = ('env',) + units + ('actions', 'masks', 'logp', 'rewards') + (('values',) if st.gae_mode else ())
        for name in names:
            src = v[name]
            buf = pad.get(name)
            if buf is None or buf.dtype != src.dtype or buf.shape[1:] != src.shape[1:] or buf.shape[0] < st.L:
                buf = pad[name] = torch.empty((max(st.L, 2 * (buf.shape[0] if buf is not None else 0)),) +
                                              tuple(src.shape[1:]), dtype=src.dtype, device=self.device)
            out[name] = buf[:st.L]
        valid = pad.get('valid')
        if valid is None or valid.shape[0] < st.L:
            valid = pad['valid'] = torch.empty(max(st.L, 2 * (valid.shape[0] if valid is not None else 0)),
                                               device=self.device)
        vb = valid[:st.L]
        C = _ops() if self.cuda else None
        if C is not None and 'inv' in v:
            # every field's padded rows and the validity mask in one launch (ops/csrc/ingest.hip)
            C.ingest_scatter([out[n] for n in names], [v[n] for n in names], v['inv'], vb)
        else:
            for name in names:
                out[name].zero_()
                out[name].index_copy_(0, rows, v[name])
            vb.zero_()
            vb.index_fill_(0, rows, 1.0)
        out['valid'] = vb
        if st.raw:
            # GPU featurization of the padded rows (ops/csrc/featurize.hip; padding rows are empty records → zero
            # features, as the featurized path's zero fill)
            raw_t, hero_t = out.pop('units_raw'), out.pop('hero')
            buf = pad.get('units')
            shape = tuple(raw_t.shape[1:2]) + (10,)
            if buf is None or buf.shape[1:] != shape or buf.shape[0] < st.L:
                buf = pad['units'] = torch.empty((max(st.L, 2 * (buf.shape[0] if buf is not None else 0)),) + shape,
                                                 dtype=torch.float32, device=self.device)
            out['units'] = buf[:st.L]
            if C is not None:
                C.featurize_raw(raw_t, hero_t, out['units'])
            else:
                from ..features.raw import featurize_raw_np
                out['units'].copy_(torch.from_numpy(featurize_raw_np(raw_t.numpy(), hero_t.numpy())[0]))
        if 'hid' in v:
            out['hid'] = v['hid'].clone()
        if 'reset' in v:
            out['reset'] = v['reset'].clone()
        slot = self.slots[st.slot]
        if cur is not None:
            ev = torch.cuda.Event(blocking=True)
            ev.record(cur)
            slot.consumed = ev
        slot.free.release()
        return out

    def close(self) -> int:
        """Stop and join the stager; returns the decoded rollouts it had to drop."""
        self.stop.set()
        if self.th is None:
            return 0
        self.th.join(timeout=30.0)
        if self.th.is_alive():
            raise RuntimeError('experience stager thread did not stop')
        dropped = self.lost + (1 if self._carry is not None else 0)
        if self._carry is not None:
            _release_all([self._carry])
        self._carry = None
        while True:
            try:
                dropped += len(self.q.get_nowait().rollouts)
            except queue.Empty:
                break
        return dropped
