"""GIL hand-off latency probe (diagnostics, ``DCA_GIL_PROBE=1`` in the node loop): a daemon thread sleeps 1 ms at a
time and measures how late it gets the interpreter back. When a wake-up is late by more than ``slow_ms`` it records
where every other thread of the process stands right after (``sys._current_frames``): the thread that just gave the
GIL up is usually still inside, or just past, the call that held it. :meth:`report` aggregates the late wake-ups by
(thread name, file:line, function)."""
from __future__ import annotations

import collections
import sys
import threading
import time


class GilProbe:
    def __init__(self, slow_ms: float = 2.0, period_s: float = 0.001):
        self.slow = slow_ms / 1e3
        self.period = period_s
        self.stop = threading.Event()
        self.n = 0
        self.late = []
        self.where = collections.Counter()
        self.th = threading.Thread(target=self._run, name='gil-probe', daemon=True)
        self.th.start()

    def _run(self):
        me = threading.get_ident()
        names = {}
        while not self.stop.is_set():
            t = time.perf_counter()
            time.sleep(self.period)
            d = time.perf_counter() - t - self.period
            self.n += 1
            if d > self.slow:
                self.late.append(d)
                if len(names) != threading.active_count():
                    names = {th.ident: th.name for th in threading.enumerate()}
                for tid, fr in sys._current_frames().items():
                    if tid == me:
                        continue
                    # the innermost frame inside this repository (else the innermost one)
                    f, pick = fr, None
                    while f is not None:
                        if 'dotaclient_amd' in f.f_code.co_filename and pick is None:
                            pick = f
                        f = f.f_back
                    pick = pick or fr
                    self.where[(names.get(tid, str(tid)), f'{pick.f_code.co_filename.split("/")[-1]}:{pick.f_lineno}',
                                pick.f_code.co_name, fr.f_code.co_name)] += 1

    def report(self, top: int = 15) -> str:
        self.stop.set()
        self.th.join(1.0)
        lat = sorted(self.late)
        lines = [f'[gil probe] {self.n} wake-ups, {len(lat)} late > {1e3 * self.slow:.1f} ms, '
                 f'late total {1e3 * sum(lat):.0f} ms, p50/p90/max late {1e3 * lat[len(lat) // 2] if lat else 0:.1f}/'
                 f'{1e3 * lat[int(0.9 * len(lat))] if lat else 0:.1f}/{1e3 * lat[-1] if lat else 0:.1f} ms']
        for (name, loc, fn, inner), c in self.where.most_common(top):
            lines.append(f'[gil probe]   {c:6d}  {name:22s} {loc:28s} {fn}  (innermost: {inner})')
        return '\n'.join(lines)
