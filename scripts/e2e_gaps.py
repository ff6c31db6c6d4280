#!/usr/bin/env python3
"""GPU occupancy of the node loop from a rocprofv3 ``--kernel-trace`` of ``bench.py --e2e`` (learner + actor process on
one GPU): per process the kernel count, summed kernel time and busy time (union of its kernels' intervals), the
device's busy union, and the learner's idle gaps (no learner kernel running) by size — with how much of each gap the
actor's kernels filled. ``python scripts/e2e_gaps.py <trace dir> [--window-s S]`` (the last S seconds, default 6).

The learner is the process that ran the team recurrence (``lstm_team``)."""
import csv
import glob
import sys
from collections import defaultdict


def union(iv):
    iv = sorted(iv)
    out = []
    for s, e in iv:
        if out and s <= out[-1][1]:
            out[-1][1] = max(out[-1][1], e)
        else:
            out.append([s, e])
    return out


def covered(gap, iv_sorted, starts):
    """ns of [gap) covered by the (merged, sorted) intervals."""
    import bisect
    s, e = gap
    i = max(0, bisect.bisect_right(starts, s) - 1)
    tot = 0
    while i < len(iv_sorted) and iv_sorted[i][0] < e:
        a, b = max(s, iv_sorted[i][0]), min(e, iv_sorted[i][1])
        if b > a:
            tot += b - a
        i += 1
    return tot


def main():
    path = sys.argv[1]
    win = float(sys.argv[sys.argv.index('--window-s') + 1]) if '--window-s' in sys.argv else 6.0
    import os
    rows = []
    for f in glob.glob(f'{path}/**/*kernel_trace.csv', recursive=True):
        pid = os.path.basename(f).split('_')[0]          # rocprofv3 writes one <pid>_kernel_trace.csv per process
        rows += [(pid, r) for r in csv.DictReader(open(f))]
    if not rows:
        sys.exit('no kernel_trace.csv under ' + path)
    by = defaultdict(list)
    names = defaultdict(set)
    for p, r in rows:
        s, e = int(r['Start_Timestamp']), int(r['End_Timestamp'])
        by[p].append((s, e, r['Kernel_Name']))
        if 'lstm_team' in r['Kernel_Name']:
            names[p].add('learner')
    t_end = max(e for v in by.values() for _, e, _ in v)
    t0 = t_end - int(win * 1e9)
    learner = next((p for p in by if 'learner' in names[p]), None)
    print(f'window: last {win:.1f} s of the trace; processes: {len(by)}; learner pid {learner}')
    merged = {}
    for p, v in by.items():
        iv = [(max(s, t0), e) for s, e, _ in v if e > t0]
        m = union(iv)
        merged[p] = m
        busy = sum(e - s for s, e in m)
        ksum = sum(e - s for s, e in iv)
        role = 'learner' if p == learner else 'actor'
        print(f'  {role:8s} pid {p}: {len(iv):7d} kernels, summed {ksum / 1e6:9.1f} ms, busy {busy / 1e6:9.1f} ms '
              f'({100 * busy / (win * 1e9):5.1f} %)')
    allm = union([tuple(x) for m in merged.values() for x in m])
    busy = sum(e - s for s, e in allm)
    print(f'  device busy (any process): {busy / 1e6:.1f} ms ({100 * busy / (win * 1e9):.1f} %)')
    dg = [allm[i + 1][0] - allm[i][1] for i in range(len(allm) - 1)]
    print('  device idle gaps: ' + ', '.join(f'[{lo / 1e3:.0f}, {hi / 1e3:.0f}) µs: {sum(1 for g in dg if lo <= g < hi)} / '
                                             f'{sum(g for g in dg if lo <= g < hi) / 1e6:.1f} ms'
                                             for lo, hi in ((0, 20e3), (20e3, 100e3), (100e3, 1e6), (1e6, 1e12))))
    if learner is None:
        return
    lm = merged[learner]
    others = union([tuple(x) for p, m in merged.items() if p != learner for x in m])
    ostarts = [s for s, _ in others]
    gaps = [(lm[i][1], lm[i + 1][0]) for i in range(len(lm) - 1)]
    bins = [(0, 20e3), (20e3, 100e3), (100e3, 500e3), (500e3, 2e6), (2e6, 1e12)]
    print('  learner idle gaps (ns bins): count, total ms, filled by actor kernels ms')
    for lo, hi in bins:
        g = [x for x in gaps if lo <= x[1] - x[0] < hi]
        tot = sum(e - s for s, e in g)
        fill = sum(covered(x, others, ostarts) for x in g)
        print(f'    [{lo / 1e3:7.0f} µs, {hi / 1e3:9.0f} µs): {len(g):6d}  {tot / 1e6:8.1f} ms  {fill / 1e6:8.1f} ms')
    # the learner's heaviest kernels in the window
    agg = defaultdict(lambda: [0, 0])
    for s, e, n in by[learner]:
        if e > t0:
            agg[n][0] += 1
            agg[n][1] += e - max(s, t0)
    print('  learner kernels by time:')
    for n, (c, t) in sorted(agg.items(), key=lambda x: -x[1][1])[:12]:
        print(f'    {t / 1e6:8.1f} ms {c:6d}  {n[:90]}')
    # the learner's longest idle gaps, with the learner kernels on either side
    ks = sorted((s, e, n) for s, e, n in by[learner] if e > t0)
    big = sorted(((ks[i + 1][0] - max(e for _, e, _ in ks[:i + 1][-64:]), i) for i in range(len(ks) - 1)),
                 reverse=True)[:8]
    print('  longest learner gaps (µs): before -> after')
    for g, i in big:
        print(f'    {g / 1e3:8.0f}  {ks[i][2][:50]} -> {ks[i + 1][2][:50]}')


if __name__ == '__main__':
    main()
