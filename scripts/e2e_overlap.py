#!/usr/bin/env python3
"""What runs beside the learner's persistent recurrence in the node loop: from a rocprofv3 ``--kernel-trace`` (csv) of
``bench.py --e2e``, the per-call durations of ``lstm_team_fwd`` / ``lstm_team_bwd`` (median, mean) and, by kernel name
and process, how much of the recurrence's time other kernels overlapped it. ``python scripts/e2e_overlap.py <trace dir>
[--window-s S]``."""
import csv
import glob
import os
import statistics
import sys
from collections import defaultdict


def main():
    path = sys.argv[1]
    win = float(sys.argv[sys.argv.index('--window-s') + 1]) if '--window-s' in sys.argv else 5.0
    ks = []
    for f in glob.glob(f'{path}/**/*kernel_trace.csv', recursive=True):
        pid = os.path.basename(f).split('_')[0]
        for r in csv.DictReader(open(f)):
            ks.append((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'], pid))
    t_end = max(e for _, e, _, _ in ks)
    t0 = t_end - int(win * 1e9)
    ks = [k for k in ks if k[1] > t0]
    rec = [k for k in ks if 'lstm_team' in k[2]]
    learner = rec[0][3] if rec else None
    for tag in ('lstm_team_fwd', 'lstm_team_bwd'):
        d = [(e - s) / 1e3 for s, e, n, _ in rec if tag in n]
        if d:
            print(f'{tag}: {len(d)} calls, median {statistics.median(d):.0f} µs, mean {statistics.mean(d):.0f} µs')
    others = sorted((k for k in ks if 'lstm_team' not in k[2]), key=lambda k: k[0])
    ov = defaultdict(lambda: [0, 0])
    import bisect
    starts = [k[0] for k in others]
    maxdur = max((e - s for s, e, _, _ in others), default=0)
    tot_rec = 0
    for s, e, n, _ in rec:
        tot_rec += e - s
        i = bisect.bisect_left(starts, s - maxdur)
        while i < len(others) and others[i][0] < e:
            a, b = max(s, others[i][0]), min(e, others[i][1])
            if b > a:
                key = ('learner' if others[i][3] == learner else 'actor', others[i][2][:70])
                ov[key][0] += 1
                ov[key][1] += b - a
            i += 1
    print(f'recurrence time in the window: {tot_rec / 1e6:.1f} ms; overlapped by (process, kernel): count, ms')
    for (proc, name), (c, t) in sorted(ov.items(), key=lambda x: -x[1][1])[:25]:
        print(f'  {proc:7s} {t / 1e6:8.1f} ms {c:7d}  {name}')


if __name__ == '__main__':
    main()
