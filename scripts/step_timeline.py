#!/usr/bin/env python3
"""Kernel-by-kernel timeline of ONE learner step from a rocprofv3 ``--kernel-trace`` database: the kernels between
the last two ``adam_update_kernel`` launches, with start offset, duration, grid and gaps.

    python scripts/step_timeline.py gpurun_out/prof/run_results.db [--step -1]
"""
import argparse
import re
import sqlite3

ap = argparse.ArgumentParser()
ap.add_argument('db')
ap.add_argument('--step', type=int, default=-1, help='which step (python index over adam launches)')
ap.add_argument('--marker', default='adam_update')
a = ap.parse_args()
c = sqlite3.connect(a.db)
rows = c.execute('select start, end, name, grid_x, grid_y, workgroup_x from kernels order by start').fetchall()
ends = [i for i, r in enumerate(rows) if a.marker in r[2]]
k = ends[a.step]
j = ends[a.step - 1] if len(ends) > 1 else 0
t0 = rows[j][1]
busy = 0
prev_end = t0
for r in rows[j + 1:k + 1]:
    n = re.sub(r'\(.*', '', r[2].replace('(anonymous namespace)::', ''))[:80]
    gap = (r[0] - prev_end) / 1e3
    busy += (r[1] - r[0])
    prev_end = max(prev_end, r[1])
    print(f'{(r[0] - t0) / 1e3:9.1f} {(r[1] - r[0]) / 1e3:8.1f} gap{gap:6.1f} {r[3]}x{r[4]}/{r[5]} {n}')
print(f'step span {(rows[k][1] - t0) / 1e3:.1f} us, kernel busy {busy / 1e3:.1f} us, {k - j} kernels')
