#!/usr/bin/env python3
"""Per-kernel totals from a rocprofv3 ``--kernel-trace`` database as a markdown table (µs per step = total / steps).

    python scripts/kernel_summary.py gpurun_out/prof/run_results.db --steps 8 [--top 25]
"""
import argparse
import re
import sqlite3
from collections import defaultdict

ap = argparse.ArgumentParser()
ap.add_argument('db')
ap.add_argument('--steps', type=int, required=True, help='learner steps in the profiled run (warmup + timed)')
ap.add_argument('--top', type=int, default=25)
a = ap.parse_args()
c = sqlite3.connect(a.db)
tot, cnt = defaultdict(float), defaultdict(int)
for start, end, name in c.execute('select start, end, name from kernels'):
    n = re.sub(r'\(.*', '', name.replace('(anonymous namespace)::', '')).replace('void ', '')
    if n.startswith('Cijk_'):
        m = re.search(r'Cijk_(\w+?)_.*?(MT\d+x\d+x\d+)', n)
        n = f'hipBLASLt GEMM {m.group(1)} {m.group(2)}' if m else 'hipBLASLt GEMM'
    tot[n] += (end - start) / 1e3
    cnt[n] += 1
all_us = sum(tot.values())
print('| kernel | calls | total µs | µs/step | share |')
print('|---|---:|---:|---:|---:|')
for n, t in sorted(tot.items(), key=lambda kv: -kv[1])[:a.top]:
    print(f'| `{n[:70]}` | {cnt[n]} | {t:.0f} | {t / a.steps:.0f} | {100 * t / all_us:.1f}% |')
print(f'| **all kernels** | | {all_us:.0f} | {all_us / a.steps:.0f} | 100% |')
