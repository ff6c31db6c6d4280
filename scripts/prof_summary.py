#!/usr/bin/env python3
"""Summarise a rocprofv3 ``--kernel-trace --stats`` run (``*_results.db`` or ``*kernel_stats.csv``) into a short
markdown table: per-kernel total / per-call / share, with kernel names shortened. Usage:

    python scripts/prof_summary.py gpurun_out/prof1/run_results.db --steps 4 > profiles/xyz.md
"""
import argparse
import csv
import glob
import os
import re
import sqlite3


def short(name: str) -> str:
    name = name.replace('(anonymous namespace)::', '')
    name = re.sub(r'\(.*', '', name)          # drop argument lists
    if name.startswith('Cijk_'):
        m = re.search(r'MT(\d+x\d+x\d+)', name)
        return f'hipBLASLt GEMM {name[5:21]} MT{m.group(1) if m else "?"}'
    name = name.replace('void ', '').replace('(anonymous namespace)::', '')
    name = re.sub(r'at::native::', '', name)
    return name[:110]


def load(path):
    if path.endswith('.db'):
        c = sqlite3.connect(path)
        return [(r[0], int(r[1]), float(r[2])) for r in c.execute('select name, total_calls, total_duration from top_kernels')]
    rows = []
    with open(path) as f:
        for r in csv.DictReader(f):
            rows.append((r['Name'], int(r['Calls']), float(r['TotalDurationNs']) / 1e3))
    return rows


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument('path')
    ap.add_argument('--steps', type=int, default=1, help='number of training steps in the trace (for per-step µs)')
    ap.add_argument('--top', type=int, default=25)
    a = ap.parse_args()
    p = a.path
    if os.path.isdir(p):
        c = glob.glob(os.path.join(p, '**', '*.db'), recursive=True) + glob.glob(os.path.join(p, '**', '*kernel_stats.csv'), recursive=True)
        p = c[0]
    rows = load(p)
    merged = {}
    for n, calls, tot in rows:
        k = short(n)
        c0, t0 = merged.get(k, (0, 0.0))
        merged[k] = (c0 + calls, t0 + tot)
    total = sum(t for _, t in merged.values())
    print(f'| kernel | calls | total µs | µs/step | share |')
    print('|---|---:|---:|---:|---:|')
    for k, (calls, tot) in sorted(merged.items(), key=lambda kv: -kv[1][1])[:a.top]:
        print(f'| `{k}` | {calls} | {tot:.0f} | {tot / a.steps:.0f} | {100 * tot / total:.1f}% |')
    print(f'| **all kernels** | | {total:.0f} | {total / a.steps:.0f} | 100% |')


if __name__ == '__main__':
    main()
