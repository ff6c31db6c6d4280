#!/usr/bin/env python3
"""Markdown table of the derived PMC columns from scripts/pmc_step.sh output (sq.txt, fetch.txt, write.txt):

    python scripts/pmc_table.py gpurun_out/pmc_step [--top 16]
"""
import argparse
import collections
import os
import re

ap = argparse.ArgumentParser()
ap.add_argument('dir')
ap.add_argument('--top', type=int, default=16)
a = ap.parse_args()
vals = collections.defaultdict(dict)
for f in ('sq.txt', 'fetch.txt', 'write.txt'):
    cur = None
    for line in open(os.path.join(a.dir, f)):
        m = re.match(r'\s+(\w+)\s+([\d.]+)\s+\(n=(\d+)\)', line)
        if m and cur:
            vals[cur][m.group(1)] = float(m.group(2))
        elif line.strip():
            cur = line.strip()
rows = []
for k, v in vals.items():
    g = v.get('GRBM_GUI_ACTIVE')
    if not g:
        continue
    us = g / 8 / 2.4e3
    cyc = g / 8
    mfma = v.get('SQ_VALU_MFMA_BUSY_CYCLES', 0) / (cyc * 256 * 4) if cyc else 0   # per SIMD (4 per CU)
    lds = v.get('SQ_INSTS_LDS', 0)
    bc = v.get('SQ_LDS_BANK_CONFLICT', 0) / lds if lds else 0
    hit, miss = v.get('TCC_HIT_sum', 0), v.get('TCC_MISS_sum', 0)
    fetch = v.get('FETCH_SIZE', 0) / 1024
    write = v.get('WRITE_SIZE', 0) / 1024
    valu = v.get('SQ_INSTS_VALU', 0)
    rows.append((us, k, mfma, valu, bc, hit / (hit + miss) if hit + miss else 0, fetch, fetch / 1024 / (us * 1e-6) if us else 0,
                 write))
rows.sort(reverse=True)
print('| kernel | µs/dispatch (GRBM/8 @2.4 GHz) | MFMA busy / SIMD-cycles | VALU instr (M) | LDS bank-conflict cycles / '
      'LDS instr | L2 hit | HBM fetch MB | fetch GB/s | write MB |')
print('|---|---:|---:|---:|---:|---:|---:|---:|---:|')
for us, k, mfma, valu, bc, hit, fetch, bw, write in rows[:a.top]:
    print(f'| `{k}` | {us:.0f} | {100 * mfma:.1f}% | {valu / 1e6:.2f} | {bc:.2f} | {100 * hit:.0f}% | {fetch:.1f} | '
          f'{bw:.0f} | {write:.1f} |')
