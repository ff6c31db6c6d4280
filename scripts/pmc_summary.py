#!/usr/bin/env python3
"""Per-kernel mean counter values from rocprofv3 --pmc sqlite output:  pmc_summary.py <db> [kernel-substring ...]"""
import sqlite3
import sys
from collections import defaultdict

db = sys.argv[1]
keys = sys.argv[2:]
c = sqlite3.connect(db)
acc = defaultdict(lambda: defaultdict(list))
for name, ctr, val, disp in c.execute('select kernel_name, counter_name, value, dispatch_id from counters_collection'):
    short = name.replace('(anonymous namespace)::', '').replace('void ', '').split('(')[0][:60]
    if keys and not any(k in short for k in keys):
        continue
    acc[short][ctr].append(val)
for k, d in acc.items():
    print(k)
    for ctr, v in sorted(d.items()):
        print(f'   {ctr:28s} {sum(v) / len(v):16.0f}  (n={len(v)})')
