#!/usr/bin/env python3
"""Summarise a rocprofv3 PMC database (rocpd sqlite): mean counter value per kernel (name filter optional).
usage: pmc_summary.py <run_results.db> [substring ...]"""
import sqlite3
import sys
from collections import defaultdict


def main(path, subs):
    db = sqlite3.connect(path)
    acc = defaultdict(lambda: defaultdict(list))
    for name, cn, v in db.execute('select kernel_name, counter_name, value from counters_collection'):
        short = name.replace('(anonymous namespace)::', '').split('(')[0].replace('void ', '')[:60]
        if subs and not any(s in name for s in subs):
            continue
        acc[short][cn].append(v)
    for k, d in acc.items():
        print(k)
        for cn in sorted(d):
            vals = d[cn]
            print(f'    {cn:28s} {sum(vals) / len(vals):16.1f}   (n={len(vals)})')


if __name__ == '__main__':
    main(sys.argv[1], sys.argv[2:])
