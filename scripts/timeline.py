#!/usr/bin/env python3
"""Print a per-kernel timeline (start/end µs relative to the first kernel of a window) from a rocprofv3
``--kernel-trace --output-format csv`` run: ``python scripts/timeline.py <dir> [--last N]``."""
import csv
import glob
import sys

path = sys.argv[1]
last = int(sys.argv[sys.argv.index('--last') + 1]) if '--last' in sys.argv else 120
f = sorted(glob.glob(f'{path}/**/*kernel_trace.csv', recursive=True))[0]
rows = list(csv.DictReader(open(f)))
ks = sorted(((int(r['Start_Timestamp']), int(r['End_Timestamp']), r['Kernel_Name'][:60], r.get('Stream_Id', '?'))
             for r in rows))
ks = ks[-last:]
t0 = ks[0][0]
for s, e, n, q in ks:
    print(f'{(s - t0) / 1e3:10.1f} {(e - t0) / 1e3:10.1f} {(e - s) / 1e3:8.1f}  q{q}  {n}')
