#!/usr/bin/env python3
"""Flag kernels whose global loads are serialised (a load followed within a few instructions by s_waitcnt vmcnt(0),
i.e. one memory round trip per load) in gfx950 assembly listings:  serial_loads.py a.s [b.s ...]"""
import re
import sys

for path in sys.argv[1:]:
    s = open(path).read()
    for m in re.finditer(r'^(_Z\S+):', s, re.M):
        end = s.find('s_endpgm', m.end())
        lines = [l.strip() for l in s[m.end():end].split('\n') if l.strip() and not l.strip().startswith((';', '.'))]
        loads = serial = 0
        for i, l in enumerate(lines):
            if l.startswith(('global_load', 'buffer_load')):
                loads += 1
                if any(x.startswith('s_waitcnt vmcnt(0)') for x in lines[i + 1:i + 4]):
                    serial += 1
        if serial >= 4:
            print(f'{path.split("/")[-1]:18s} {m.group(1)[:60]:60s} loads {loads:4d} serialised {serial:4d}')
