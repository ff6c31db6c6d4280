#!/usr/bin/env python3
"""Inspect the hottest basic block (most MFMAs) of each kernel in a gfx950 assembly listing:
instruction mix and every vmcnt wait inside it (a vmcnt wait in a loop that also stores waits out those stores).

  hipcc --offload-arch=gfx950 -O3 --cuda-device-only -S x.hip -o x.s && python scripts/asm_loops.py x.s [kernel-substr]
"""
import re
import sys
from collections import Counter


def main():
    s = open(sys.argv[1]).read()
    want = sys.argv[2:]
    for m in re.finditer(r'^(_Z\S+):', s, re.M):
        name = m.group(1)
        if want and not any(w in name for w in want):
            continue
        end = s.find('s_endpgm', m.end())
        body = s[m.end():end].split('\n')
        blocks, cur = [], None
        for ln in body:
            t = ln.strip()
            if re.match(r'^\.LBB\S+:', t):
                cur = [t.split()[0], []]
                blocks.append(cur)
                continue
            if cur is not None and t and not t.startswith(('.', ';')):
                cur[1].append(t)
        if not blocks:
            continue
        big = max(blocks, key=lambda b: sum('mfma' in x for x in b[1]))
        mix = Counter()
        for x in big[1]:
            op = x.split()[0]
            mix['mfma' if 'mfma' in op else 'ds' if op.startswith('ds_') else
                'vmem' if op.startswith(('global_', 'buffer_')) else 'salu' if op.startswith('s_') else 'valu'] += 1
        print(f'{name[:70]} {big[0]} n={len(big[1])} {dict(mix)}')
        print('   vmcnt waits:', [x for x in big[1] if 'vmcnt' in x])


if __name__ == '__main__':
    main()
