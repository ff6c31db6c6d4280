#!/usr/bin/env python3
"""Cost of sequence packing inside the exact-fp32 team recurrence: forward / backward per-call time at B = 8, S = 1400,
H = 512 with no reset tensor, an all-zero one, and the packed node loop's density (≈2 episode starts per row).
python scripts/reset_probe.py [reps] [path/to/_C.so — A/B against another build of the extension]"""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.lstm import team_ctl  # noqa: E402


def _time(fn, reps):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 10
    C = ops.require()
    if len(sys.argv) > 2:
        import importlib.util
        spec = importlib.util.spec_from_file_location('dotaclient_amd.ops._C', sys.argv[2])
        C = importlib.util.module_from_spec(spec)
        spec.loader.exec_module(C)
    dev = 'cuda'
    B, S, H = 8, 1400, 512
    torch.manual_seed(0)
    whh = torch.randn(4 * H, H, device=dev) * 0.03
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    xp = torch.randn(S, B, H, 4, device=dev) * 0.5
    dh = torch.randn(S, B, H, device=dev)
    sparse = torch.zeros(S, B, dtype=torch.uint8, device=dev)
    for b in range(B):
        for t in (400 + 37 * b, 900 + 23 * b):
            sparse[t, b] = 1
    cases = {'none': None, 'zeros': torch.zeros(S, B, dtype=torch.uint8, device=dev), 'packed': sparse}
    for name, rst in cases.items():
        kw = {'time_major': True, 'reset': rst}
        out = C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True, **kw)
        tf = _time(lambda: C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True, **kw), reps)
        tb = _time(lambda: C.lstm_team_bwd(dh, out[3], out[2], h0, None, None, whh, err, team_ctl(), **kw), reps)
        print(json.dumps({'reset': name, 'fwd_us': round(tf, 1), 'bwd_us': round(tb, 1), 'err': int(err.item())}),
              flush=True)


if __name__ == '__main__':
    main()
