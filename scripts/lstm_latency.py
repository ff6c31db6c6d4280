#!/usr/bin/env python3
"""Per-timestep latency of the persistent LSTM recurrence kernels (forward / backward) on one GPU, for both kernel
family (the XCD-local team kernels). Prints one JSON line per configuration."""
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
    return (time.perf_counter() - t0) / reps


def bench(B, S, H, reps=5, impl='team'):
    C = ops.require()
    dev = 'cuda'
    torch.manual_seed(0)
    whh = (torch.randn(4 * H, H, device=dev) * 0.05).to(torch.bfloat16)
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    dh = torch.randn(B, S, H, device=dev)
    xp = torch.randn(B, S, H, 4, device=dev) * 0.5
    out = C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True)
    tf = _time(lambda: C.lstm_team_fwd(xp, whh, h0, h0, err, team_ctl(), True), reps)
    tb = _time(lambda: C.lstm_team_bwd(dh, out[3], out[2], h0, None, None, whh, err, team_ctl()), reps)
    return {'impl': impl, 'B': B, 'S': S, 'H': H, 'fwd_us_per_step': tf / S * 1e6, 'bwd_us_per_step': tb / S * 1e6,
            'err': int(err.item())}


if __name__ == '__main__':
    impls = sys.argv[1:] or ['team']
    for impl in impls:
        for H in (512, 128):
            for B in (8, 16, 32, 64, 128, 256):
                if impl == 'ring' and B > 128:
                    continue
                print(json.dumps(bench(B, 1400, H, impl=impl)), flush=True)
