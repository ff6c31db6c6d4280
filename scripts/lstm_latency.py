#!/usr/bin/env python3
"""Per-timestep latency of the persistent LSTM recurrence kernels (forward / backward) on one GPU.
Compares hand-off modes; prints one JSON line per configuration."""
import json
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402


def bench(B, S, H, reps=5):
    C = ops.require()
    dev = 'cuda'
    torch.manual_seed(0)
    xp = torch.randn(B, S, 4 * H, device=dev) * 0.5
    whh = (torch.randn(4 * H, H, device=dev) * 0.05).to(torch.bfloat16)
    h0 = torch.zeros(B, H, device=dev)
    err = torch.zeros(1, dtype=torch.int32, device=dev)
    out = C.lstm_fwd(xp, whh, h0, h0, err, True)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        out = C.lstm_fwd(xp, whh, h0, h0, err, True)
    torch.cuda.synchronize()
    tf = (time.perf_counter() - t0) / reps
    dh = torch.randn(B, S, H, device=dev)
    bw = C.lstm_bwd(dh, out[3], out[2], h0, None, None, whh, err)
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        bw = C.lstm_bwd(dh, out[3], out[2], h0, None, None, whh, err)
    torch.cuda.synchronize()
    tb = (time.perf_counter() - t0) / reps
    return {'B': B, 'S': S, 'H': H, 'fwd_us_per_step': tf / S * 1e6, 'bwd_us_per_step': tb / S * 1e6,
            'err': int(err.item())}


if __name__ == '__main__':
    for H in (512, 128):
        for B in (8, 16, 32, 64, 128):
            print(json.dumps(bench(B, 1400, H)), flush=True)
