#!/usr/bin/env python3
"""Standalone fp32 entity-encoder backward at the 1v1 learner shape (N = 8·1400), for rocprofv3 counter passes:
    rocprofv3 --pmc <counters> -- python scripts/enc_fb_probe.py [reps]"""
import os
import sys

import torch

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from dotaclient_amd import ops  # noqa: E402


def main(reps=3, N=11200, counts=(1, 5, 16, 16, 1, 1)):
    C = ops.require()
    g = torch.Generator(device='cuda').manual_seed(0)
    U = sum(counts)
    units = torch.randn(N, U, 10, device='cuda', generator=g)
    env = torch.randn(N, 3, device='cuda', generator=g)
    w1 = torch.randn(128, 10, device='cuda', generator=g) * 0.3
    b1 = torch.randn(128, device='cuda', generator=g) * 0.1
    wt = torch.randn(6, 128, 128, device='cuda', generator=g) * 0.1
    bt = torch.randn(6, 128, device='cuda', generator=g) * 0.1
    we = torch.randn(128, 3, device='cuda', generator=g)
    be = torch.randn(128, device='cuda', generator=g)
    cl = list(counts)
    _, _, arg = C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, cl, False)
    wtT = wt.transpose(1, 2).contiguous()
    dtl = torch.randn(N, U, device='cuda', generator=g)
    z = torch.randn(N, 160, device='cuda', generator=g)
    dx = torch.randn(N, 896, device='cuda', generator=g)
    for _ in range(reps):
        C.encoder_bwd(units, w1, b1, wtT, dtl, z, dx, arg, cl, False)
    torch.cuda.synchronize()
    print('ok', flush=True)


if __name__ == '__main__':
    main(int(sys.argv[1]) if len(sys.argv) > 1 else 3)
