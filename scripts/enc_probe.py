#!/usr/bin/env python3
"""Standalone entity-encoder forward/backward at the headline shape (1v1 lstm512: N = 8·1400 rows, U = 40) for
kernel timing and rocprofv3 counter passes:  python scripts/enc_probe.py [reps]"""
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402


def main():
    reps = int(sys.argv[1]) if len(sys.argv) > 1 else 20
    C = ops.require()
    dev = 'cuda'
    g = torch.Generator(device=dev).manual_seed(0)
    N, U = 11200, 40
    counts = [1, 5, 16, 16, 1, 1]
    units = torch.randn(N, U, 10, device=dev, generator=g)
    env = torch.randn(N, 3, device=dev, generator=g)
    w1 = torch.randn(128, 10, device=dev, generator=g) * 0.3
    b1 = torch.randn(128, device=dev, generator=g) * 0.1
    wt = torch.randn(6, 128, 128, device=dev, generator=g) * 0.1
    wt16 = wt.to(torch.bfloat16)
    wtT16 = wt16.transpose(1, 2).contiguous()
    bt = torch.randn(6, 128, device=dev, generator=g) * 0.1
    we = torch.randn(128, 3, device=dev, generator=g)
    be = torch.randn(128, device=dev, generator=g)
    x896, emb, arg = C.encoder_fwd(units, env, w1, b1, wt16, bt, we, be, counts, False)
    dtl = torch.randn(N, U, device=dev, generator=g)
    q = torch.randn(N, 160, device=dev, generator=g)
    dx = torch.randn(N, 896, device=dev, generator=g)
    fwd = lambda: C.encoder_fwd(units, env, w1, b1, wt16, bt, we, be, counts, False)  # noqa: E731
    bwd = lambda: C.encoder_bwd(units, w1, b1, wtT16, dtl, q, dx, arg, counts, False)  # noqa: E731
    for name, fn in (('fwd', fwd), ('bwd', bwd)):
        fn()
        torch.cuda.synchronize()
        t0 = time.perf_counter()
        for _ in range(reps):
            fn()
        torch.cuda.synchronize()
        print(f'encoder_{name}: {(time.perf_counter() - t0) / reps * 1e6:.1f} us/call (incl. launch)', flush=True)


if __name__ == '__main__':
    main()
