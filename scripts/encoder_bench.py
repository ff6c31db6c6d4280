#!/usr/bin/env python3
"""Time the fused entity-encoder kernels (forward / backward incl. the dW_type GEMM) at the learner shape
(N = B·S rows) on one GPU and report effective HBM bandwidth of their compulsory traffic. One JSON line per layout."""
import json
import sys
import time

import torch

sys.path.insert(0, __import__('os').path.dirname(__import__('os').path.dirname(__import__('os').path.abspath(__file__))))
from dotaclient_amd import ops  # noqa: E402


def _time(fn, reps=20):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps


def run(N=11200, counts=(1, 5, 16, 16, 1, 1), f32=False):
    C = ops.require()
    torch.manual_seed(0)
    U = sum(counts)
    d = 'cuda'
    units = torch.randn(N, U, 10, device=d)
    env = torch.randn(N, 3, device=d)
    w1 = torch.randn(128, 10, device=d) * 0.3
    b1 = torch.randn(128, device=d) * 0.1
    wt = (torch.randn(6, 128, 128, device=d) * 0.1).to(torch.float32 if f32 else torch.bfloat16)
    wtT = wt.transpose(1, 2).contiguous()
    bt = torch.randn(6, 128, device=d) * 0.1
    we = torch.randn(128, 3, device=d)
    be = torch.randn(128, device=d)
    cl = list(counts)
    x896, emb, arg = C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, cl, False)
    dtl = torch.randn(N, U, device=d)
    z = torch.randn(N, 160, device=d)
    dx = torch.randn(N, 896, device=d)
    tf = _time(lambda: C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, cl, False))
    tb = _time(lambda: C.encoder_bwd(units, w1, b1, wtT, dtl, z, dx, arg, cl, False))
    e = 4 if f32 else 2
    fwd_bytes = N * U * 40 + N * U * 128 * e + N * 896 * e + N * 768
    # backward incl. the ∂W_τ GEMM: inputs + K-blocked ∂emb/basic images written once and read once
    bwd_bytes = N * U * 40 + N * U * 4 + N * 160 * 4 + N * 896 * 4 + N * 768 + (8 if f32 else 4) * N * U * 256
    print(json.dumps({'N': N, 'counts': cl, 'f32': f32, 'fwd_us': tf * 1e6, 'bwd_incl_dWt_us': tb * 1e6,
                      'fwd_GBps': fwd_bytes / tf / 1e9, 'bwd_GBps': bwd_bytes / tb / 1e9}), flush=True)


if __name__ == '__main__':
    for f in (True, False):
        run(f32=f)
        run(N=11200, counts=(5, 5, 24, 24, 3, 3), f32=f)
