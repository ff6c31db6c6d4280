#!/usr/bin/env python3
"""Time the learner step's weight-gradient GEMM shapes (C = Aᵀ·B, K = B·S rows) under different operand layouts on
hipBLASLt, plus the in-tree split-K TN kernel if built: decides which layout the fused step should produce."""
import sys
import time

import torch

sys.path.insert(0, '.')
from dotaclient_amd.models.fused import tn_splitk  # noqa: E402

dev = torch.device('cuda')
K = 11200
shapes = {'dWcat': (160, 512), 'dWhh': (2048, 512), 'dWih': (2048, 256), 'dWpre': (256, 896)}


def timeit(fn, n=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    g = torch.cuda.CUDAGraph()
    with torch.cuda.graph(g):
        for _ in range(n):
            fn()
    g.replay()
    torch.cuda.synchronize()
    t = time.perf_counter()
    g.replay()
    torch.cuda.synchronize()
    return (time.perf_counter() - t) / n * 1e6


C = None
try:
    from dotaclient_amd import ops
    C = ops.require()
except Exception as e:
    print('no ext', e)
for name, (M, N) in shapes.items():
    a = torch.randn(K, M, device=dev).to(torch.bfloat16)
    b = torch.randn(K, N, device=dev).to(torch.bfloat16)
    at, bt = a.t().contiguous(), b.t().contiguous()
    ref = a.float().t() @ b.float()
    res = {}
    res['TN mm(a.t(), b)'] = timeit(lambda: torch.mm(a.t(), b, out_dtype=torch.float32))
    res['NT mm(at, bt.t())'] = timeit(lambda: torch.mm(at, bt.t(), out_dtype=torch.float32))
    res['NN mm(at, b)'] = timeit(lambda: torch.mm(at, b, out_dtype=torch.float32))
    res['TT mm(a.t(), bt.t())'] = timeit(lambda: torch.mm(a.t(), bt.t(), out_dtype=torch.float32))
    res['splitk bmm 2048'] = timeit(lambda: tn_splitk(a, b))
    res['splitk bmm 1400'] = timeit(lambda: tn_splitk(a, b, chunk=1400))
    res['transpose a (copy)'] = timeit(lambda: a.t().contiguous())
    if C is not None and hasattr(C, 'gemm_tn'):
        from dotaclient_amd.ops.gemm import gemm_tn
        out = gemm_tn(a, b)
        err = (out - ref).abs().max().item() / ref.abs().max().item()
        o = torch.empty(M, N, device=dev)
        res[f'dca gemm_tn (rel err {err:.1e})'] = timeit(lambda: gemm_tn(a, b, out=o))
    fl = 2 * M * N * K
    print(f'{name} M={M} N={N} K={K} ({fl / 1e9:.1f} GFLOP)')
    for k, v in res.items():
        print(f'   {k:34s} {v:8.1f} us  {fl / v / 1e6:7.1f} TF/s')
