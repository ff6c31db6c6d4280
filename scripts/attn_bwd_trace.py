#!/usr/bin/env python3
"""Phase timestamps (s_memrealtime, 10 ns) of the fused fp32 5v5 block backward (ops/csrc/attn_block.hip,
the 5v5 fp32 default; DCA_ATTN_BWD_FUSED=0 selects the chain) at the learner shape N = 11 200 rows: per-phase µs of rows 0-63 (median over rows and
waves) and the kernel time. Phases: 0 ∂E1, 1 ∂O GEMM, 2 attention backward (+ ∂QKV store), 3 ∂Xn partials,
4 LayerNorm backward, 5 the row's LN partial sums."""
import json
import sys

import numpy as np
import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.models.pipelined import _frag_order, _k16_order  # noqa: E402

TYPE_OFF = [0, 5, 10, 34, 58, 61, 64]


def main(N=11200):
    C = ops.require()
    g = torch.Generator(device='cuda').manual_seed(0)
    D = 128
    r = lambda *s: torch.randn(*s, device='cuda', generator=g)   # noqa: E731
    e0 = r(N * 64, D)
    bout, gamma, beta = r(D) * 0.1, 1 + 0.1 * r(D), 0.1 * r(D)
    wq, bq, wo = r(3 * D, D) * D ** -0.5, r(3 * D) * 0.2, r(D, D) * D ** -0.5
    x896 = torch.zeros(N, 896, device='cuda')
    arg = torch.empty(N, 6, 128, dtype=torch.uint8, device='cuda')
    qh, ql = (_frag_order(t) for t in C.split_bf16x2(wq))
    oh, ol = (_frag_order(t) for t in C.split_bf16x2(wo))
    xn, mu, rs, qkv, o, lse, e1 = C.attn_block_fwd(e0, bout, gamma, beta, qh, ql, bq, oh, ol, TYPE_OFF, x896, arg,
                                                   False, 1e-5)
    dtl, z, dx = r(N, 64), r(N, 256), r(N, 896)
    toh, tol = (_frag_order(t) for t in C.split_bf16x2(wo.t().contiguous()))
    w4h, w4l = (_k16_order(t) for t in C.split_bf16x2(wq))
    tr = torch.zeros(64 * 4 * 8, dtype=torch.int64, device='cuda')
    args = (dtl, z, dx, arg, TYPE_OFF, False, o, qkv, bq, lse, e0, bout, mu, rs, gamma, toh, tol, w4h, w4l)
    for _ in range(2):
        C.attn_block_bwd(*args, None)
    ev = [torch.cuda.Event(enable_timing=True) for _ in range(2)]
    ev[0].record()
    for _ in range(5):
        C.attn_block_bwd(*args, None)
    ev[1].record()
    torch.cuda.synchronize()
    C.attn_block_bwd(*args, tr)
    torch.cuda.synchronize()
    t = tr.view(64, 4, 8).cpu().numpy().astype(np.float64) * 10.0          # ns (100 MHz counter)
    out = {'N': N, 'kernel_ms': ev[0].elapsed_time(ev[1]) / 5}
    names = ['demb', 'dO_gemm', 'attention', 'dxn_partials', 'ln_bwd', 'ln_partials']
    for k, nm in enumerate(names):
        out[nm + '_us'] = float(np.median(t[:, :, k + 1] - t[:, :, k])) / 1e3
    out['row_us'] = float(np.median(t[:, :, 6] - t[:, :, 0])) / 1e3
    print(json.dumps(out), flush=True)


if __name__ == '__main__':
    main()
