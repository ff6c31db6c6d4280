"""5v5 fp32 attention GEMM shapes on hipBLASLt: QKV projection (716 800 × 128 → 384) and out-projection
(→ 128) variants — bias epilogue vs none, fast-fp32 (allow_tf32) vs exact, transposed output, residual copy."""
import json
import time

import torch


def t(fn, reps=10):
    fn()
    torch.cuda.synchronize()
    t0 = time.perf_counter()
    for _ in range(reps):
        fn()
    torch.cuda.synchronize()
    return (time.perf_counter() - t0) / reps * 1e6


R, D = 716800, 128
x = torch.randn(R, D, device='cuda')
w = torch.randn(3 * D, D, device='cuda')
b = torch.randn(3 * D, device='cuda')
wo = torch.randn(D, D, device='cuda')
bo = torch.randn(D, device='cuda')
o = torch.randn(R, D, device='cuda')
e0 = torch.randn(R, D, device='cuda')
out = torch.empty(R, 3 * D, device='cuda')
outT = torch.empty(3 * D, R, device='cuda')
res = {}
for fast in (True, False):
    torch.backends.cuda.matmul.allow_tf32 = fast
    k = 'fast' if fast else 'exact'
    res[f'qkv_addmm_bias_{k}'] = t(lambda: torch.addmm(b, x, w.t()))
    res[f'qkv_mm_{k}'] = t(lambda: torch.mm(x, w.t(), out=out))
    res[f'qkv_mm_wT_contig_{k}'] = t(lambda: torch.mm(x, w.t().contiguous(), out=out))
    res[f'qkvT_mm_{k}'] = t(lambda: torch.mm(w, x.t(), out=outT))
    res[f'out_addmm_resid_{k}'] = t(lambda: torch.addmm(e0, o, wo.t()))
    res[f'out_addmm_bias_{k}'] = t(lambda: torch.addmm(bo, o, wo.t()))
    res[f'out_addmm_inplace_{k}'] = t(lambda: e0.addmm_(o, wo.t()))
    res[f'dxn_mm_{k}'] = t(lambda: torch.mm(out, w))
res['copy_367MB'] = t(lambda: e0.clone())
print(json.dumps({k: round(v, 1) for k, v in res.items()}, indent=0))
