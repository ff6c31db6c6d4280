"""Microbenchmark of the fused pre-RNN ∂X chain (ops/csrc/dx_chain.hip) against the library path it replaces
(hipBLASLt ∂pre GEMM + threshold_backward + ∂x896 GEMM) at the deploy shape N = 11 200, 4H = 2048, 256, 896."""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402


def timeit(fn, reps=20):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    a, b = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    a.record()
    for _ in range(reps):
        fn()
    b.record()
    torch.cuda.synchronize()
    return a.elapsed_time(b) / reps * 1e3


if __name__ == '__main__':
    C = ops.require()
    N, K1, P, X = 11200, 2048, 256, 896
    g = torch.Generator(device='cuda').manual_seed(0)
    dG = torch.randn(N, K1, device='cuda', generator=g) * 1e-3
    wihT = torch.randn(P, K1, device='cuda', generator=g) * 0.05
    x = torch.relu(torch.randn(N, P, device='cuda', generator=g))
    wpreT = torch.randn(X, P, device='cuda', generator=g) * 0.05
    wpre = wpreT.t().contiguous()
    torch.backends.cuda.matmul.allow_tf32 = True

    def lib():
        d = torch.ops.aten.threshold_backward(torch.mm(dG, wihT.t()), x, 0)
        return d, d @ wpre
    only = 'fused' in sys.argv
    w1h, w1l = C.split_bf16x2(wihT, True)
    w2h, w2l = C.split_bf16x2(wpreT, True)
    e = wihT.new_empty(0)
    print(f'dpre_dx bf16x3: {timeit(lambda: C.dpre_dx(dG, w1h, w1l, x, w2h, w2l)):.1f} us', flush=True)
    print(f'split_bf16x2 of both weights: {timeit(lambda: (C.split_bf16x2(wihT, True), C.split_bf16x2(wpreT, True))):.1f} us',
          flush=True)
    if not only:
        print(f'dpre_dx exact: {timeit(lambda: C.dpre_dx(dG, wihT, e, x, wpreT, e)):.1f} us', flush=True)
    if not only:
        print(f'library path (fast fp32): {timeit(lib):.1f} us', flush=True)
