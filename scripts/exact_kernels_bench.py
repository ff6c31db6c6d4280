"""Standalone timings of the IEEE-fp32 learner's MFMA kernels at the deploy shape (lstm512, B·S = 11 200 rows):
encoder forward / backward (exact), forward chain, ∂X chain, heads stages, the four weight-gradient TN GEMMs and the
5v5 attention block's two (K = 716 800).
python scripts/exact_kernels_bench.py [iters]"""
import sys

import torch

sys.path.insert(0, '.')
from dotaclient_amd import ops  # noqa: E402
from dotaclient_amd.ops.gemm import gemm_tn  # noqa: E402

C = ops.require()
dev = torch.device('cuda')
it = int(sys.argv[1]) if len(sys.argv) > 1 else 20
N, U, H = 11200, 40, 512
g = torch.Generator(device=dev).manual_seed(0)
r = lambda *s: torch.randn(*s, device=dev, generator=g)   # noqa: E731


def timeit(name, fn, flop=None):
    for _ in range(3):
        fn()
    torch.cuda.synchronize()
    e0, e1 = torch.cuda.Event(enable_timing=True), torch.cuda.Event(enable_timing=True)
    e0.record()
    for _ in range(it):
        fn()
    e1.record()
    torch.cuda.synchronize()
    us = e0.elapsed_time(e1) * 1e3 / it
    tf = f'  {flop / us / 1e6:6.1f} TF/s' if flop else ''
    print(f'{name:34s} {us:8.1f} us{tf}', flush=True)


units, env = r(N, U, 10), r(N, 3)
w1, b1, wt, bt, we, be = r(128, 10) * 0.3, r(128) * 0.1, r(6, 128, 128) * 0.1, r(6, 128) * 0.1, r(128, 3), r(128)
counts = [1, 5, 16, 16, 1, 1]
x896, emb, arg = C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, counts, False, exact=True)
timeit('encoder_fwd exact', lambda: C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, counts, False, exact=True),
       2 * N * U * 128 * 138)
timeit('encoder_fwd bf16x3', lambda: C.encoder_fwd(units, env, w1, b1, wt, bt, we, be, counts, False))
wtT = wt.transpose(1, 2).contiguous()
dtl, z, dx = r(N, U), r(N, 256), r(N, 896)
timeit('encoder_bwd exact', lambda: C.encoder_bwd(units, w1, b1, wtT, dtl, z, dx, arg, counts, False, exact=True),
       2 * N * U * 128 * (256 + 20))
timeit('encoder_bwd bf16x3', lambda: C.encoder_bwd(units, w1, b1, wtT, dtl, z, dx, arg, counts, False))
wpre, wih, bpre = r(256, 896) * 0.03, r(2048, 256) * 0.06, r(256) * 0.1
nil = wpre.new_empty(0)
timeit('pre_rnn_chain exact', lambda: C.pre_rnn_chain(x896, wpre, nil, bpre, wih, nil), 2 * N * 256 * (896 + 2048))
dG = r(N, 2048)
x = torch.relu(r(N, 256))
wihT, wpreT = wih.t().contiguous(), wpre.t().contiguous()
timeit('dpre_dx exact', lambda: C.dpre_dx(dG, wihT, nil, x, wpreT, nil), 2 * N * 256 * (896 + 2048))
wcat, bcat = r(256, 512) * 0.04, r(256)
hs = r(N, 512)
timeit('rowmm_out256 exact (heads)', lambda: C.rowmm_out256(hs, wcat, nil, bcat), 2 * N * 256 * 512)
dz = r(N, 256)
wcatT = wcat.t().contiguous()
timeit('rowmm_in256 exact (heads dX)', lambda: C.rowmm_in256(dz, wcatT, nil), 2 * N * 256 * 512)
for nm, (a, b) in {'dW_hh (2048x512)': (dG, hs), 'dW_ih (2048x256)': (dG, x), 'dW_pre (256x896)': (x, x896),
                   'dW_cat (160x512)': (dz[:, :160].contiguous(), hs)}.items():
    out = torch.empty(a.shape[1], b.shape[1], device=dev)
    timeit(f'gemm_tn exact {nm}', lambda: gemm_tn(a, b, out=out, exact=True), 2 * N * a.shape[1] * b.shape[1])
    timeit(f'gemm_tn bf16x3 {nm}', lambda: gemm_tn(a, b, out=out))
# the 5v5 attention weight gradients: K = 716 800 unit rows (11 200 timesteps × 64 slots), skinny outputs
R5 = N * 64
dqkv, xn, o5, de1 = r(R5, 384), r(R5, 128), r(R5, 128), r(R5, 128)
for nm, (a, b) in {'dW_qkv 5v5 (384x128, K=716800)': (dqkv, xn), 'dW_out 5v5 (128x128, K=716800)': (de1, o5)}.items():
    out = torch.empty(a.shape[1], b.shape[1], device=dev)
    timeit(f'gemm_tn exact {nm}', lambda: gemm_tn(a, b, out=out, exact=True), 2 * R5 * a.shape[1] * b.shape[1])
    timeit(f'gemm_tn bf16x3 {nm}', lambda: gemm_tn(a, b, out=out), 2 * R5 * a.shape[1] * b.shape[1])
