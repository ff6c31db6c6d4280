"""Fused pre-RNN ∂X chain (ops/csrc/dx_chain.hip) vs a float64 torch reference of the same two products + ReLU mask:
dpre = (dG·W_ih)⊙[x>0], dx = dpre·W_pre. bf16x3 mode at the fp32 learner's accuracy class, exact mode at fp32
rounding. Shapes: the deploy step (N = 8·1400, 4H = 2048, 256, 896) and a ragged row count."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('N', [11200, 1000])
@pytest.mark.parametrize('exact', [False, True])
def test_dpre_dx_matches_fp64(gpu_ops, N, exact):
    g = torch.Generator(device='cuda').manual_seed(N)
    K1, P, X = 2048, 256, 896
    dG = torch.randn(N, K1, device='cuda', generator=g) * 1e-3
    wihT = torch.randn(P, K1, device='cuda', generator=g) * 0.05
    x = torch.relu(torch.randn(N, P, device='cuda', generator=g))
    wpreT = torch.randn(X, P, device='cuda', generator=g) * 0.05
    for _ in range(2):
        if exact:
            e = wihT.new_empty(0)
            dpre, dx = gpu_ops.dpre_dx(dG, wihT, e, x, wpreT, e)
        else:
            w1h, w1l = gpu_ops.split_bf16x2(wihT, True)       # slab-major images [K/32][rows][32]
            w2h, w2l = gpu_ops.split_bf16x2(wpreT, True)
            back = (w1h.float() + w1l.float()).permute(1, 0, 2).reshape(P, K1)
            torch.testing.assert_close(back, wihT, rtol=2e-5, atol=0)
            h2, l2 = gpu_ops.split_bf16x2(wpreT)                # plain layout: same values, row-major
            torch.testing.assert_close(h2, w2h.permute(1, 0, 2).reshape(X, P), rtol=0, atol=0)
            torch.testing.assert_close(l2, w2l.permute(1, 0, 2).reshape(X, P), rtol=0, atol=0)
            dpre, dx = gpu_ops.dpre_dx(dG, w1h, w1l, x, w2h, w2l)
        torch.cuda.synchronize()
    ref_pre = (dG.double() @ wihT.double().t()) * (x > 0)
    ref_dx = ref_pre @ wpreT.double().t()
    tol = 5e-6 if exact else 3e-5
    for got, ref in ((dpre, ref_pre), (dx, ref_dx)):
        err = (got.double() - ref).abs().max() / ref.abs().max()
        assert err < tol, (float(err), exact)
    assert bool((dpre[x <= 0] == 0).all())                 # the ReLU mask is exact


@pytest.mark.parametrize('N', [11200, 1000])
def test_pre_rnn_chain_matches_fp64(gpu_ops, N):
    """Forward twin (bias + ReLU epilogue): x = relu(x896·W_preᵀ + b), xp = x·W_ihᵀ at the deploy dims."""
    g = torch.Generator(device='cuda').manual_seed(N + 1)
    K1, P, X = 896, 256, 2048
    x896 = torch.relu(torch.randn(N, K1, device='cuda', generator=g))
    wpre = torch.randn(P, K1, device='cuda', generator=g) * K1 ** -0.5
    b = torch.randn(P, device='cuda', generator=g) * 0.1
    wih = torch.randn(X, P, device='cuda', generator=g) * P ** -0.5
    w1h, w1l = gpu_ops.split_bf16x2(wpre, True)
    w2h, w2l = gpu_ops.split_bf16x2(wih, True)
    x, xp = gpu_ops.pre_rnn_chain(x896, w1h, w1l, b, w2h, w2l)
    torch.cuda.synchronize()
    ref_x = torch.relu(x896.double() @ wpre.double().t() + b.double())
    ref_xp = ref_x @ wih.double().t()
    for got, ref in ((x, ref_x), (xp, ref_xp)):
        err = (got.double() - ref).abs().max() / ref.abs().max()
        assert err < 3e-5, float(err)
    assert bool((x >= 0).all())


@pytest.mark.parametrize('N', [11200, 1000])
def test_rowmm_stages_match_fp64(gpu_ops, N):
    """The chain kernel's stages alone: C = A·Wᵀ + b (N, 256) and C = A·Wᵀ (N, X) from A (N, 256) — the heads GEMM
    (W_cat zero-padded to 256 rows) and its ∂X product."""
    g = torch.Generator(device='cuda').manual_seed(N + 2)
    K, X = 512, 512
    a = torch.randn(N, K, device='cuda', generator=g)
    w = torch.randn(256, K, device='cuda', generator=g) * K ** -0.5
    w[160:] = 0.0
    b = torch.randn(256, device='cuda', generator=g)
    b[160:] = 0.0
    z = gpu_ops.rowmm_out256(a, *gpu_ops.split_bf16x2(w, True), b)
    dz = torch.randn(N, 256, device='cuda', generator=g)
    dx = gpu_ops.rowmm_in256(dz, *gpu_ops.split_bf16x2(w.t().contiguous(), True))
    torch.cuda.synchronize()
    ref_z = a.double() @ w.double().t() + b.double()
    ref_dx = dz.double() @ w.double()
    for got, ref in ((z, ref_z), (dx, ref_dx)):
        err = (got.double() - ref).abs().max() / ref.abs().max()
        assert err < 3e-5, float(err)
    assert bool((z[:, 160:] == 0).all())
