"""Split-K bf16 TN GEMM (ops/csrc/gemm_tn.hip) vs an fp32 torch reference of the same product."""
import pytest
import torch

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize('M,N,K', [(160, 512, 11200), (2048, 512, 11200), (2048, 256, 1400), (256, 896, 3333),
                                   (64, 128, 40), (8, 8, 1)])
def test_gemm_tn_matches_fp32(gpu_ops, M, N, K):
    from dotaclient_amd.ops.gemm import gemm_tn
    g = torch.Generator(device='cuda').manual_seed(M + N + K)
    a = torch.randn(K, M, device='cuda', generator=g).to(torch.bfloat16)
    b = torch.randn(K, N, device='cuda', generator=g).to(torch.bfloat16)
    ref = a.float().t() @ b.float()
    for _ in range(2):                                   # tile counters must reset for a second launch
        out = gemm_tn(a, b)
        torch.cuda.synchronize()
        torch.testing.assert_close(out, ref, rtol=1e-4, atol=1e-3 * max(1.0, K ** 0.5))


def test_gemm_tn_perm_accumulate_rowsplit_strided(gpu_ops):
    from dotaclient_amd.ops.gemm import gemm_tn
    K, M, N = 5000, 512, 256
    g = torch.Generator(device='cuda').manual_seed(0)
    big = torch.randn(K, M + 64, device='cuda', generator=g).to(torch.bfloat16)
    a = big[:, 32:32 + M]                                # strided view (row stride M + 64)
    b_all = torch.randn(K, N, device='cuda', generator=g).to(torch.bfloat16)
    b0, b = b_all[:8].contiguous(), b_all[8:]
    perm = torch.randperm(M, device='cuda', generator=g).to(torch.int32)
    base = torch.randn(M, N, device='cuda', generator=g)
    out = base.clone()
    gemm_tn(a, b, out=out, perm=perm, accumulate=True, b0=b0)
    ref = base.clone()
    ref[perm.long()] += a.float().t() @ b_all.float()
    torch.cuda.synchronize()
    torch.testing.assert_close(out, ref, rtol=1e-4, atol=0.1)


@pytest.mark.parametrize('M,N,K', [(160, 512, 11200), (256, 896, 300)])
def test_gemm_tn_colsum(gpu_ops, M, N, K):
    """Optional Σ_k A[k, m] (bias gradient) alongside the product, split-K and single-split plans, accumulate."""
    from dotaclient_amd.ops.gemm import gemm_tn
    g = torch.Generator(device='cuda').manual_seed(K)
    a = torch.randn(K, M, device='cuda', generator=g).to(torch.bfloat16)
    b = torch.randn(K, N, device='cuda', generator=g).to(torch.bfloat16)
    cs = torch.full((M,), 0.5, device='cuda')
    out = gemm_tn(a, b, colsum=cs)
    cs2 = torch.full((M,), 0.5, device='cuda')
    gemm_tn(a, b, out=out.clone(), accumulate=True, colsum=cs2)
    torch.cuda.synchronize()
    ref = a.float().sum(0)
    torch.testing.assert_close(cs, ref, rtol=1e-4, atol=1e-2)
    torch.testing.assert_close(cs2, ref + 0.5, rtol=1e-4, atol=1e-2)


@pytest.mark.parametrize('M,N,K', [(160, 512, 11200), (2048, 512, 11200), (256, 896, 3333), (64, 128, 40), (8, 8, 1)])
def test_gemm_tn_exact_matches_fp64(gpu_ops, M, N, K):
    """Exact-fp32 mode (v_mfma_f32_16x16x4_f32, two-level summation): within fp32 round-off of a float64 product —
    at least as close as torch's own fp32 product on the same operands."""
    from dotaclient_amd.ops.gemm import gemm_tn
    g = torch.Generator(device='cuda').manual_seed(M + N + K + 1)
    a = torch.randn(K, M, device='cuda', generator=g)
    b = torch.randn(K, N, device='cuda', generator=g)
    ref = (a.double().t() @ b.double())
    scale = (a.double().abs().t() @ b.double().abs())     # Σ|a·b|: the round-off scale of each output
    for _ in range(2):
        out = gemm_tn(a, b, exact=True)
        torch.cuda.synchronize()
        err = ((out.double() - ref).abs() / scale).max().item()
        assert err < 2e-7 * max(1.0, (K / 32) ** 0.5), err


def test_gemm_tn_exact_perm_accumulate_rowsplit_colsum(gpu_ops):
    from dotaclient_amd.ops.gemm import gemm_tn
    K, M, N = 5000, 512, 256
    g = torch.Generator(device='cuda').manual_seed(3)
    big = torch.randn(K, M + 64, device='cuda', generator=g)
    a = big[:, 32:32 + M]
    b_all = torch.randn(K, N, device='cuda', generator=g)
    b0, b = b_all[:8].contiguous(), b_all[8:]
    perm = torch.randperm(M, device='cuda', generator=g).to(torch.int32)
    base = torch.randn(M, N, device='cuda', generator=g)
    out = base.clone()
    cs = torch.full((M,), 0.5, device='cuda')
    gemm_tn(a, b, out=out, perm=perm, accumulate=True, b0=b0, colsum=cs, exact=True)
    ref = base.double().clone()
    ref[perm.long()] += a.double().t() @ b_all.double()
    csr = torch.full((M,), 0.5, device='cuda', dtype=torch.float64)
    csr[perm.long()] += a.double().sum(0)
    torch.cuda.synchronize()
    torch.testing.assert_close(out.double(), ref, rtol=1e-6, atol=1e-4)
    torch.testing.assert_close(cs.double(), csr, rtol=1e-6, atol=1e-4)
