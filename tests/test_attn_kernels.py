"""5v5 entity-attention kernels — the fused block forward / backward (ops/csrc/attn_block.hip) and the encoder with a
given ∂E0 (ops/csrc/encoder.hip) — vs plain PyTorch fp32 / float64 references of the same ops."""
import pytest
import torch
import torch.nn.functional as F

pytestmark = pytest.mark.gpu

N = 37                       # timestep rows (not a multiple of anything on purpose)
U, D, NH, HD = 64, 128, 4, 32
TYPE_OFF = [0, 5, 10, 34, 58, 61, 64]   # 5v5 layout (5, 5, 24, 24, 3, 3)


def _bf(t):
    return t.to(torch.bfloat16)


def _g(seed):
    return torch.Generator(device='cuda').manual_seed(seed)


def test_encoder_bwd_with_given_demb(gpu_ops):
    """encoder_bwd(demb_in=∂E0): ∂W_τ, ∂W1, ∂b1 of the unit MLP + per-type linear for an arbitrary ∂E0."""
    g = _g(4)
    units = torch.randn(N, U, 10, device='cuda', generator=g)
    w1 = torch.randn(D, 10, device='cuda', generator=g) * 0.3
    b1 = torch.randn(D, device='cuda', generator=g) * 0.1
    wt = torch.randn(6, D, D, device='cuda', generator=g) * 0.1
    demb = _bf(torch.randn(N, U, D, device='cuda', generator=g))
    counts = [TYPE_OFF[t + 1] - TYPE_OFF[t] for t in range(6)]
    wtT16 = _bf(wt).transpose(1, 2).contiguous()
    dummy_q = torch.zeros(N, 160, device='cuda')
    dwt, dw1, db1 = gpu_ops.encoder_bwd(units, w1, b1, wtT16, torch.zeros(N, U, device='cuda'), dummy_q,
                                        torch.zeros(N, 896, device='cuda'),
                                        torch.zeros(N, 6, 128, dtype=torch.uint8, device='cuda'), counts, False,
                                        demb_in=demb)
    W1 = w1.clone().requires_grad_(True)
    B1 = b1.clone().requires_grad_(True)
    WT = wt.clone().requires_grad_(True)
    basic = F.relu(units @ W1.t() + B1)
    embs = [basic[:, TYPE_OFF[t]:TYPE_OFF[t + 1]] @ _bf(WT[t]).float().t() for t in range(6)]
    torch.cat(embs, 1).backward(demb.float())
    for got, ref, name in ((dwt, WT.grad, 'dwt'), (dw1, W1.grad, 'dw1'), (db1, B1.grad, 'db1')):
        assert (got - ref).norm() / ref.norm() < 3e-2, name


def test_exact_encoder_bwd_with_given_demb_matches_fp64(gpu_ops):
    """encoder_bwd(demb_in=∂E0, exact=True) — the 5v5 fp32-exact step's encoder backward (encoder_bwd_x2_kernel
    GIVEN): ∂W_τ, ∂W1, ∂b1 against float64 autograd, within max(2e-6, 2× the torch-fp32 evaluation's own error)
    (∂W1 / ∂b1 sum through the ReLU mask, whose rare near-zero pre-activations both fp32 evaluations may flip)."""
    g = _g(4)
    Nr = 1111
    units = torch.randn(Nr, U, 10, device='cuda', generator=g)
    w1 = torch.randn(D, 10, device='cuda', generator=g) * 0.3
    b1 = torch.randn(D, device='cuda', generator=g) * 0.1
    wt = torch.randn(6, D, D, device='cuda', generator=g) * 0.1
    demb = torch.randn(Nr, U, D, device='cuda', generator=g)
    counts = [TYPE_OFF[t + 1] - TYPE_OFF[t] for t in range(6)]
    dwt, dw1, db1 = gpu_ops.encoder_bwd(units, w1, b1, wt.transpose(1, 2).contiguous(),
                                        torch.zeros(Nr, U, device='cuda'), torch.zeros(Nr, 160, device='cuda'),
                                        torch.zeros(Nr, 896, device='cuda'),
                                        torch.zeros(Nr, 6, 128, dtype=torch.uint8, device='cuda'), counts, False,
                                        demb_in=demb, exact=True)

    def ref(dt):
        W1, B1, WT = (t.to(dt).requires_grad_(True) for t in (w1, b1, wt))
        basic = F.relu(units.to(dt) @ W1.t() + B1)
        torch.cat([basic[:, TYPE_OFF[t]:TYPE_OFF[t + 1]] @ WT[t].t() for t in range(6)], 1).backward(demb.to(dt))
        return {'dwt': WT.grad, 'dw1': W1.grad, 'db1': B1.grad}
    prev = torch.backends.cuda.matmul.allow_tf32
    torch.backends.cuda.matmul.allow_tf32 = False
    try:
        r64, r32 = ref(torch.float64), ref(torch.float32)
    finally:
        torch.backends.cuda.matmul.allow_tf32 = prev
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())   # noqa: E731
    got = {'dwt': dwt, 'dw1': dw1, 'db1': db1}
    errs = {k: (rel(got[k], r64[k]), rel(r32[k], r64[k])) for k in got}
    print('exact encoder bwd (given demb), (fused, torch-fp32) vs fp64:', errs)
    for k, (e, e32) in errs.items():
        assert e <= max(2e-6, 2 * e32), (k, e, e32)


@pytest.mark.parametrize('layout', ['1v1', '5v5'])
def test_encoder_fwd_matches_fp32(gpu_ops, layout):
    """encoder_fwd (LDS-DMA staging, split-bf16 layer 1, per-type MFMA GEMMs, running max/argmax) vs a plain fp32
    PyTorch reference of the same ops (policy.py:97-138): unit embeddings, pools, env embedding, argmax."""
    g = _g(5)
    counts = [1, 5, 16, 16, 1, 1] if layout == '1v1' else [5, 5, 24, 24, 3, 3]
    Uc = sum(counts)
    off = [0]
    for c in counts:
        off.append(off[-1] + c)
    Nr = 75                                          # not a multiple of the 16-row groups on purpose
    units = torch.randn(Nr, Uc, 10, device='cuda', generator=g)
    env = torch.randn(Nr, 3, device='cuda', generator=g)
    w1 = torch.randn(D, 10, device='cuda', generator=g) * 0.3
    b1 = torch.randn(D, device='cuda', generator=g) * 0.1
    wt = torch.randn(6, D, D, device='cuda', generator=g) * 0.1
    bt = torch.randn(6, D, device='cuda', generator=g) * 0.1
    we = torch.randn(D, 3, device='cuda', generator=g)
    be = torch.randn(D, device='cuda', generator=g)
    x896, emb, arg = gpu_ops.encoder_fwd(units, env, w1, b1, _bf(wt), bt, we, be, counts, False)
    basic = torch.relu(units @ w1.t() + b1)                                   # fp32 reference
    ref = torch.cat([basic[:, off[t]:off[t + 1]] @ _bf(wt[t]).float().t() + bt[t] for t in range(6)], 1)
    err = (emb.float() - ref).norm() / ref.norm()
    assert err < 1e-2, float(err)                    # bf16 storage + bf16 layer-2 operand
    torch.testing.assert_close(x896[:, :D].float(), torch.relu(env @ we.t() + be), rtol=1e-2, atol=1e-2)
    for t in range(6):
        seg = ref[:, off[t]:off[t + 1]]
        mx, am = seg.max(1)
        torch.testing.assert_close(x896[:, D + t * D:D + (t + 1) * D].float(), mx, rtol=1e-2, atol=2e-2)
        # argmax must agree wherever the reference maximum is separated from the runner-up by more than rounding
        if seg.shape[1] > 1:
            top2 = seg.topk(2, dim=1).values
            clear = (top2[:, 0] - top2[:, 1]) > 2e-2
            assert torch.equal(arg[:, t].long()[clear], am[clear])


def _block_images(gpu_ops, w, order, exact):
    """Weight images of the block kernels: bf16 hi / lo pairs (bf16x3) or the fp32 image and an empty lo (exact)."""
    if exact:
        return order(w), w.new_empty(0)
    return tuple(order(t) for t in gpu_ops.split_bf16x2(w))


@pytest.mark.parametrize('compat,exact', [(False, False), (True, False), (False, True), (True, True)])
def test_attn_block_fwd_f32_matches_fp64(gpu_ops, compat, exact):
    """Fused fp32 block forward (ops/csrc/attn_block.hip: LN → QKV → attention → out-projection + residual → pools)
    against float64 torch ops of the same block, every saved tensor (Xn, stats, QKV without bias, O, LSE, E1) and
    the pools / argmax; bf16x3 products, or (exact) the IEEE-fp32 twin at a 10× tighter bound."""
    g = _g(5)
    e0 = torch.randn(N * U, D, device='cuda', generator=g) * 1.5 + 0.3
    bout = torch.randn(D, device='cuda', generator=g) * 0.1
    gamma = 1 + 0.1 * torch.randn(D, device='cuda', generator=g)
    beta = 0.1 * torch.randn(D, device='cuda', generator=g)
    wq = torch.randn(3 * D, D, device='cuda', generator=g) * D ** -0.5
    bq = torch.randn(3 * D, device='cuda', generator=g) * 0.2
    wo = torch.randn(D, D, device='cuda', generator=g) * D ** -0.5
    x896 = torch.zeros(N, 896, device='cuda')
    arg = torch.empty(N, 6, 128, dtype=torch.uint8, device='cuda')
    from dotaclient_amd.models.pipelined import _frag_order
    qh, ql = _block_images(gpu_ops, wq, _frag_order, exact)
    oh, ol = _block_images(gpu_ops, wo, _frag_order, exact)
    xn, mu, rs, qkv, o, lse, e1 = gpu_ops.attn_block_fwd(e0, bout, gamma, beta, qh, ql, bq, oh, ol, TYPE_OFF, x896,
                                                         arg, compat, 1e-5)
    torch.cuda.synchronize()
    f = 0.1 if exact else 1.0
    d = lambda t: t.double()   # noqa: E731
    x = d(e0) - d(bout)
    xr = F.layer_norm(x, (D,), d(gamma), d(beta), 1e-5)
    qkv_r = xr @ d(wq).t()
    q, k, v = (qkv_r + d(bq)).view(N, U, 3, NH, HD).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    s = q @ k.transpose(-1, -2) / HD ** 0.5
    o_r = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(N * U, D)
    e1_r = d(e0) + o_r @ d(wo).t()
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())   # noqa: E731
    assert rel(xn, xr) < 1e-6
    torch.testing.assert_close(mu.double(), x.mean(-1), rtol=1e-5, atol=1e-5)
    print('fwd rel errors (qkv, o, e1):', rel(qkv, qkv_r), rel(o, o_r), rel(e1, e1_r))
    assert rel(qkv, qkv_r) < 2e-5 * f
    assert rel(o, o_r) < 3e-5 * f
    torch.testing.assert_close(lse.double(), torch.logsumexp(s, -1), rtol=1e-5 * f, atol=1e-5 * f)
    assert rel(e1, e1_r) < 2e-5 * f
    e = e1_r.view(N, U, D)
    for t in range(6):
        src = 3 if (compat and t == 5) else t
        seg = e[:, TYPE_OFF[src]:TYPE_OFF[src + 1]]
        mx = seg.max(1).values
        torch.testing.assert_close(x896[:, D + t * D:D + (t + 1) * D].double(), mx, rtol=1e-4, atol=1e-4)
        got = e1.view(N, U, D)[:, TYPE_OFF[src]:TYPE_OFF[src + 1]].gather(1, arg[:, t].long().unsqueeze(1)).squeeze(1)
        torch.testing.assert_close(got, x896[:, D + t * D:D + (t + 1) * D], rtol=0, atol=0)   # arg = the kernel's max


@pytest.mark.parametrize('compat,exact', [(False, False), (True, False), (False, True), (True, True)])
def test_attn_block_bwd_f32_matches_fp64(gpu_ops, compat, exact):
    """Fused fp32 block backward (ops/csrc/attn_block.hip: ∂E1 routing → ∂O → attention backward → ∂Xn → LayerNorm
    backward + residual) against float64 autograd through the same block: ∂E1, ∂QKV (pre-bias), ∂E0 and the
    [∂γ | ∂β | per-type ∂b_τ] sums, on the forward kernel's own saved tensors; bf16x3, or (exact) the IEEE-fp32
    twin at a 10× tighter bound."""
    from dotaclient_amd.models.pipelined import _frag_order, _k16_order
    g = _g(7)
    e0 = torch.randn(N * U, D, device='cuda', generator=g) * 1.5 + 0.3
    bout = torch.randn(D, device='cuda', generator=g) * 0.1
    gamma = 1 + 0.1 * torch.randn(D, device='cuda', generator=g)
    beta = 0.1 * torch.randn(D, device='cuda', generator=g)
    wq = torch.randn(3 * D, D, device='cuda', generator=g) * D ** -0.5
    bq = torch.randn(3 * D, device='cuda', generator=g) * 0.2
    wo = torch.randn(D, D, device='cuda', generator=g) * D ** -0.5
    x896 = torch.zeros(N, 896, device='cuda')
    arg = torch.empty(N, 6, 128, dtype=torch.uint8, device='cuda')
    qh, ql = _block_images(gpu_ops, wq, _frag_order, exact)
    oh, ol = _block_images(gpu_ops, wo, _frag_order, exact)
    xn, mu, rs, qkv, o, lse, e1 = gpu_ops.attn_block_fwd(e0, bout, gamma, beta, qh, ql, bq, oh, ol, TYPE_OFF, x896,
                                                         arg, compat, 1e-5)
    f = 0.1 if exact else 1.0
    dtl = torch.randn(N, U, device='cuda', generator=g)
    z = torch.randn(N, 256, device='cuda', generator=g)          # the heads' 256-wide rows; q = z[:, :128]
    dx = torch.randn(N, 896, device='cuda', generator=g)
    toh, tol = _block_images(gpu_ops, wo.t().contiguous(), _frag_order, exact)
    w4h, w4l = _block_images(gpu_ops, wq, _k16_order, exact)
    de1, dqkv, de0, sums = gpu_ops.attn_block_bwd(dtl, z, dx, arg, TYPE_OFF, compat, o, qkv, bq, lse, e0, bout, mu, rs,
                                                  gamma, toh, tol, w4h, w4l, None)
    torch.cuda.synchronize()
    d = lambda t: t.double()   # noqa: E731
    rel = lambda a, b: float((a.double() - b).norm() / b.norm())   # noqa: E731
    # ∂E1 (demb semantics, routed to the forward kernel's argmax)
    de1_r = d(dtl).unsqueeze(-1) * d(z)[:, None, :D]
    for t in range(6):
        src = 3 if (compat and t == 5) else t
        u = TYPE_OFF[src] + arg[:, t].long()
        de1_r.scatter_add_(1, u.unsqueeze(1), d(dx)[:, D + t * D:D + (t + 1) * D].unsqueeze(1))
    de1_r = de1_r.view(N * U, D)
    assert rel(de1, de1_r) < 1e-6
    E0 = d(e0).requires_grad_(True)
    gm, bt = d(gamma).requires_grad_(True), d(beta).requires_grad_(True)
    xr = F.layer_norm(E0 - d(bout), (D,), gm, bt, 1e-5)
    qkv_r = xr @ d(wq).t()
    qkv_r.retain_grad()
    q, k, v = (qkv_r + d(bq)).view(N, U, 3, NH, HD).unbind(2)
    q, k, v = (t.transpose(1, 2) for t in (q, k, v))
    s = q @ k.transpose(-1, -2) / HD ** 0.5
    o_r = (torch.softmax(s, -1) @ v).transpose(1, 2).reshape(N * U, D)
    e1_r = E0 + o_r @ d(wo).t()
    e1_r.backward(de1_r)
    print('bwd rel errors (dqkv, de0, dgamma, dbeta):', rel(dqkv, qkv_r.grad), rel(de0, E0.grad),
          rel(sums[:D], gm.grad), rel(sums[D:2 * D], bt.grad))
    assert rel(dqkv, qkv_r.grad) < 5e-5 * f
    assert rel(de0, E0.grad) < 5e-5 * f
    assert rel(sums[:D], gm.grad) < 5e-5 * f
    assert rel(sums[D:2 * D], bt.grad) < 5e-5 * f
    dbt_r = torch.stack([E0.grad.view(N, U, D)[:, TYPE_OFF[t]:TYPE_OFF[t + 1]].sum((0, 1)) for t in range(6)])
    assert rel(sums[2 * D:].view(6, D), dbt_r) < 5e-5 * f


