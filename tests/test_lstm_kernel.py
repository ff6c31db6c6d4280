"""XCD-team persistent LSTM recurrence kernels (ops/csrc/lstm_team.hip) vs an fp32 torch ``nn.LSTM`` reference."""
import pytest
import torch

from dotaclient_amd.ops.lstm import team_bwd, team_fwd

pytestmark = pytest.mark.gpu


def gpu_C():
    from dotaclient_amd.ops import require
    return require()

# --- test glue: an nn.LSTM-shaped autograd wrapper around the team kernels (input projection and the weight
# gradients as torch GEMMs, the recurrence forward / backward on lstm_team.hip)
def _mm_f32(a: torch.Tensor, b: torch.Tensor) -> torch.Tensor:
    """bf16 × bf16 → fp32 GEMM (torch, test glue only) — fp32 accumulation and output."""
    return torch.mm(a.to(torch.bfloat16), b.to(torch.bfloat16), out_dtype=torch.float32)


class _Recurrence(torch.autograd.Function):
    @staticmethod
    def forward(ctx, xp, w_hh, h0, c0, err):
        C = gpu_C()
        whh16 = w_hh.detach().to(torch.bfloat16).contiguous()
        B, S, G4 = xp.shape
        H = G4 // 4
        ctx.err = err
        xp4 = xp.view(B, S, 4, H).transpose(2, 3).contiguous()
        hs16, hsf, cs, gates4, hn, cn = team_fwd(C, xp4, whh16, h0, c0, err, True)
        ctx.save_for_backward(gates4, cs, c0, whh16, hs16, h0)
        ctx.mark_non_differentiable(hs16)
        return hsf, hn, cn, hs16

    @staticmethod
    def backward(ctx, dhs, dhn, dcn, _dhs16):
        C = gpu_C()
        gates, cs, c0, whh16, hs16, h0 = ctx.saved_tensors
        B, S, H = cs.shape
        dhs = dhs.contiguous() if dhs is not None else torch.zeros_like(cs)
        dhn = None if dhn is None else dhn.contiguous()
        dcn = None if dcn is None else dcn.contiguous()
        dg4, dh0, dc0 = team_bwd(C, dhs, gates, cs, c0, dhn, dcn, whh16, ctx.err)
        dgates = dg4.permute(0, 1, 3, 2).reshape(B, S, 4 * H)
        hprev = torch.cat([h0.to(torch.bfloat16).unsqueeze(1), hs16[:, :-1]], dim=1).reshape(B * S, H)
        dw_hh = _mm_f32(dgates.reshape(B * S, 4 * H).t(), hprev)
        return dgates, dw_hh, dh0, dc0, None


class _InputProjection(torch.autograd.Function):
    """xp = x·W_ihᵀ + b_ih + b_hh as one bf16 GEMM with fp32 output."""

    @staticmethod
    def forward(ctx, x, w_ih, b_ih, b_hh):
        B, S, I = x.shape
        x2 = x.reshape(B * S, I).to(torch.bfloat16)
        w16 = w_ih.detach().to(torch.bfloat16)
        xp = _mm_f32(x2, w16.t()) + (b_ih + b_hh)
        ctx.save_for_backward(x2, w16)
        ctx.shape = (B, S, I)
        return xp.view(B, S, -1)

    @staticmethod
    def backward(ctx, dxp):
        x2, w16 = ctx.saved_tensors
        B, S, I = ctx.shape
        g2 = dxp.reshape(B * S, -1)
        g16 = g2.to(torch.bfloat16)
        dx = torch.mm(g16, w16, out_dtype=torch.float32).view(B, S, I)
        dw = torch.mm(g16.t(), x2, out_dtype=torch.float32)
        db = g2.sum(0)
        return dx, dw, db, db


def lstm_sequence(x, w_ih, w_hh, b_ih, b_hh, h0, c0, err):
    """Returns (out f32 (B,S,H), h_n (B,H), c_n (B,H), out_bf16 (B,S,H))."""
    xp = _InputProjection.apply(x, w_ih, b_ih, b_hh)
    return _Recurrence.apply(xp, w_hh, h0, c0, err)



def _rel(a, b):
    return ((a - b).norm() / (b.norm() + 1e-12)).item()


@pytest.mark.parametrize('B,S,H', [(5, 37, 128), (8, 64, 512), (24, 20, 256), (40, 16, 512), (64, 8, 128), (100, 9, 512), (300, 5, 128)])
def test_lstm_fwd_bwd_matches_torch(gpu_ops, B, S, H):
    torch.manual_seed(B * 1000 + S)
    dev = 'cuda'
    I = 96
    ref = torch.nn.LSTM(I, H, batch_first=True).to(dev)
    x = torch.randn(B, S, I, device=dev, requires_grad=True)
    h0 = (torch.randn(B, H, device=dev) * 0.3).requires_grad_()
    c0 = (torch.randn(B, H, device=dev) * 0.3).requires_grad_()
    # references computed from the SAME bf16-rounded weights/inputs the kernel consumes
    w_ih, w_hh = ref.weight_ih_l0, ref.weight_hh_l0
    out_ref, (hn_ref, cn_ref) = ref(x, (h0.unsqueeze(0), c0.unsqueeze(0)))
    g_out = torch.randn_like(out_ref)
    g_hn = torch.randn_like(hn_ref[0])
    loss_ref = (out_ref * g_out).sum() + (hn_ref[0] * g_hn).sum() + cn_ref[0].sum()
    gr = torch.autograd.grad(loss_ref, [x, w_ih, w_hh, ref.bias_ih_l0, h0, c0])

    err = torch.zeros(1, dtype=torch.int32, device=dev)
    out, hn, cn, out16 = lstm_sequence(x, w_ih, w_hh, ref.bias_ih_l0, ref.bias_hh_l0, h0, c0, err)
    loss = (out * g_out).sum() + (hn * g_hn).sum() + cn.sum()
    gk = torch.autograd.grad(loss, [x, w_ih, w_hh, ref.bias_ih_l0, h0, c0])
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert _rel(out, out_ref) < 2e-2
    assert _rel(hn, hn_ref[0]) < 2e-2 and _rel(cn, cn_ref[0]) < 2e-2
    assert (out16.float() - out).abs().max().item() < 1e-2
    for name, a, b in zip(['x', 'w_ih', 'w_hh', 'b', 'h0', 'c0'], gk, gr):
        assert _rel(a, b) < 3e-2, (name, _rel(a, b))


def test_lstm_repeat_launch_consistent(gpu_ops):
    """Exchange-buffer re-initialisation: back-to-back launches on the same stream give identical results."""
    torch.manual_seed(0)
    B, S, H = 8, 100, 512
    w_ih = torch.randn(4 * H, 256, device='cuda') * 0.05
    w_hh = torch.randn(4 * H, H, device='cuda') * 0.05
    b = torch.zeros(4 * H, device='cuda')
    x = torch.randn(B, S, 256, device='cuda')
    h0 = torch.zeros(B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    outs = [lstm_sequence(x, w_ih, w_hh, b, b, h0, h0, err)[0] for _ in range(3)]
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert torch.equal(outs[0], outs[1]) and torch.equal(outs[1], outs[2])


def test_team_many_chains_queue(gpu_ops):
    """More chains than XCD teams (B=600 → 19 chains of 32): teams pull chains from the queue; result == torch."""
    torch.manual_seed(1)
    B, S, H, I = 600, 12, 128, 64
    ref = torch.nn.LSTM(I, H, batch_first=True).cuda()
    x = torch.randn(B, S, I, device='cuda')
    h0 = torch.randn(B, H, device='cuda') * 0.1
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    out_t = lstm_sequence(x, ref.weight_ih_l0, ref.weight_hh_l0, ref.bias_ih_l0, ref.bias_hh_l0, h0, h0, err)[0]
    with torch.no_grad():
        out_r = ref(x, (h0.unsqueeze(0), h0.unsqueeze(0)))[0]
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert _rel(out_t, out_r) < 2e-2


@pytest.mark.parametrize('B,S,H,tm', [(8, 40, 512, True), (20, 17, 256, False), (3, 25, 128, True)])
def test_team_folded_bias_bf16_dgates_and_bias_grad(gpu_ops, B, S, H, tm):
    """Folded bias (bias4) == bias added to xp4; bf16 ∂gates == f32 ∂gates rounded; the in-kernel bias gradient
    == Σ over rows and steps of the f32 ∂gates."""
    C = gpu_ops
    torch.manual_seed(7)
    shp = (S, B, H, 4) if tm else (B, S, H, 4)
    xp = torch.randn(*shp, device='cuda') * 0.5
    bias = torch.randn(4 * H, device='cuda') * 0.3
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(torch.bfloat16)
    h0 = torch.randn(B, H, device='cuda') * 0.1
    c0 = torch.randn(B, H, device='cuda') * 0.1
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    ref = team_fwd(C, xp + bias.view(H, 4), whh, h0, c0, err, True, time_major=tm)
    got = team_fwd(C, xp, whh, h0, c0, err, True, time_major=tm, bias4=bias)
    torch.testing.assert_close(got[1], ref[1], atol=1e-5, rtol=1e-5)
    torch.testing.assert_close(got[3], ref[3], atol=1e-5, rtol=1e-5)
    dh = torch.randn(*shp[:3], device='cuda')
    g32 = team_bwd(C, dh, ref[3], ref[2], c0, None, None, whh, err, time_major=tm)
    g16 = team_bwd(C, dh, ref[3], ref[2], c0, None, None, whh, err, time_major=tm, dg_bf16=True, want_dbias=True)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    assert g16[0].dtype == torch.bfloat16
    torch.testing.assert_close(g16[0].float(), g32[0].to(torch.bfloat16).float(), atol=1e-6, rtol=0)
    torch.testing.assert_close(g16[1], g32[1], atol=1e-6, rtol=1e-6)
    # the bias gradient comes in PyTorch's gate-major order (unit-major ∂gates summed, then (H, 4) → (4, H))
    torch.testing.assert_close(g16[3], g32[0].sum((0, 1)).t().reshape(-1), atol=1e-3, rtol=1e-4)


def test_trace_buffers_are_checked_before_launch(gpu_ops):
    """The recurrence kernels stamp timestamps into the optional trace buffer without bounds checks, so the
    bindings reject an undersized or wrong-dtype buffer before launching (bindings.cpp trace_ptr)."""
    from dotaclient_amd import ops
    from dotaclient_amd.ops.lstm import team_ctl
    C = ops.require()
    B, S, H = 8, 4, 128
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    h0 = torch.zeros(B, H, device='cuda')
    xp4 = torch.randn(B, S, H, 4, device='cuda')
    whh = (torch.randn(4 * H, H, device='cuda') * 0.05).to(torch.bfloat16)
    for bad in [torch.zeros(32 * 4 * 64 * 8 - 1, dtype=torch.int64, device='cuda'),
                torch.zeros(32 * 4 * 64 * 8, dtype=torch.int32, device='cuda')]:
        with pytest.raises(RuntimeError, match='trace'):
            C.lstm_team_fwd(xp4, whh, h0, h0, err, team_ctl(), False, bad)
    tr = torch.zeros(32 * 4 * 64 * 8, dtype=torch.int64, device='cuda')
    C.lstm_team_fwd(xp4, whh, h0, h0, err, team_ctl(), False, tr)
    torch.cuda.synchronize()
    assert int(err.item()) == 0 and int((tr != 0).sum().item()) > 0
