"""The XCD-team recurrence beside resident kernels (VERDICT r5 weak #8 / next #5b).

A team is the 32 workgroups of one XCD (one per CU), formed from HW_REG_XCC_ID tickets (ops/csrc/lstm_team.hip
``join_team``); chains are pulled from a queue. When part of one XCD is held by another kernel — an actor replay, a
collective, another process — that XCD's team cannot gather its 32 members: its leader gives up after a bounded wait
(state 2, no error), the other XCDs' teams drain the chain queue, and the results are the SAME bits (a chain's
arithmetic does not depend on which team runs it). ``err = 3`` is raised only when no team processed some chain —
pinned by tests/test_fused_policy.py::test_team_formation_failure_never_reaches_the_weights (DCA_TEAM_FAIL=1)."""
import time

import pytest
import torch

from dotaclient_amd.ops.lstm import team_bwd, team_fwd

pytestmark = pytest.mark.gpu


def _run(C, xp4, whh, h0, c0, bias, dh, err):
    S, B, H, _ = xp4.shape
    fw = team_fwd(C, xp4, whh, h0, c0, err, False, time_major=True, bias4=bias)
    hs, cs, gates = fw[0], fw[2], fw[3]
    bw = team_bwd(C, dh, gates, cs, c0, None, None, whh, err, time_major=True, want_dbias=True)
    return [hs, cs, gates, fw[4], fw[5]] + [t for t in bw if isinstance(t, torch.Tensor)]


@pytest.mark.parametrize('xcd,held', [(3, 24), (0, 31), (7, 12)])
def test_team_recurrence_finishes_on_the_free_xcds_with_identical_bits(gpu_ops, xcd, held):
    C = gpu_ops
    torch.manual_seed(0)
    B, S, H = 8, 300, 512                 # the headline shape's chains: 8 sequences = 8 XCD chains (exact fp32 VALU)
    xp4 = torch.randn(S, B, H, 4, device='cuda') * 0.5
    whh = torch.randn(4 * H, H, device='cuda') * (0.5 / H ** 0.5)
    bias = torch.randn(4 * H, device='cuda') * 0.1
    h0 = torch.randn(B, H, device='cuda') * 0.1
    c0 = torch.randn(B, H, device='cuda') * 0.1
    dh = torch.randn(S, B, H, device='cuda')
    err = torch.zeros(1, dtype=torch.int32, device='cuda')
    ref = _run(C, xp4, whh, h0, c0, bias, dh, err)
    torch.cuda.synchronize()
    assert int(err.item()) == 0
    side = torch.cuda.Stream()
    with torch.cuda.stream(side):
        # 8·held workgroups: `held` of them land on each XCD; those on XCD `xcd` keep their CU (160 KB LDS) for 0.4 s
        seen = C.occupy_xcd(xcd, 8 * held, 0.4, xp4)
    time.sleep(0.05)                      # (the host: the occupying workgroups are resident by now)
    t0 = time.perf_counter()
    got = _run(C, xp4, whh, h0, c0, bias, dh, err)
    torch.cuda.synchronize()
    dt = time.perf_counter() - t0
    assert int(err.item()) == 0, int(err.item())
    on = int((seen == xcd + 1).sum().item())
    assert on >= held // 2, (on, seen.tolist())           # the occupation really sat on that XCD
    for i, (a, b) in enumerate(zip(got, ref)):
        assert torch.equal(a, b), (i, (a - b).abs().max().item())
    print(f'[residency] xcd {xcd}: {on} CUs held; loaded fwd+bwd {1e3 * dt:.1f} ms (includes the hold)')
