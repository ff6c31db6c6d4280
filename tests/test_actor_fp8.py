"""fp8 actor policy step (ops/csrc/actor_fp8.hip, actor/batched.py Fp8ActorPolicy; BASELINE config 5).

* the e4m3 MFMA core against a torch emulation of the same quantisation (per-channel weight scales, per-row
  activation scales, fp8 round trip) in fp32 — a wrong fragment map or quad transpose shows as O(1) errors, the
  tolerance only covers accumulation order and an occasional rounding tie of an intermediate;
* resets (keep = 0) and inactive slots (state untouched) like the bf16 step;
* the fp8 entity encoder (unit-type GEMMs on 16x16x128 f8f6f4) against the same emulation;
* enum-action agreement of the whole graph-captured fp8 step with the bf16 step on the same observations and
  sampling noise ≥ 99 %.
The fragment-order weight layout round-trips on the CPU."""
import numpy as np
import pytest
import torch

from dotaclient_amd.actor.batched import fp8_weight
from dotaclient_amd.models.policy import Policy, get_config


def _unfrag(f, s, N, K):
    # [N/16][K/128][lane = 16·(k%128 // 32) + n%16][k % 32] (the 16x16x128 f8f6f4 operand order)
    q = f.view(N // 16, K // 128, 4, 16, 32).permute(0, 3, 1, 2, 4).reshape(N, K)
    return q.view(torch.float8_e4m3fn).float() * s[:, None]


def test_fp8_weight_fragment_order_roundtrip():
    torch.manual_seed(0)
    w = torch.randn(48, 256)
    f, s = fp8_weight(w)
    back = _unfrag(f, s, 48, 256)
    assert float((back - w).abs().max() / w.abs().max()) < 0.07         # e4m3: 3 mantissa bits
    # exact for values that are e4m3 numbers times the channel scale
    w2 = torch.tensor([[1.0, -2.0, 0.5, 448.0] * 32] * 16)
    f2, s2 = fp8_weight(w2)
    torch.testing.assert_close(_unfrag(f2, s2, 16, 128), w2, rtol=0, atol=0)


def _qrows(x):
    amax = x.abs().amax(1, keepdim=True)
    s = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    return (x / s).to(torch.float8_e4m3fn).float() * s


@pytest.mark.gpu
def test_fp8_core_matches_quantised_emulation(gpu_ops):
    from dotaclient_amd.actor.batched import Fp8ActorPolicy
    torch.manual_seed(0)
    pol = Policy(get_config('lstm512'))
    n = 100                                          # 7 workgroups, the last one partial
    gp = Fp8ActorPolicy(pol, n, device='cuda', use_graph=False)
    w = gp.w
    g = torch.Generator(device='cuda').manual_seed(1)
    x896 = torch.relu(torch.randn(n, 896, device='cuda', generator=g)).to(torch.bfloat16)
    h = torch.randn(n, 512, device='cuda', generator=g) * 0.3
    c = torch.randn(n, 512, device='cuda', generator=g)
    keep = torch.ones(n, device='cuda')
    keep[::7] = 0.0
    active = torch.ones(n, device='cuda')
    active[3::11] = 0.0
    z = torch.empty(n, 160, device='cuda')
    h1, c1 = h.clone(), c.clone()
    gpu_ops.actor_fp8(x896, w['wpre8'], w['spre'], w['bpre32'], w['wg8'], w['sg'], w['bg'], w['wh8'], w['sh8'],
                      w['bh'], h1, c1, keep, z, active)
    torch.cuda.synchronize()
    # emulation
    Wp = _unfrag(w['wpre8'], w['spre'], 256, 896)
    Wg = _unfrag(w['wg8'], w['sg'], 2048, 768)
    Wh = _unfrag(w['wh8'], w['sh8'], 160, 512)
    pre = torch.relu(_qrows(x896.float()) @ Wp.t() + w['bpre32'])
    hk, ck = h * keep[:, None], c * keep[:, None]
    a = _qrows(torch.cat([pre, hk], 1))
    G = (a @ Wg.t() + w['bg']).view(n, 512, 4)              # unit-major gate columns
    cn = torch.sigmoid(G[..., 1]) * ck + torch.sigmoid(G[..., 0]) * torch.tanh(G[..., 2])
    hn = torch.sigmoid(G[..., 3]) * torch.tanh(cn)
    zr = _qrows(hn) @ Wh.t() + w['bh']
    on = active > 0
    rel = lambda a_, b_: float((a_ - b_).norm() / b_.norm())   # noqa: E731
    assert rel(h1[on], hn[on]) < 2e-2, rel(h1[on], hn[on])
    assert rel(c1[on], cn[on]) < 2e-2, rel(c1[on], cn[on])
    assert rel(z[:, :150], zr[:, :150]) < 3e-2, rel(z[:, :150], zr[:, :150])
    # inactive slots: state untouched, except the reset (keep = 0 → zero state) of this step
    off = ~on
    torch.testing.assert_close(h1[off], hk[off], rtol=0, atol=0)
    torch.testing.assert_close(c1[off], ck[off], rtol=0, atol=0)


@pytest.mark.gpu
@pytest.mark.parametrize('dtype,n,per_unit', [(torch.float16, 100, False), (torch.float32, 4096, False),
                                              (torch.float16, 100, True), (torch.float32, 4096, True)])
def test_fp8_encoder_matches_quantised_emulation(gpu_ops, dtype, n, per_unit):
    """The fp8 entity encoder (ops/csrc/actor_fp8.hip: the wave-parallel encoder_fp8w_kernel and the per-unit
    encoder_fp8_kernel) against a torch emulation of the same quantisation: basic per (row, unit) and W_τ per output
    channel in e4m3, fp32 products, bf16 outputs. Pools are the max over the type's units of the emitted emb
    (bitwise: bf16 rounding is monotone)."""
    from dotaclient_amd.actor.batched import fp8_weight
    from dotaclient_amd.models.policy import TYPE_SUFFIX
    torch.manual_seed(0)
    pol = Policy(get_config('lstm512')).cuda()
    cfg = pol.config
    U = cfg.layout.max_units
    counts = list(cfg.layout.counts)
    g = torch.Generator(device='cuda').manual_seed(3)
    units = torch.randn(n, U, 10, device='cuda', generator=g).to(dtype)
    env = torch.randn(n, 3, device='cuda', generator=g)
    P = {k: v.detach().float() for k, v in pol.state_dict().items()}
    wts = [fp8_weight(P[f'affine_unit_{s}.weight']) for s in TYPE_SUFFIX]
    wt8 = torch.cat([q for q, _ in wts]).contiguous()
    st8 = torch.stack([s_ for _, s_ in wts]).contiguous()
    bt = torch.stack([P[f'affine_unit_{s}.bias'] for s in TYPE_SUFFIX]).contiguous()
    x896, emb = gpu_ops.encoder_fp8(units, env, P['affine_unit_basic_stats.weight'].contiguous(),
                                    P['affine_unit_basic_stats.bias'], wt8, st8, bt,
                                    P['affine_env.weight'].contiguous(), P['affine_env.bias'], counts,
                                    per_unit=per_unit)
    torch.cuda.synchronize()
    # emulation
    basic = torch.relu(units.float() @ P['affine_unit_basic_stats.weight'].t() + P['affine_unit_basic_stats.bias'])
    amax = basic.amax(-1, keepdim=True)
    sc = torch.where(amax > 0, amax / 448.0, torch.ones_like(amax))
    qb = (basic / sc).to(torch.float8_e4m3fn).float() * sc
    ref = torch.empty(n, U, 128, device='cuda')
    o = 0
    for t, (q, s_) in enumerate(wts):
        W = _unfrag(q, s_, 128, 128)
        ref[:, o:o + counts[t]] = qb[:, o:o + counts[t]] @ W.t() + bt[t]
        o += counts[t]
    rel = lambda a_, b_: float((a_.float() - b_).norm() / b_.norm())   # noqa: E731
    assert rel(emb, ref) < 1e-2, rel(emb, ref)
    env_ref = torch.relu(env @ P['affine_env.weight'].t() + P['affine_env.bias'])
    assert rel(x896[:, :128], env_ref) < 1e-2
    o = 0
    for t in range(6):
        pool = emb[:, o:o + counts[t]].float().amax(1)
        torch.testing.assert_close(x896[:, 128 + 128 * t:256 + 128 * t].float(), pool, rtol=0, atol=0)
        o += counts[t]


@pytest.mark.gpu
def test_fp8_policy_enum_agreement_with_bf16(gpu_ops):
    from dotaclient_amd.actor.batched import Fp8ActorPolicy, GpuActorPolicy
    torch.manual_seed(0)
    pol = Policy(get_config('lstm512'))
    n = 4096
    U = pol.layout.max_units
    rng = np.random.default_rng(0)
    bf = GpuActorPolicy(pol, n, device='cuda', seed=7)
    f8 = Fp8ActorPolicy(pol, n, device='cuda', seed=7)
    agree, moves = [], []
    for _ in range(3):
        env = rng.standard_normal((n, 3)).astype(np.float32)
        units = rng.standard_normal((n, U, 10)).astype(np.float32)
        handles = np.where(rng.random((n, U)) < 0.5, rng.integers(1, 1000, (n, U)), -1).astype(np.int64)
        o16 = bf.step(env, units, handles)
        o8 = f8.step(env, units, handles)
        agree.append(float((o16['idx'][:, 0] == o8['idx'][:, 0]).mean()))
        moves.append(float((o16['idx'][:, 0] == 1).mean()))
    print('fp8 vs bf16 enum agreement per step', agree, 'move share', moves)
    assert min(agree) >= 0.99, agree


@pytest.mark.gpu
def test_vec_actor_runs_fp8_policy(gpu_ops):
    """The self-play runtime on the fp8 step (fp32 host staging written in place by the native engine): rollouts
    flow, like the bf16 runtime."""
    from dotaclient_amd import native
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    from dotaclient_amd.actor.vec import measure_vec_actor
    torch.manual_seed(0)
    pol = Policy(get_config('lstm512'))
    r = measure_vec_actor(pol, 'cuda', n_games=64, steps=40, warmup=4, threads=4, rollout_size=16,
                          max_dota_time=30.0, precision='fp8')
    assert r['precision'] == 'fp8' and r['steps_per_s'] > 0 and r['rollouts_per_s'] > 0, r


@pytest.mark.parametrize('mode', [0, 1])
def test_core_weight_fragment_order(mode):
    """actor_core.hip fragment order (actor/batched.py frag_weight): element j of lane l in k-group g of column tile
    t is w[16t + (l & 15)][KG·g + (KG/4)·(l >> 4) + j] (KG = 16 fp32 / 32 bf16)."""
    from dotaclient_amd.actor.batched import frag_weight
    torch.manual_seed(0)
    N, K = 48, 64
    w = torch.randn(N, K)
    f = frag_weight(w, mode)
    kg, e = (16, 4) if mode == 0 else (32, 8)
    ref = w if mode == 0 else w.to(torch.bfloat16)
    f = f.view(N // 16, K // kg, 64, e)
    for t, g, l, j in ((0, 0, 0, 0), (1, 2, 37, 3), (2, 1, 63, e - 1), (2, K // kg - 1, 17, 1)):
        g = min(g, K // kg - 1)
        assert f[t, g, l, j] == ref[16 * t + (l & 15), kg * g + (kg // 4) * (l >> 4) + j]
    assert torch.equal(f.flatten().sort().values, ref.flatten().sort().values)
