"""GPU unit featurization from compact raw records (ops/csrc/featurize.hip, features/raw.py, native/core.h
featurize_one_raw).

* CPU: the native raw records + the numpy oracle of the kernel reproduce the host featurizer's features and handles
  exactly — protobuf path (1v1 / 5v5 synthetic states) and the engine's direct path (SimGame, both teams, 400 steps);
  the python raw path (:func:`featurize_raw_obs`) equals the native one.
* VecEnv(raw=True): the same games as a featurizing VecEnv (same seed, same policy outputs) publish rollouts whose
  ``units_raw`` / ``hero`` featurize to the other's ``units`` exactly, and every other array is byte-identical.
* GPU: the kernel equals the numpy oracle (fp32 / int64 and the fp8 step's fp16 / int32 outputs); the raw-staged
  IEEE-fp32 actor step gives the same log-probs as the host-featurized one (within 1e-5 of torch fp32).
"""
import numpy as np
import pytest
import torch

from dotaclient_amd import native
from dotaclient_amd.constants import LAYOUT_1V1, LAYOUT_5V5, TEAM_DIRE, TEAM_RADIANT
from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config, get_5v5_selfplay_config
from dotaclient_amd.features.featurizer import featurize
from dotaclient_amd.features.raw import featurize_raw_np, featurize_raw_obs
from dotaclient_amd.protos import pb

pytestmark = pytest.mark.skipif(not native.AVAILABLE, reason='native module not built')


def _states(cfg_fn, n_steps=300, seed=0):
    svc = SyntheticDotaService(seed=seed)
    svc.reset_sync(cfg_fn())
    out = []
    for i in range(n_steps):
        for team in (TEAM_RADIANT, TEAM_DIRE):
            o = svc.observe_sync(pb.ObserveConfig(team_id=team))
            if o.status != 0:
                return out
            if i % 7 == 0:
                out.append((o.world_state.SerializeToString(), team))
            svc.act_sync(pb.Actions(actions=pb.CMsgBotWorldState.Actions(), team_id=team))
    return out


def _batch(cfg_fn, players):
    blobs, pids, tids = [], [], []
    for b, team in _states(cfg_fn):
        for p in players[team]:
            blobs.append(b)
            pids.append(p)
            tids.append(team)
    return blobs, pids, tids


CASES = [(get_1v1_selfplay_config, LAYOUT_1V1, {TEAM_RADIANT: [0], TEAM_DIRE: [5]}),
         (get_5v5_selfplay_config, LAYOUT_5V5, {TEAM_RADIANT: [0, 2], TEAM_DIRE: [5, 9]})]


@pytest.mark.parametrize('cfg_fn,layout,players', CASES)
def test_raw_records_featurize_to_the_host_features(cfg_fn, layout, players):
    blobs, pids, tids = _batch(cfg_fn, players)
    counts = list(layout.counts)
    env, units, handles, _ = native.featurize_batch(blobs, pids, tids, counts, 4)
    env_r, hero, raw, handles_r, _ = native.featurize_batch_raw(blobs, pids, tids, counts, 4)
    assert raw.dtype == np.int32 and raw.shape == (len(blobs), layout.max_units, 8)
    np.testing.assert_array_equal(env_r, env)
    np.testing.assert_array_equal(handles_r, handles)
    u, h = featurize_raw_np(raw, hero)
    np.testing.assert_array_equal(u, units)
    np.testing.assert_array_equal(h, handles)
    assert (units != 0).any(axis=-1).sum() > len(blobs)        # real units, not just empty slots
    for i in range(0, len(blobs), 5):                          # the python raw path is the same record
        ws = pb.CMsgBotWorldState.FromString(blobs[i])
        e, hr, rr = featurize_raw_obs(ws, pids[i], tids[i], layout=layout)
        np.testing.assert_array_equal(rr, raw[i])
        np.testing.assert_array_equal(hr, hero[i])
        np.testing.assert_array_equal(e, env[i])
        np.testing.assert_array_equal(featurize(ws, pids[i], tids[i], layout=layout).units, units[i])


def test_engine_raw_path_matches_engine_features():
    from dotaclient_amd.native import _native as N
    cfg = get_1v1_selfplay_config()
    picks = [(p.team_id, p.hero_id, p.control_mode) for p in cfg.hero_picks]
    g = N.SimGame(picks, 7)
    rng = np.random.default_rng(7)
    counts = list(LAYOUT_1V1.counts)
    checked = 0
    for step in range(400):
        for team, pid in ((TEAM_RADIANT, 0), (TEAM_DIRE, 5)):
            env, units, handles = g.featurize(team, pid, counts)
            env_r, hero, raw, handles_r = g.featurize_raw(team, pid, counts)
            u, h = featurize_raw_np(raw, hero)
            np.testing.assert_array_equal(env_r, env)
            np.testing.assert_array_equal(u, units)
            np.testing.assert_array_equal(h, handles)
            np.testing.assert_array_equal(handles_r, handles)
            checked += int((raw[:, 6] & 1).sum())
        g.step([(0, int(rng.integers(3)), float(rng.uniform(-3000, 3000)), float(rng.uniform(-3000, 3000)), -1),
                (5, int(rng.integers(3)), float(rng.uniform(-3000, 3000)), float(rng.uniform(-3000, 3000)), -1)])
        if g.status != 0:
            break
    assert checked > 1000


def _run_vecenv(raw: bool, steps: int = 120, seed: int = 5):
    from dotaclient_amd.native import _native as N
    from dotaclient_amd.transport.codec import decode
    U = LAYOUT_1V1.max_units
    ve = N.VecEnv(4, mode=0, seed=seed, max_dota_time=30.0, rollout_size=25, hidden_stride=0, hidden_size=0,
                  counts=list(LAYOUT_1V1.counts), threads=2, raw=raw)
    S, A = ve.slots, 21 + U
    env = np.zeros((S, 3), np.float32)
    units = np.zeros((S, U, 10), np.float32)
    hero = np.zeros((S, 4), np.float32)
    rawb = np.zeros((S, U, 8), np.int32)
    handles = np.full((S, U), -1, np.int64)
    active = np.zeros(S, np.uint8)
    rng = np.random.default_rng(seed)
    out, feats = [], []
    for _ in range(steps):
        ve.begin_step()
        if raw:
            ve.observe_raw(env, hero, rawb, handles, active)
            feats.append(featurize_raw_np(rawb, hero)[0].copy())
        else:
            ve.observe(env, units, handles, active)
            feats.append(units.copy())
        idx = np.zeros((S, 4), np.int32)
        idx[:, 0] = rng.integers(0, 2, S)
        idx[:, 1:3] = rng.integers(0, 9, (S, 2))
        act = np.zeros((S, A), np.uint8)
        msk = np.ones((S, A), np.uint8)
        ve.act(idx, act, msk, rng.standard_normal(S).astype(np.float32), rng.standard_normal(S).astype(np.float32),
               None, None, handles, 0)
        out += [decode(b) for b in ve.pop_rollouts()]
    # (the worker threads publish in completion order: compare per player, chronologically)
    out.sort(key=lambda r: (r.game_id, r.team_id, r.player_id))
    return out, feats


def test_vecenv_raw_rollouts_match_featurized_rollouts():
    ra, fa = _run_vecenv(False)
    rb, fb = _run_vecenv(True)
    assert len(ra) == len(rb) and len(ra) > 4
    for x, y in zip(fa, fb):
        np.testing.assert_array_equal(x * (np.abs(x).sum(-1, keepdims=True) > 0), y)
    for a, b in zip(ra, rb):
        assert a.units_raw is None and b.units is None and b.units_raw is not None
        u, _ = featurize_raw_np(b.units_raw, b.hero)
        np.testing.assert_array_equal(u, a.units)
        np.testing.assert_array_equal(b.ensure_units().units, a.units)
        for name in ('env', 'actions', 'masks', 'rewards', 'logp', 'values'):
            np.testing.assert_array_equal(getattr(a, name), getattr(b, name))


@pytest.mark.gpu
def test_featurize_kernel_matches_numpy(gpu_ops):
    blobs, pids, tids = _batch(get_1v1_selfplay_config, {TEAM_RADIANT: [0], TEAM_DIRE: [5]})
    env, hero, raw, handles, _ = native.featurize_batch_raw(blobs, pids, tids, list(LAYOUT_1V1.counts), 4)
    want_u, want_h = featurize_raw_np(raw, hero)
    d_raw, d_hero = torch.from_numpy(raw).cuda(), torch.from_numpy(hero).cuda()
    u = torch.empty(raw.shape[:2] + (10,), device='cuda')
    h = torch.empty(raw.shape[:2], dtype=torch.long, device='cuda')
    gpu_ops.featurize_raw(d_raw, d_hero, u, h)
    np.testing.assert_array_equal(u.cpu().numpy(), want_u)
    np.testing.assert_array_equal(h.cpu().numpy(), want_h)
    u16 = torch.empty(raw.shape[:2] + (10,), dtype=torch.float16, device='cuda')
    h32 = torch.empty(raw.shape[:2], dtype=torch.int32, device='cuda')
    gpu_ops.featurize_raw(d_raw, d_hero, u16, h32)
    np.testing.assert_array_equal(u16.cpu().numpy(), want_u.astype(np.float16))
    np.testing.assert_array_equal(h32.cpu().numpy(), want_h.astype(np.int32))
    u2 = torch.empty_like(u)
    gpu_ops.featurize_raw(d_raw, d_hero, u2)                   # handles optional (the learner's ingest)
    assert torch.equal(u2, u)


def _raw_rollout(T, seed, U=40):
    from dotaclient_amd.transport.codec import Rollout
    rng = np.random.default_rng(seed)
    A = 21 + U
    raw = np.zeros((T, U, 8), np.int32)
    f = raw.view(np.float32)
    present = rng.random((T, U)) < 0.4
    f[..., 0:2] = rng.uniform(-7000, 7000, (T, U, 2))
    f[..., 2] = rng.uniform(0, 512, (T, U))
    f[..., 3] = rng.uniform(0, 360, (T, U))
    f[..., 4] = rng.uniform(0, 1, (T, U))
    raw[..., 5] = np.where(rng.random((T, U)) < 0.5, rng.integers(1, 10 ** 6, (T, U)), -1)
    raw[..., 6] = present * (1 | 2 * rng.integers(0, 2, (T, U)) | 4 * rng.integers(0, 2, (T, U)))
    raw[~present] = 0
    hero = np.zeros((T, 4), np.float32)
    hero[:, :2] = rng.uniform(-7000, 7000, (T, 2))
    hero[:, 2] = rng.choice([500.0, 600.0, 3000.0], T)
    act = np.zeros((T, A), np.uint8)
    act[np.arange(T), rng.integers(0, 3, T)] = 1
    r = Rollout(game_id=f'g{seed}', team_id=2, player_id=0, env=rng.standard_normal((T, 3)).astype(np.float32),
                units=None, units_raw=raw, hero=hero, actions=act, masks=act.copy(),
                rewards=rng.standard_normal((T, 9)), weight_version=0, logp=np.zeros(T, np.float32),
                values=np.zeros(T, np.float32))
    return r


def _featurized(r):
    import copy
    c = copy.copy(r)
    c.units, c.units_raw, c.hero = featurize_raw_np(r.units_raw, r.hero)[0], None, None
    return c


def _ingest(device, rollouts):
    from dotaclient_amd.learner.ingest import IngestPipeline
    pl = IngestPipeline(None, 16, 2, 'ppo', 8, device, pack=True)
    st = pl.stage(rollouts)
    x = pl.expand(st, {})
    return st, {k: v.cpu().numpy() for k, v in x.items() if isinstance(v, torch.Tensor)}


def test_ingest_featurizes_raw_rollouts_cpu():
    rs = [_raw_rollout(5, 1), _raw_rollout(20, 2), _raw_rollout(7, 3)]
    st, a = _ingest('cpu', rs)
    assert st.raw
    _, b = _ingest('cpu', [_featurized(r) for r in rs])
    assert set(a) == set(b)
    for k in a:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)
    # a mixed iteration converts its raw rollouts on the host
    st, c = _ingest('cpu', [_raw_rollout(5, 1), _featurized(_raw_rollout(20, 2)), _raw_rollout(7, 3)])
    assert not st.raw
    for k in a:
        np.testing.assert_array_equal(c[k], b[k], err_msg=k)


@pytest.mark.gpu
def test_ingest_featurizes_raw_rollouts_on_gpu(gpu_ops):
    rs = [_raw_rollout(5, 1), _raw_rollout(20, 2), _raw_rollout(7, 3), _raw_rollout(40, 4)]
    st, a = _ingest('cuda', rs)
    assert st.raw
    _, b = _ingest('cuda', [_featurized(r) for r in rs])
    for k in b:
        np.testing.assert_array_equal(a[k], b[k], err_msg=k)


@pytest.mark.gpu
@pytest.mark.parametrize('preset,precision', [('lstm512', 'fp32'), ('lstm512', 'bf16'), ('lstm512', 'fp8'),
                                              ('5v5', 'fp32')])
def test_raw_staged_actor_step_equals_feature_staged(gpu_ops, preset, precision):
    """The actor step fed raw unit records (featurized by the step's first kernel) returns exactly what the step fed
    the host featurizer's features returns — sampled actions, log-probs, values, recurrent state — so the IEEE-fp32
    actor's log-probs keep their 1e-5 bound against torch fp32 (tests/test_actor_gpu.py) on GPU features. (fp8: the
    16-byte records, within the fp16 features' quantisation.)"""
    from dotaclient_amd.actor.batched import _synthetic_states, make_slot_policy
    from dotaclient_amd.models.policy import Policy, get_config
    torch.manual_seed(3)
    cfg = get_config(preset)
    pol = Policy(cfg).cuda().eval()
    n = 64
    kw = {'compact': True} if precision == 'fp8' else {}
    a = make_slot_policy(pol, n, device='cuda', precision=precision, seed=5, **kw)
    b = make_slot_policy(pol, n, device='cuda', precision=precision, seed=5, raw=True, **kw)
    assert b.raw and not a.raw
    lay = cfg.layout
    if cfg.layout.counts[0] > 1:
        states = _states(get_5v5_selfplay_config)
    else:
        st = _synthetic_states(2 * n + 8)
        states = [(x, 2 if j % 2 == 0 else 3) for j, x in enumerate(st)]
    for step in range(4):
        env, units, handles, hero, raw = [], [], [], [], []
        for i in range(n):
            blob, team = states[(i + step * n) % len(states)]
            ws = pb.CMsgBotWorldState.FromString(blob)
            pid = 0 if team == 2 else 5
            f = featurize(ws, pid, team, lay)
            e, hr, rr = featurize_raw_obs(ws, pid, team, layout=lay)
            env.append(f.env); units.append(f.units); handles.append(f.handles); hero.append(hr); raw.append(rr)
        env, units, handles = np.stack(env), np.stack(units), np.stack(handles)
        hero, raw = np.stack(hero), np.stack(raw)
        reset = np.zeros(n, bool)
        if step == 2:
            reset[::3] = True
        oa = a.step(env, units, handles, reset=reset)
        ob = b.step_raw(env, hero, raw, reset=reset)
        if precision == 'fp8':
            # the fp8 step stages the 16-byte records (binary16 fields, fp32 arithmetic): features within its fp16
            # quantisation of the exact ones, so the same actions nearly everywhere and log-probs at fp8 tolerance
            same = (ob['idx'] == oa['idx']).all(1)
            assert same.mean() >= 0.9, (step, same.mean())
            assert np.abs(ob['logp'][same] - oa['logp'][same]).mean() < 2e-2
            continue
        for k in ('idx', 'logp', 'value', 'actions', 'masks'):
            np.testing.assert_array_equal(ob[k], oa[k], err_msg=f'{k} step {step}')
        assert torch.equal(a.hidden()[0], b.hidden()[0])


def test_pack_raw16_native_equals_numpy():
    from dotaclient_amd.features.raw import _pack_raw16_np as pack_raw16
    from dotaclient_amd.native import _native as N
    blobs, pids, tids = _batch(get_1v1_selfplay_config, {TEAM_RADIANT: [0], TEAM_DIRE: [5]})
    _, hero, raw, _, _ = native.featurize_batch_raw(blobs, pids, tids, list(LAYOUT_1V1.counts), 4)
    a, b = N.pack_raw16(raw), pack_raw16(raw)
    np.testing.assert_array_equal(a, b)
    f = np.random.default_rng(0).standard_normal((4096, 8)).astype(np.float32) * np.float32(3e4)
    f[:8] = [[0.0, -0.0, 6e-8, 1e-5, 65504.0, 65520.0, np.inf, 1.0]] * 8    # subnormal / overflow edges
    r = f.view(np.int32)
    np.testing.assert_array_equal(N.pack_raw16(r), pack_raw16(r))


def test_vecenv_raw16_staging_matches_raw_records():
    """observe_raw16 stages the 16-byte form of exactly the records observe_raw writes, and keeps the full records in
    the trajectories (the learner's exact features): the published rollouts are identical."""
    from dotaclient_amd.features.raw import pack_raw16
    from dotaclient_amd.native import _native as N
    from dotaclient_amd.transport.codec import decode
    U = LAYOUT_1V1.max_units
    out = {}
    for mode in ('raw', 'raw16'):
        ve = N.VecEnv(4, mode=0, seed=5, max_dota_time=30.0, rollout_size=25, counts=list(LAYOUT_1V1.counts),
                      threads=2, raw=True)
        S, A = ve.slots, 21 + U
        env, hero = np.zeros((S, 3), np.float32), np.zeros((S, 4), np.float32)
        buf = np.zeros((S, U, 8 if mode == 'raw' else 4), np.int32)
        handles, active = np.full((S, U), -1, np.int64), np.zeros(S, np.uint8)
        rng = np.random.default_rng(5)
        staged, rolls = [], []
        for _ in range(80):
            ve.begin_step()
            getattr(ve, 'observe_' + mode)(env, hero, buf, handles, active)
            staged.append(buf.copy())
            idx = np.zeros((S, 4), np.int32)
            idx[:, 0] = rng.integers(0, 2, S)
            idx[:, 1:3] = rng.integers(0, 9, (S, 2))
            ve.act(idx, np.zeros((S, A), np.uint8), np.ones((S, A), np.uint8), np.zeros(S, np.float32),
                   np.zeros(S, np.float32), None, None, handles, 0)
            rolls += [decode(b) for b in ve.pop_rollouts()]
        rolls.sort(key=lambda r: (r.game_id, r.team_id, r.player_id))
        out[mode] = staged, rolls
    for a, b in zip(out['raw'][0], out['raw16'][0]):
        np.testing.assert_array_equal(pack_raw16(a), b)
    assert len(out['raw'][1]) == len(out['raw16'][1]) > 4
    for a, b in zip(out['raw'][1], out['raw16'][1]):
        np.testing.assert_array_equal(a.units_raw, b.units_raw)


@pytest.mark.gpu
def test_featurize_raw16_kernel_matches_numpy(gpu_ops):
    from dotaclient_amd.features.raw import featurize_raw16_np, pack_raw16
    blobs, pids, tids = _batch(get_1v1_selfplay_config, {TEAM_RADIANT: [0], TEAM_DIRE: [5]})
    env, hero, raw, handles, _ = native.featurize_batch_raw(blobs, pids, tids, list(LAYOUT_1V1.counts), 4)
    r16 = pack_raw16(raw)
    want_u, want_h = featurize_raw16_np(r16, hero)
    u = torch.empty(raw.shape[:2] + (10,), dtype=torch.float16, device='cuda')
    h = torch.empty(raw.shape[:2], dtype=torch.int32, device='cuda')
    gpu_ops.featurize_raw(torch.from_numpy(r16).cuda(), torch.from_numpy(hero).cuda(), u, h)
    got = u.cpu().numpy()
    np.testing.assert_array_equal(h.cpu().numpy(), want_h)
    np.testing.assert_array_equal(want_h, handles.astype(np.int32))
    # fp32 sinf / cosf may differ from numpy's by an ulp: at most one fp16 step on a handful of entries
    d = np.abs(got.astype(np.float32) - want_u.astype(np.float32))
    assert d.max() <= 2e-3 and (d > 0).mean() < 1e-3, (d.max(), (d > 0).mean())
    # against the exact features: the fp16 path's quantisation only
    exact, _ = featurize_raw_np(raw, hero)
    assert np.abs(got.astype(np.float32) - exact).max() < 1e-2


def test_decode_rejects_incomplete_raw_rollouts():
    from dotaclient_amd.transport.codec import CorruptMessage, decode, encode
    r = _raw_rollout(6, 11)
    back = decode(encode(r))
    np.testing.assert_array_equal(back.units_raw, r.units_raw)
    np.testing.assert_array_equal(back.hero, r.hero)
    r.hero = None
    with pytest.raises(CorruptMessage):
        decode(encode(r))
    r = _raw_rollout(6, 11)
    r.units_raw = r.units_raw[:, :, :6].copy()
    with pytest.raises(CorruptMessage):
        decode(encode(r))


def test_optimizer_trains_raw_rollouts_like_featurized_ones(tmp_path):
    """DotaOptimizer on CPU: an iteration fed raw rollouts (featurized by the learner) ends on exactly the weights of
    the same iteration fed the host features."""
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    from dotaclient_amd.transport.broker import InProcBroker
    from dotaclient_amd.transport.codec import encode
    outs = []
    for raw in (True, False):
        br = InProcBroker()
        for i in range(8):
            r = _raw_rollout(24, 100 + i)
            r.actions[:] = 0
            r.actions[:, 0] = 1
            r.masks[:] = 0
            r.masks[:, :3] = 1
            br.publish_experience(encode(r if raw else _featurized(r)))
        cfg = OptimizerConfig(log_dir=str(tmp_path / f'r{int(raw)}'), model='lstm128', epochs=1, seq_per_epoch=4,
                              batch_size=2, seq_len=24, device='cpu', xp_timeout=30, seed=3)
        torch.manual_seed(0)
        opt = DotaOptimizer(cfg, br)
        opt.run(iterations=2)
        outs.append({k: v.detach().clone() for k, v in opt.policy.state_dict().items()})
    for k in outs[0]:
        assert torch.equal(outs[0][k], outs[1][k]), k
