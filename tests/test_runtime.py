"""Returns/GAE, codec + broker transports, metrics/tfevents/png/checkpoint utilities, actor + learner end-to-end."""
import os
import pickle
import struct
import tempfile
import threading
import time

import numpy as np
import pytest
import torch

from dotaclient_amd.learner.returns import RunningMeanStd, discount, gae
from dotaclient_amd.transport.broker import InProcBroker, TcpBroker, TcpBrokerServer
from dotaclient_amd.transport.codec import Rollout, decode, decode_any, encode
from dotaclient_amd.utils import checkpoint as ckpt
from dotaclient_amd.utils.png import decode_png, encode_png
from dotaclient_amd.utils.tfevents import EventWriter, masked_crc, read_events


def test_discount_matches_lfilter():
    scipy_signal = pytest.importorskip('scipy.signal')
    x = np.random.RandomState(0).randn(300).astype(np.float32)
    ref = scipy_signal.lfilter([1], [1, -0.98], x[::-1], axis=0)[::-1].astype(np.float32)   # optimizer.py:52-53
    np.testing.assert_allclose(discount(x, 0.98), ref, rtol=1e-5, atol=1e-5)


def test_gae_lambda_one_is_discounted_return():
    r = np.random.RandomState(1).randn(50)
    v = np.random.RandomState(2).randn(50)
    adv, ret = gae(r, v, 0.0, 0.9, 1.0, done=True)
    np.testing.assert_allclose(ret, discount(r, 0.9), rtol=1e-5, atol=1e-5)
    adv0, _ = gae(r, v, 0.5, 0.9, 0.0, done=False)
    np.testing.assert_allclose(adv0[:-1], r[:-1] + 0.9 * v[1:] - v[:-1], rtol=1e-5, atol=1e-6)
    assert adv0[-1] == pytest.approx(r[-1] + 0.9 * 0.5 - v[-1], rel=1e-5)


def test_running_mean_std_ema():
    rms = RunningMeanStd(0.99)
    rms.update(np.array([1.0, 3.0]), 2)
    assert rms.mean[2] == 2.0 and rms.std[2] == 1.0
    rms.update(np.array([5.0, 5.0]), 2)
    assert rms.mean[2] == pytest.approx(2.0 * 0.99 + 5.0 * 0.01)
    assert rms.std[2] == pytest.approx(1.0 * 0.99)


def _rollout(T=30, U=40):
    rng = np.random.RandomState(0)
    return Rollout(game_id='g', team_id=2, player_id=0, env=rng.randn(T, 3).astype(np.float32),
                   units=rng.randn(T, U, 10).astype(np.float32), actions=(rng.rand(T, 21 + U) > 0.9).astype(np.uint8),
                   masks=(rng.rand(T, 21 + U) > 0.5).astype(np.uint8), rewards=rng.randn(T, 9), weight_version=7,
                   canvas=np.zeros((256, 256, 3), np.uint8), logp=rng.randn(T).astype(np.float32),
                   values=rng.randn(T).astype(np.float32), hiddens=rng.randn(2, 2, 16).astype(np.float32),
                   hidden_stride=16, bootstrap_value=0.5, done=False)


def test_codec_roundtrip_binary_and_reference_pickle():
    r = _rollout()
    d = decode(encode(r))
    for k in ['env', 'units', 'actions', 'masks', 'rewards', 'logp', 'values', 'hiddens', 'canvas']:
        np.testing.assert_array_equal(getattr(d, k), getattr(r, k))
    assert (d.weight_version, d.bootstrap_value, d.done, d.hidden_stride) == (7, 0.5, False, 16)
    ref = r.to_reference_dict()
    assert set(ref['states']) == {'env', 'allied_heroes', 'enemy_heroes', 'allied_nonheroes', 'enemy_nonheroes',
                                  'allied_towers', 'enemy_towers'}
    assert ref['states']['enemy_heroes'].shape == (30, 5, 10) and ref['actions']['target_unit'].shape == (30, 40)
    back = decode_any(pickle.dumps(ref), allow_pickle=True)
    np.testing.assert_array_equal(back.units, r.units)
    np.testing.assert_array_equal(back.actions, r.actions)


def test_pickle_experience_is_opt_in_and_restricted():
    """Reference pickles are refused unless allowed, and even then only arrays / containers can be built: a
    message that would run code on unpickling is a CorruptMessage, not an exploit."""
    import os
    from dotaclient_amd.transport.codec import CorruptMessage
    ref = _rollout().to_reference_dict()
    with pytest.raises(CorruptMessage):
        decode_any(pickle.dumps(ref))                  # default: DCX1 only

    class Evil:
        def __reduce__(self):
            return (os.system, ('echo pwned > /dev/null',))
    with pytest.raises(CorruptMessage):
        decode_any(pickle.dumps({'game_id': Evil()}), allow_pickle=True)
    with pytest.raises(CorruptMessage):
        decode_any(b'\x80\x04garbage', allow_pickle=True)


def test_inproc_broker_recent_history_and_backpressure():
    b = InProcBroker(maxsize=2, drop_oldest=True)
    for i in range(3):
        b.publish_experience(bytes([i]))
    assert b.xp_queue_size == 2 and b.consume_experience(0.1) == b'\x01'
    b.publish_model(b'm1', 1)
    seen = []
    b.subscribe_model(lambda v, body: seen.append((v, body)))   # late joiner gets the latest immediately
    b.publish_model(b'm2', 2)
    assert seen == [(1, b'm1'), (2, b'm2')]
    assert b.latest_model(newer_than=2) is None and b.latest_model(newer_than=1)[0] == 2


def test_tcp_broker_roundtrip():
    srv = TcpBrokerServer('127.0.0.1', 0).start()
    try:
        cli = TcpBroker('127.0.0.1', srv.port)
        cli.publish_experience(b'x' * 100000)
        assert cli.xp_queue_size == 1
        assert cli.consume_experience(1.0) == b'x' * 100000
        assert cli.consume_experience(0.05) is None
        cli.publish_model(b'weights', 5)
        assert cli.latest_model(newer_than=4) == (5, b'weights')
        got = []
        sub = TcpBroker('127.0.0.1', srv.port)
        sub.subscribe_model(lambda v, body: got.append(v), poll=0.05)
        t0 = time.time()
        while not got and time.time() - t0 < 5:
            time.sleep(0.01)
        assert got and got[0] == 5
        sub.close()
        cli.close()
    finally:
        srv.stop()


def test_png_and_tfevents(tmp_path):
    img = (np.random.RandomState(0).rand(8, 5, 3) * 255).astype(np.uint8)
    np.testing.assert_array_equal(decode_png(encode_png(img)), img)
    w = EventWriter(str(tmp_path))
    w.add_scalar('loss/sum', 1.5, 3)
    w.add_histogram('losses', np.arange(10), 3)
    w.add_image('canvas', img, 3)
    w.close()
    evs = list(read_events(w.path))
    assert len(evs) == 4 and b'loss/sum' in evs[1] and b'canvas' in evs[3]
    # crc32c known-answer: crc32c('123456789') = 0xE3069283
    from dotaclient_amd.utils.tfevents import crc32c
    assert crc32c(b'123456789') == 0xE3069283


def test_checkpoint_naming_and_resume(tmp_path):
    from dotaclient_amd.models.policy import Policy
    p = Policy('compat')
    path, data = ckpt.save_model(p.state_dict(), str(tmp_path), 12)
    assert os.path.basename(path) == 'model_000000012.pt'
    ckpt.save_model(p.state_dict(), str(tmp_path), 3)
    assert ckpt.latest_model(str(tmp_path)).endswith('model_000000012.pt')
    assert ckpt.iteration_from_model_filename(path) == 12
    q = Policy('compat')
    q.load_state_dict(ckpt.load_model_file(path), strict=True)
    for a, b in zip(p.parameters(), q.parameters()):
        assert torch.equal(a, b)


def test_actor_learner_end_to_end_cpu(tmp_path):
    """BASELINE config 1 (plumbing): synthetic games → experience queue → LSTM-128 PPO learner on CPU →
    model publish → actor hot-swap; checkpoint reload equals the in-memory weights; resume continues numbering."""
    from dotaclient_amd.actor.game import Actor
    from dotaclient_amd.actor.runner import PolicyRunner
    from dotaclient_amd.actor.weights import WeightStore
    from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    br = InProcBroker()
    cfg = OptimizerConfig(log_dir=str(tmp_path), model='lstm128', epochs=1, seq_per_epoch=4, batch_size=2,
                          seq_len=32, device='cpu', xp_timeout=60)
    opt = DotaOptimizer(cfg, br)
    ws = WeightStore('lstm128')
    br.subscribe_model(ws.add_bytes)
    runners = {}
    actor = Actor([SyntheticDotaService(seed=s) for s in range(2)], ws,
                  lambda p: runners.setdefault(id(p), PolicyRunner(p, seed=0)), br.publish_experience,
                  get_1v1_selfplay_config, rollout_size=64, max_dota_time=120, hidden_size=128, hidden_stride=32)
    stop = threading.Event()
    th = threading.Thread(target=lambda: [actor.step() for _ in iter(lambda: stop.is_set(), True)], daemon=True)
    th.start()
    try:
        opt.run(iterations=2)
    finally:
        stop.set()
        th.join(timeout=30)
    assert np.isfinite(opt.last_metrics['loss/sum'])
    assert ws.latest_policy.weight_version == 2
    sd = ckpt.load_model_file(os.path.join(str(tmp_path), 'model_000000002.pt'))
    for k, v in opt.policy.state_dict().items():
        assert torch.equal(sd[k], v.cpu())
    opt2 = DotaOptimizer(cfg, br)
    assert opt2.iteration_start == 3
    torch.testing.assert_close(opt2.learner.opt.exp_avg, opt.learner.opt.exp_avg)
