"""Failure paths: corrupted / dropped experience, injected actor crashes under a supervisor, NaN loss
→ raise → resume from the last checkpoint."""
import os
import random
import sys
import time

import numpy as np
import pytest
import torch

from dotaclient_amd.constants import LAYOUT_1V1
from dotaclient_amd.transport.broker import InProcBroker
from dotaclient_amd.transport.codec import CorruptMessage, Rollout, decode, encode
from dotaclient_amd.utils.faults import Faults


def _rollout(i, T=16):
    rng = np.random.default_rng(i)
    U, A = LAYOUT_1V1.max_units, 21 + LAYOUT_1V1.max_units
    act = np.zeros((T, A), np.uint8)
    act[:, 0] = 1
    msk = np.zeros((T, A), np.uint8)
    msk[:, :3] = 1
    return Rollout(game_id=f'g{i}', team_id=2 + i % 2, player_id=0, weight_version=0,
                   env=rng.standard_normal((T, 3)).astype(np.float32),
                   units=rng.standard_normal((T, U, 10)).astype(np.float32), actions=act, masks=msk,
                   rewards=rng.standard_normal((T, 9)), logp=np.full(T, -1.0, np.float32),
                   values=np.zeros(T, np.float32), done=True)


def test_crc_rejects_every_single_byte_flip():
    body = encode(_rollout(0, T=4))
    f = Faults('seed=3')
    for _ in range(50):
        bad = f.corrupt(body)
        with pytest.raises(ValueError):
            decode(bad)
    with pytest.raises(CorruptMessage):
        decode(body[:-7])
    assert decode(body).game_id == 'g0'


def test_corrupted_magic_bytes_are_dropped_not_unpickled(tmp_path):
    """A flipped byte inside the 4 magic bytes used to route the message to pickle.loads (UnpicklingError crashed
    the learner): it must be dropped like any other corrupted message."""
    br = InProcBroker()
    opt = _optimizer(tmp_path, br)
    for i in range(4):
        body = bytearray(encode(_rollout(i)))
        if i == 0:
            body[0] ^= 0x5A                  # byte 0 of the DCX1 magic
        br.publish_experience(bytes(body))
    opt.run(iterations=1)
    assert opt.corrupt_rollouts == 1
    assert np.isfinite(opt.last_metrics['loss/sum'])


def _optimizer(tmp_path, br, **kw):
    from dotaclient_amd.learner.optimizer import DotaOptimizer, OptimizerConfig
    kw.setdefault('xp_timeout', 10)
    cfg = OptimizerConfig(log_dir=str(tmp_path), model='lstm128', epochs=1, seq_per_epoch=2, batch_size=2,
                          seq_len=16, device='cpu', **kw)
    return DotaOptimizer(cfg, br)


@pytest.mark.parametrize('prefetch', [0, 3])
def test_learner_drops_corrupted_messages_and_keeps_training(tmp_path, prefetch):
    br = InProcBroker()
    opt = _optimizer(tmp_path, br, prefetch_rollouts=prefetch)
    f = Faults('seed=1')
    for i in range(6):
        body = encode(_rollout(i))
        br.publish_experience(f.corrupt(body) if i % 3 == 0 else body)
    opt.run(iterations=2)
    assert opt.corrupt_rollouts == 2
    assert np.isfinite(opt.last_metrics['loss/sum'])


def test_actor_drop_and_corrupt_injection(monkeypatch):
    from dotaclient_amd.actor.game import Actor
    from dotaclient_amd.actor.runner import PolicyRunner
    from dotaclient_amd.actor.weights import WeightStore
    from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config
    from dotaclient_amd.models.policy import Policy
    from dotaclient_amd.utils import faults as F
    monkeypatch.setenv('DCA_FAULTS', 'drop_xp=0.5,corrupt_xp=0.5,seed=2')
    ws = WeightStore('compat')
    ws.add(0, Policy('compat').state_dict())
    sent = []
    runners = {}
    actor = Actor([SyntheticDotaService(seed=s) for s in range(2)], ws,
                  lambda p: runners.setdefault(id(p), PolicyRunner(p, seed=0)), sent.append,
                  get_1v1_selfplay_config, rollout_size=16, max_dota_time=30, rng=random.Random(0))
    while actor.games_finished < 2:
        actor.step()
    inj = F.faults().counts
    assert inj.get('drop_xp', 0) > 0 and inj.get('corrupt_xp', 0) > 0
    bad = 0
    for body in sent:
        try:
            decode(body)
        except ValueError:
            bad += 1
    assert bad == inj['corrupt_xp'] and len(sent) + inj['drop_xp'] == actor.rollouts_sent + inj['drop_xp']


def test_actor_crash_injection_raises(monkeypatch):
    from dotaclient_amd.actor.game import Actor
    monkeypatch.setenv('DCA_FAULTS', 'actor_crash=1.0')
    actor = Actor([], None, None, None, None)
    with pytest.raises(RuntimeError, match='injected actor crash'):
        actor.step()


def test_supervisor_restarts_crashing_children(tmp_path):
    from dotaclient_amd.cli.launch import Supervisor
    marker = tmp_path / 'runs'
    crash = [sys.executable, '-c', f"open(r'{marker}', 'a').write('x'); raise SystemExit(3)"]
    ok = [sys.executable, '-c', 'import time; time.sleep(30)']
    sup = Supervisor({'crashy': crash, 'steady': ok}, max_restarts=3).start()
    try:
        deadline = time.time() + 60
        alive = True
        while alive and time.time() < deadline:
            alive = sup.poll()
            time.sleep(0.2)
        assert not alive and sup.failed == ('crashy', 3)
        assert sup.restarts == {'crashy': 3, 'steady': 0}
        assert marker.read_text() == 'xxxx'            # first run + 3 restarts
    finally:
        sup.stop()


def test_nan_loss_raises_then_resume_from_checkpoint(tmp_path, monkeypatch):
    br = InProcBroker()
    for i in range(12):
        br.publish_experience(encode(_rollout(i)))
    opt = _optimizer(tmp_path, br)
    opt.run(iterations=2)                               # checkpoints model_000000001/2
    monkeypatch.setenv('DCA_FAULTS', 'nan_loss_at=3')
    with pytest.raises(ValueError, match='NaN loss'):
        opt.run_iteration(3)
    monkeypatch.delenv('DCA_FAULTS')
    opt2 = _optimizer(tmp_path, br)                     # "restartPolicy: OnFailure" → resume
    assert opt2.iteration_start == 3
    for a, b in zip(opt.policy.state_dict().values(), opt2.policy.state_dict().values()):
        if a.dtype.is_floating_point:
            assert torch.isfinite(b).all()
    opt2.run(iterations=1)
    assert np.isfinite(opt2.last_metrics['loss/sum'])


def test_prefetch_thread_surfaces_the_experience_timeout(tmp_path):
    """Decode-ahead thread: the broker's experience timeout raised on the thread reaches the learner's caller, and
    close() stops the thread."""
    br = InProcBroker()
    opt = _optimizer(tmp_path, br, prefetch_rollouts=2)
    opt.cfg.xp_timeout = 0.2
    with pytest.raises(TimeoutError):
        opt.run(iterations=1)
    assert getattr(opt, '_prefetcher', None) is None


class _HugeView:
    """Pickles as a tensor whose claimed size far exceeds its 4-element storage (``set_`` used to grow
    the storage to fit, so such a message could force an allocation of any size)."""

    def __init__(self, size, stride, offset=0):
        self.size, self.stride, self.offset = size, stride, offset

    def __reduce__(self):
        import collections
        import torch._utils
        st = torch.zeros(4).untyped_storage()
        return (torch._utils._rebuild_tensor_v2,
                (torch.storage.TypedStorage(wrap_storage=st, dtype=torch.float32, _internal=True), self.offset,
                 self.size, self.stride, False, collections.OrderedDict()))


@pytest.mark.parametrize('size,stride,offset', [((1 << 45,), (1,), 0), ((1 << 26, 1, 10), (10, 10, 1), 0),
                                                ((2,), (1,), 3), ((2,), (-1,), 1)])
def test_pickled_tensor_views_beyond_their_storage_are_corrupt(size, stride, offset):
    import pickle
    from dotaclient_amd.transport.codec import decode_any
    body = pickle.dumps({'states': {'env': _HugeView(size, stride, offset)}})
    with pytest.raises(CorruptMessage):
        decode_any(body, allow_pickle=True)


def test_pickled_tensor_views_inside_their_storage_still_decode():
    import pickle
    from dotaclient_amd.transport.codec import _ArrayUnpickler
    import io
    t = torch.arange(12, dtype=torch.float32).view(3, 4)[1:, 1:3]
    out = _ArrayUnpickler(io.BytesIO(pickle.dumps({'x': t}))).load()
    torch.testing.assert_close(out['x'], t)


def test_background_publish_failure_surfaces_on_the_main_thread(tmp_path):
    """with async checkpoints the model publish / file writes run on a writer thread; a failure there must
    raise on the learner's thread (at the next publish or at flush), not vanish."""
    br = InProcBroker()
    opt = _optimizer(tmp_path, br, async_checkpoint=True)
    calls = []

    def broken_publish(body, version):
        calls.append(version)
        raise OSError('publish failed')
    br.publish_model = broken_publish
    for i in range(4):
        br.publish_experience(encode(_rollout(i)))
    with pytest.raises(OSError, match='publish failed'):
        opt.run(iterations=1)                 # run() flushes the writer on the way out
    assert calls == [1]


def test_prefetch_thread_stops_promptly_and_counts_drops(tmp_path):
    """close() must end the decode-ahead thread even when it is waiting on an empty queue (the default
    experience timeout is None), and report decoded rollouts it had to drop."""
    br = InProcBroker()
    opt = _optimizer(tmp_path, br, prefetch_rollouts=8, xp_timeout=None)
    for i in range(5):
        br.publish_experience(encode(_rollout(i)))
    opt.run(iterations=1)                     # consumes 2 of 5; the thread decodes ahead and then blocks
    t0 = time.time()
    opt.close()
    assert time.time() - t0 < 5.0
    assert opt.prefetch_dropped == 3
