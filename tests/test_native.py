"""Native host runtime: C++ protobuf featurizer vs the python featurizer, shm ring (incl. multi-process), crc32c."""
import multiprocessing as mp
import os
import uuid

import numpy as np
import pytest

from dotaclient_amd import native
from dotaclient_amd.constants import LAYOUT_1V1, LAYOUT_5V5, TEAM_DIRE, TEAM_RADIANT
from dotaclient_amd.env import SyntheticDotaService, get_1v1_selfplay_config, get_5v5_selfplay_config
from dotaclient_amd.features.featurizer import featurize
from dotaclient_amd.protos import FIELD_NUMBERS, pb

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


def test_field_numbers_match_cpp_decoder():
    # the C++ decoder hard-codes these numbers (native/featurizer.cpp parse_unit / parse_world)
    assert FIELD_NUMBERS['WorldState']['dota_time'] == 3 and FIELD_NUMBERS['WorldState']['units'] == 11
    u = FIELD_NUMBERS['Unit']
    assert (u['handle'], u['unit_type'], u['name'], u['team_id'], u['location'], u['is_alive'], u['player_id']) == \
        (1, 2, 3, 4, 6, 7, 8)
    assert (u['facing'], u['health'], u['health_max'], u['attack_range'], u['attack_target_handle'],
            u['anim_activity'], u['is_invulnerable'], u['is_attack_immune'],
            u['incoming_tracking_projectiles']) == (11, 20, 21, 30, 35, 40, 50, 51, 70)
    assert FIELD_NUMBERS['Projectile'] == {'caster_handle': 1, 'location': 2, 'is_attack': 4}


@pytest.mark.parametrize('cfg_fn,layout,players', [(get_1v1_selfplay_config, LAYOUT_1V1, {TEAM_RADIANT: [0], TEAM_DIRE: [5]}),
                                                    (get_5v5_selfplay_config, LAYOUT_5V5,
                                                     {TEAM_RADIANT: [0, 2], TEAM_DIRE: [5, 9]})])
def test_native_featurizer_matches_python(cfg_fn, layout, players):
    states = _states(cfg_fn)
    blobs, pids, tids = [], [], []
    for b, team in states:
        for p in players[team]:
            blobs.append(b)
            pids.append(p)
            tids.append(team)
    env, units, handles, ncreep = native.featurize_batch(blobs, pids, tids, list(layout.counts), 4)
    for i, (b, p, t) in enumerate(zip(blobs, pids, tids)):
        f = featurize(pb.CMsgBotWorldState.FromString(b), p, t, layout=layout)
        np.testing.assert_allclose(env[i], f.env, rtol=1e-5, atol=1e-6)
        np.testing.assert_allclose(units[i], f.units, rtol=1e-5, atol=1e-5)
        np.testing.assert_array_equal(handles[i], f.handles)
        assert ncreep[i] == f.n_allied_creep


def test_native_featurizer_rejects_garbage():
    with pytest.raises(RuntimeError):
        native.featurize_batch([b'\xff\xff\xff'], [0], [2], list(LAYOUT_1V1.counts), 1)


def test_crc32c():
    assert native.crc32c(b'123456789') == 0xE3069283
    from dotaclient_amd.utils.tfevents import _TABLE
    data = os.urandom(1000)
    crc = 0xFFFFFFFF
    for x in data:
        crc = _TABLE[(crc ^ x) & 0xFF] ^ (crc >> 8)
    assert native.crc32c(data) == crc ^ 0xFFFFFFFF


def _crc_table(data: bytes) -> int:
    from dotaclient_amd.utils.tfevents import _TABLE
    crc = 0xFFFFFFFF
    for x in data:
        crc = _TABLE[(crc ^ x) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


@pytest.mark.parametrize('n', [(3 << 16) - 1, 3 << 16, (3 << 16) + 1, (3 << 16) + 7, (3 << 16) + 8, (3 << 16) + 13,
                               400_003, 3 * 131_072 + 5])
def test_crc32c_three_chain_path_known_answer(n):
    """Buffers of ≥ 192 KiB take the native three-chain CRC-32C with crc32c_combine (native/core.h): pinned against
    the table-driven reference at and around the threshold, lengths that are not multiples of 8 or of 3."""
    data = os.urandom(n)
    assert native.crc32c(data) == _crc_table(data)


def _producer(name, n, k):
    r = native.ShmRing(name, 1 << 16, False)
    for i in range(n):
        assert r.push(f'{k}:{i}:'.encode() + os.urandom(300 + i % 200), 10.0, False)


def test_shm_ring_mpmc():
    name = f'/dca_test_{uuid.uuid4().hex[:8]}'
    ring = native.ShmRing(name, 1 << 16, True)
    try:
        assert ring.pop(0.0) is None
        ctx = mp.get_context('spawn')
        ps = [ctx.Process(target=_producer, args=(name, 500, k)) for k in range(3)]
        for p in ps:
            p.start()
        got = {}
        for _ in range(1500):
            m = ring.pop(20.0)
            assert m is not None
            k, i = m.split(b':')[:2]
            got.setdefault(int(k), []).append(int(i))
        for p in ps:
            p.join(timeout=30)
            assert p.exitcode == 0
        for k in range(3):
            assert got[k] == list(range(500))    # per-producer FIFO, nothing lost across wrap-arounds
        assert ring.size() == 0
    finally:
        native.ShmRing.unlink(name)


def test_shm_ring_copies_outside_lock_exactly_once():
    """Producers copy into reserved regions and consumers copy out of claimed ones outside the ring's lock
    (native/core.h RingCore): under 3 producer and 3 consumer threads with messages of up to a quarter of the ring
    (wrap-arounds, space held by in-flight copies), every message arrives exactly once and intact; drop_oldest on a
    full ring drops committed messages only and counts them."""
    import hashlib
    import threading
    name = f'/dca_test_{uuid.uuid4().hex[:8]}'
    ring = native.ShmRing(name, 1 << 20, True)
    try:
        per, got, lock = 300, [], threading.Lock()

        def prod(k):
            rng = np.random.RandomState(k)
            for i in range(per):
                body = rng.bytes(int(rng.randint(1, 1 << 18)))
                assert ring.push(f'{k}:{i}:'.encode() + hashlib.sha1(body).hexdigest().encode() + b':' + body, 30.0,
                                 False)

        def cons():
            while True:
                m = ring.pop(5.0)
                if m is None:
                    return
                with lock:
                    got.append(m)
        ts = [threading.Thread(target=prod, args=(k,)) for k in range(3)] + \
             [threading.Thread(target=cons) for _ in range(3)]
        for t in ts:
            t.start()
        for t in ts:
            t.join(timeout=120)
        seen = set()
        for m in got:
            k, i, h, body = m.split(b':', 3)
            assert hashlib.sha1(body).hexdigest().encode() == h
            seen.add((int(k), int(i)))
        assert len(got) == 3 * per and len(seen) == 3 * per and ring.size() == 0
        # drop_oldest: a full ring makes room by discarding its oldest committed messages
        for i in range(40):
            assert ring.push(bytes([i]) * 60000, 0.0, True)
        assert ring.dropped() > 0
        first = ring.pop(0.0)
        assert first is not None and first[0] == 40 - ring.size() - 1
    finally:
        native.ShmRing.unlink(name)


def test_shm_broker_roundtrip():
    from dotaclient_amd.transport.shm import ShmBroker
    name = f'dca_b_{uuid.uuid4().hex[:8]}'
    b = ShmBroker(name, capacity=1 << 20, create=True)
    try:
        b.publish_experience(b'abc')
        assert b.xp_queue_size == 1 and b.consume_experience(1.0) == b'abc'
        b.publish_model(b'w1', 4)
        assert b.latest_model(newer_than=3) == (4, b'w1')
        assert b.latest_model(newer_than=4) is None
    finally:
        b.close(unlink=True)


def test_shm_broker_view_decodes_rollout():
    """``consume_experience_view`` (ShmRing.pop_view, native/featurizer.cpp) hands the learner's decode thread a
    uint8 array owning the message: same bytes as ``consume_experience``, and the codec decodes it in place."""
    from dotaclient_amd.transport.codec import Rollout, decode_any, encode
    from dotaclient_amd.transport.shm import ShmBroker
    rng = np.random.RandomState(0)
    T, U = 12, 20
    r = Rollout(game_id='g', team_id=2, player_id=0, env=rng.randn(T, 3).astype(np.float32),
                units=rng.randn(T, U, 10).astype(np.float32), actions=(rng.rand(T, 21 + U) > 0.9).astype(np.uint8),
                masks=(rng.rand(T, 21 + U) > 0.5).astype(np.uint8), rewards=rng.randn(T, 9), weight_version=3,
                canvas=np.zeros((8, 8, 3), np.uint8), logp=rng.randn(T).astype(np.float32),
                values=rng.randn(T).astype(np.float32), hiddens=rng.randn(2, 2, 16).astype(np.float32),
                hidden_stride=16, bootstrap_value=0.25, done=True)
    body = encode(r)
    b = ShmBroker(f'dca_v_{uuid.uuid4().hex[:8]}', capacity=1 << 20, create=True)
    try:
        assert b.consume_experience_view(0.0) is None
        b.publish_experience(body)
        b.publish_experience(body)
        v = b.consume_experience_view(1.0)
        assert isinstance(v, np.ndarray) and v.dtype == np.uint8 and v.tobytes() == body
        assert b.consume_experience(1.0) == body
        d = decode_any(v)
        del v                                          # the decoded arrays must not depend on the view staying alive
        for k in ['env', 'units', 'actions', 'masks', 'rewards', 'logp', 'values', 'hiddens']:
            np.testing.assert_array_equal(getattr(d, k), getattr(r, k))
        assert (d.weight_version, d.bootstrap_value, d.done) == (3, 0.25, True)
        # the CRC-checked pop: the trailer verified while copying out (64 KB blocks, combined CRCs)
        big = encode(Rollout(**{**r.__dict__, 'units': rng.randn(400, U, 10).astype(np.float32),
                                'env': rng.randn(400, 3).astype(np.float32),
                                'actions': np.zeros((400, 21 + U), np.uint8), 'masks': np.ones((400, 21 + U), np.uint8),
                                'rewards': rng.randn(400, 9), 'logp': rng.randn(400).astype(np.float32),
                                'values': rng.randn(400).astype(np.float32)}))
        assert len(big) > 3 * (64 << 10)
        bad = bytearray(big)
        bad[len(bad) // 2] ^= 0x10
        for msg, want in ((big, True), (bytes(bad), False), (b'not a dcx2 message', None)):
            b.publish_experience(msg)
            arr, ok = b.consume_experience_checked(1.0)
            assert ok is want and arr.tobytes() == msg
        assert b.consume_experience_checked(0.0) is None
        d2 = decode_any(np.frombuffer(big, np.uint8), crc_checked=True)
        assert d2.units.shape == (400, U, 10)
    finally:
        b.close(unlink=True)


def test_copy_jobs_parallel_memcpy():
    """native copy_jobs (the ingest stager's parallel field copy): every job lands, pieces > 1 MB split correctly."""
    rng = np.random.default_rng(0)
    srcs = [rng.integers(0, 255, n, dtype=np.uint8) for n in (1, 17, 1 << 20, (3 << 20) + 5, 4096)]
    dst = np.zeros(sum(s.nbytes for s in srcs) + 64, np.uint8)
    jobs, o = [], 0
    for s in srcs:
        jobs.append((dst.ctypes.data + o, s.ctypes.data, s.nbytes))
        o += s.nbytes
    native.copy_jobs(np.asarray(jobs, np.int64), 3)
    np.testing.assert_array_equal(dst[:o], np.concatenate(srcs))
    assert not dst[o:].any()


def test_pack_rows_copies_converts_and_zero_fills():
    """native.pack_rows (the ingest stager's field packing): per-rollout rows land at their valid-row offsets,
    f64 sources convert to f32, a missing field zero-fills, mismatched sources raise."""
    from dotaclient_amd import native
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    rng = np.random.default_rng(0)
    lens = [3, 0, 5, 2]
    pos = np.zeros(len(lens) + 1, np.int64)
    np.cumsum(lens, out=pos[1:])
    units = [rng.standard_normal((T, 7, 10)).astype(np.float32) for T in lens]
    rew = [rng.standard_normal((T, 9)) for T in lens]
    acts = [rng.integers(0, 255, (T, 61)).astype(np.uint8) for T in lens]
    du = np.full((12, 7, 10), 7.0, np.float32)
    dr = np.full((12, 9), 7.0, np.float32)
    da = np.full((12, 61), 7, np.uint8)
    dv = np.full(12, 7.0, np.float32)
    native.pack_rows([(du, units), (dr, rew), (da, acts), (dv, [None] * 4)], pos, 3)
    np.testing.assert_array_equal(du[:10], np.concatenate(units))
    np.testing.assert_array_equal(dr[:10], np.concatenate(rew).astype(np.float32))
    np.testing.assert_array_equal(da[:10], np.concatenate(acts))
    assert not dv[:10].any() and (du[10:] == 7).all() and (dv[10:] == 7).all()
    with pytest.raises(ValueError):
        native.pack_rows([(du, [u[:, :5] .copy() for u in units])], pos, 2)        # wrong row width
    with pytest.raises(ValueError):
        native.pack_rows([(da, [a.astype(np.int64) for a in acts])], pos, 2)      # another dtype
    with pytest.raises(ValueError):
        native.pack_rows([(du, units[:3])], pos, 2)                               # one source short


def test_shm_ring_abandons_a_claim_that_pins_it():
    """A consumer that dies holding a claimed message must not stop the producers for good: once the claimed region
    at the reclaim point has blocked a producer for the abandonment time (60 s by default; 0.5 s here) it is given up
    and counted as dropped, the producer's message goes in, and the late release of the old token is ignored."""
    import time
    import uuid
    from dotaclient_amd import native
    from dotaclient_amd.transport.shm import ShmBroker
    if not native.AVAILABLE:
        pytest.skip('native module not built')
    b = ShmBroker(f'dca_ab_{uuid.uuid4().hex[:8]}', capacity=1 << 20, create=True, drop_oldest=True)
    try:
        b.ring.set_claim_abandon(0.5)
        msg = b'm' * (200 << 10)
        b.publish_experience(msg, timeout=1.0)
        view, token = b.claim_experience(1.0)          # held, never released by this "dead" consumer
        assert bytes(view[:4]) == b'mmmm'
        while True:                                     # fill the ring behind the claim (no blocking)
            try:
                b.publish_experience(msg, timeout=0.0)
            except TimeoutError:
                break
        d0 = b.ring.dropped()
        t0 = time.monotonic()
        # the ring is full and pinned by the claim (drop_oldest cannot reclaim behind it): the producer waits for the
        # claim's abandonment
        b.publish_experience(b'n' * (200 << 10), timeout=5.0)
        waited = time.monotonic() - t0
        assert 0.3 < waited < 4.0, waited
        assert b.ring.dropped() > d0
        b.release_experience(token)                     # late: ignored, the region was reclaimed
        got = []
        while True:
            m = b.consume_experience(0.0)
            if m is None:
                break
            got.append(bytes(m[:1]))
        assert got and got[-1] == b'n'
        # and the ring still works end to end
        b.publish_experience(msg, timeout=1.0)
        assert b.consume_experience(1.0) == msg
    finally:
        b.close(unlink=True)


def test_ring_capacity_clamp_matches_the_broker_rule():
    """learner/e2e.py sizes the node ring with transport.shm.ring_capacity_for: whatever it returns for a given free
    /dev/shm size, ShmBroker's own headroom check accepts; too small a /dev/shm fails early with a clear message
    (the old clamp, max(64 MiB, free/2), ended in MemoryError below 128 MiB free)."""
    from dotaclient_amd.transport.shm import MIN_RING, SHM_HEADROOM, ring_capacity_for
    for free in (100 << 20, 128 << 20, 200 << 20, 1 << 30, 64 << 30):
        cap = ring_capacity_for(1 << 32, free)
        assert MIN_RING <= cap <= free // 2 and cap + SHM_HEADROOM <= free
    assert ring_capacity_for(32 << 20, 64 << 30) == 32 << 20
    assert ring_capacity_for(1 << 30, None) == 1 << 30
    with pytest.raises(MemoryError, match='shm-size'):
        ring_capacity_for(1 << 30, 64 << 20)        # the container default /dev/shm
