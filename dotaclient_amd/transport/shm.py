"""Node-local broker on shared memory: the experience queue is a native MPMC ring in POSIX shm
(``native.ShmRing``: robust process-shared mutex + condvars, bounded, blocking with timeouts); the latest model is
an atomically-replaced file in /dev/shm (x-recent-history length 1 semantics). Actors and learner ranks on one node
exchange experience without a broker process or TCP."""
from __future__ import annotations

import os
import struct
import threading
import time
from typing import Callable, Optional

from .. import native


SHM_HEADROOM = 64 << 20      # /dev/shm bytes a ring leaves free (the model file, ≈8-90 MB, lives there too)
MIN_RING = 16 << 20          # smallest useful experience ring (whole-game rollouts are ≈1.35 MB)


def ring_capacity_for(want: int, free: Optional[int]) -> int:
    """The ring size to create on a /dev/shm with ``free`` bytes: ``want``, clamped to half the free space and to
    what leaves :data:`SHM_HEADROOM` (the same rule :class:`ShmBroker` enforces); MemoryError when even
    :data:`MIN_RING` does not fit."""
    if free is None:
        return int(want)
    cap = min(int(want), free // 2, free - SHM_HEADROOM)
    if cap < MIN_RING:
        raise MemoryError(f'/dev/shm has {free >> 20} MiB free: not even a {MIN_RING >> 20} MiB experience ring fits '
                          f'beside {SHM_HEADROOM >> 20} MiB of headroom (enlarge /dev/shm, e.g. docker --shm-size)')
    return cap


def shm_free_bytes() -> Optional[int]:
    """Free bytes of /dev/shm (None where it cannot be read)."""
    try:
        import shutil
        return int(shutil.disk_usage('/dev/shm').free)
    except OSError:
        return None


class ShmBroker:
    def __init__(self, name: str, capacity: int = 1 << 28, create: Optional[bool] = None, drop_oldest: bool = False):
        if not native.AVAILABLE:
            raise RuntimeError('native module not built (python -m dotaclient_amd.native.build)')
        self.name = name.strip('/')
        path = f'/dev/shm/{self.name}_xp'
        if create is None:
            create = not os.path.exists(path)
        if create:
            # tmpfs backs the ring lazily: a ring larger than /dev/shm's free space would be created fine and then
            # SIGBUS its producers mid-write once the pages run out — refuse it here instead
            free = shm_free_bytes()
            if free is not None and capacity + SHM_HEADROOM > free:
                raise MemoryError(f'/dev/shm has {free >> 20} MiB free, the experience ring needs {capacity >> 20} MiB '
                                  f'(+ the model file): pass a smaller capacity')
        self.ring = native.ShmRing(f'/{self.name}_xp', capacity, create)
        self._capacity = os.path.getsize(path)       # (+ the ring header: close enough for claim budgeting)
        self.model_path = f'/dev/shm/{self.name}_model'
        self.drop_oldest = drop_oldest
        self._subs = []
        self._stop = threading.Event()
        self._thread = None

    def publish_experience(self, body: bytes, timeout: Optional[float] = None):
        ok = self.ring.push(body, -1.0 if timeout is None else timeout, self.drop_oldest)
        if not ok:
            raise TimeoutError('experience ring full')

    def consume_experience(self, timeout: Optional[float] = None) -> Optional[bytes]:
        return self.ring.pop(-1.0 if timeout is None else float(timeout))

    def consume_experience_view(self, timeout: Optional[float] = None):
        """:meth:`consume_experience` as a uint8 numpy array owning the message (no bytes copy under the GIL);
        the learner's decode thread takes this form when the broker offers it."""
        return self.ring.pop_view(-1.0 if timeout is None else float(timeout))

    def consume_experience_checked(self, timeout: Optional[float] = None):
        """:meth:`consume_experience_view` with the DCX2 CRC-32C trailer verified in the same pass as the copy out
        of the ring (``ShmRing.pop_checked``): ``(array, ok)`` with ok True / False for DCX2 messages and None for
        other formats (the decoder then checks them), or None when nothing arrived."""
        return self.ring.pop_checked(-1.0 if timeout is None else float(timeout))

    def claim_experience(self, timeout: Optional[float] = None):
        """Zero-copy consumption: ``(array, token)`` with the array viewing the message inside the ring (its region
        stays reserved) until :meth:`release_experience` ``(token)`` — exactly once; None when nothing arrived."""
        return self.ring.claim(-1.0 if timeout is None else float(timeout))

    def claim_valid(self, token: int) -> bool:
        """Whether a zero-copy claim still owns its ring region: False once the ring abandoned it (a claim held past
        the abandonment deadline while producers needed the space) — its bytes may have been overwritten since."""
        return bool(self.ring.claim_valid(int(token)))

    def release_experience(self, token: int):
        self.ring.release(int(token))

    def release_experience_many(self, tokens):
        """Several claims given back under one ring lock (the stager releases an iteration's rollouts at once)."""
        self.ring.release_many([int(t) for t in tokens])

    @property
    def capacity(self) -> int:
        return int(self._capacity)

    @property
    def xp_queue_size(self) -> int:
        return int(self.ring.size())

    def publish_model(self, body: bytes, version: int):
        tmp = f'{self.model_path}.{os.getpid()}.tmp'
        with open(tmp, 'wb') as f:
            f.write(struct.pack('<q', int(version)))
            f.write(body)
        os.replace(tmp, self.model_path)

    def latest_model(self, newer_than: int = -(1 << 62), timeout: Optional[float] = 0.0):
        """(version, body) of the published model if its version is newer than ``newer_than``, polling up to
        ``timeout`` s. Only the 8-byte version header is read until a newer model is there: the actor's subscriber
        polls every few ms, and reading the whole ≈8 MB file per poll cost the actor process ≈1 GB/s of copies."""
        t0 = time.time()
        while True:
            try:
                with open(self.model_path, 'rb') as f:
                    head = f.read(8)
                    v = struct.unpack('<q', head)[0]
                    if v > newer_than:
                        return v, f.read()
            except (FileNotFoundError, struct.error):
                pass
            if not timeout or time.time() - t0 > timeout:
                return None
            time.sleep(0.01)

    def subscribe_model(self, callback: Callable[[int, bytes], None], poll: float = 0.2):
        self._subs.append(callback)
        if self._thread is None:
            def run():
                have = -(1 << 62)
                while not self._stop.is_set():
                    m = self.latest_model(newer_than=have, timeout=poll)
                    if m is not None:
                        have = m[0]
                        for cb in list(self._subs):
                            cb(*m)
            self._thread = threading.Thread(target=run, daemon=True)
            self._thread.start()

    def close(self, unlink: bool = False):
        """Stop and JOIN the model subscriber thread before returning: a daemon thread still running the callback
        (weight decode inside torch C++ code) when the interpreter finalises is torn down by a forced unwind, which
        aborts the process with ``terminate called without an active exception``."""
        self._stop.set()
        th, self._thread = self._thread, None
        if th is not None and th is not threading.current_thread():
            th.join(timeout=30.0)
        if unlink:
            native.ShmRing.unlink(f'/{self.name}_xp')
            try:
                os.remove(self.model_path)
            except FileNotFoundError:
                pass
