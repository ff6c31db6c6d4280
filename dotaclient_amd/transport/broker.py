"""Experience queue + latest-model exchange (the RabbitMQ replacement).

The reference couples actors and learner through RabbitMQ: a non-durable ``experience`` queue
(competing consumers: every optimizer rank pops disjoint rollouts, optimizer.py:144-158) and a ``model`` exchange of
type ``x-recent-history`` with length 1 (late joiners immediately get the newest weights, optimizer.py:107-111,
agent.py:212-223), model messages carry an integer ``version`` header.

This module provides the same two primitives with one interface and three transports:

* :class:`InProcBroker` — threads in one process (tests, single-node runs, the batched GPU actor feeding a learner
  in the same process);
* :class:`TcpBrokerServer` / :class:`TcpBroker` — a small framed TCP protocol for multi-process / multi-host jobs
  (one server thread per connection, blocking pops with timeouts, reconnect-with-retry clients as the reference's
  ``MessageQueue.connect`` does, optimizer.py:85-97);
* ``dotaclient_amd.native.ShmRing`` — a C++ shared-memory ring for node-local actors (see native/shmring.cpp),
  wrapped by :class:`ShmExperienceQueue`.

Unlike RabbitMQ's unbounded queue, the experience queue is bounded (``maxsize``) with back-pressure or drop-oldest,
so a slow learner cannot exhaust memory.
"""
from __future__ import annotations

import logging
import queue
import socket
import socketserver
import struct
import threading
import time
from typing import Callable, List, Optional, Tuple

logger = logging.getLogger(__name__)

EXPERIENCE_QUEUE_NAME = 'experience'
MODEL_EXCHANGE_NAME = 'model'


class InProcBroker:
    def __init__(self, maxsize: int = 0, drop_oldest: bool = False):
        self._q: 'queue.Queue[bytes]' = queue.Queue(maxsize=maxsize)
        self._drop_oldest = drop_oldest
        self._model: Optional[Tuple[int, bytes]] = None
        self._cv = threading.Condition()
        self._subs: List[Callable[[int, bytes], None]] = []
        self.n_published = 0
        self.n_dropped = 0

    # experience ----------------------------------------------------------------------------------------
    def publish_experience(self, body: bytes, timeout: Optional[float] = None):
        if self._drop_oldest:
            while True:
                try:
                    self._q.put_nowait(body)
                    break
                except queue.Full:
                    try:
                        self._q.get_nowait()
                        self.n_dropped += 1
                    except queue.Empty:
                        pass
        else:
            self._q.put(body, timeout=timeout)
        self.n_published += 1

    def consume_experience(self, timeout: Optional[float] = None) -> Optional[bytes]:
        try:
            return self._q.get(timeout=timeout)
        except queue.Empty:
            return None

    @property
    def xp_queue_size(self) -> int:
        return self._q.qsize()

    # model (x-recent-history, length 1) ----------------------------------------------------------------
    def publish_model(self, body: bytes, version: int):
        with self._cv:
            self._model = (int(version), body)
            self._cv.notify_all()
            subs = list(self._subs)
        for cb in subs:
            cb(int(version), body)

    def latest_model(self, newer_than: int = -(1 << 62), timeout: Optional[float] = 0.0) -> Optional[Tuple[int, bytes]]:
        with self._cv:
            if timeout:
                self._cv.wait_for(lambda: self._model is not None and self._model[0] > newer_than, timeout=timeout)
            if self._model is not None and self._model[0] > newer_than:
                return self._model
            return None

    def subscribe_model(self, callback: Callable[[int, bytes], None]):
        """Callback on every publish; a late subscriber immediately gets the latest model (recent-history)."""
        with self._cv:
            self._subs.append(callback)
            latest = self._model
        if latest is not None:
            callback(*latest)

    def close(self):
        pass


# ------------------------------------------------------------------------------------------------------------
# TCP transport. Frame: op u8 | len u32 | payload. Replies: status u8 | len u32 | payload.
OP_PUT_XP, OP_GET_XP, OP_PUT_MODEL, OP_GET_MODEL, OP_QSIZE, OP_PING = 1, 2, 3, 4, 5, 6
_HDR = struct.Struct('<BI')


def _recv_exact(sock: socket.socket, n: int) -> bytes:
    buf = bytearray(n)
    mv = memoryview(buf)
    got = 0
    while got < n:
        k = sock.recv_into(mv[got:], n - got)
        if k == 0:
            raise ConnectionError('peer closed')
        got += k
    return bytes(buf)


def _send_frame(sock, op: int, payload: bytes = b''):
    sock.sendall(_HDR.pack(op, len(payload)) + payload)


def _recv_frame(sock) -> Tuple[int, bytes]:
    op, n = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return op, _recv_exact(sock, n) if n else b''


class _Handler(socketserver.BaseRequestHandler):
    def handle(self):
        broker: InProcBroker = self.server.broker
        sock = self.request
        sock.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
        try:
            while True:
                op, payload = _recv_frame(sock)
                if op == OP_PUT_XP:
                    broker.publish_experience(payload)
                    _send_frame(sock, 0)
                elif op == OP_GET_XP:
                    (timeout,) = struct.unpack('<d', payload)
                    body = broker.consume_experience(timeout=timeout if timeout >= 0 else None)
                    _send_frame(sock, 0 if body is not None else 1, body or b'')
                elif op == OP_PUT_MODEL:
                    (version,) = struct.unpack_from('<q', payload)
                    broker.publish_model(payload[8:], version)
                    _send_frame(sock, 0)
                elif op == OP_GET_MODEL:
                    have, timeout = struct.unpack('<qd', payload)
                    m = broker.latest_model(newer_than=have, timeout=timeout)
                    if m is None:
                        _send_frame(sock, 1)
                    else:
                        _send_frame(sock, 0, struct.pack('<q', m[0]) + m[1])
                elif op == OP_QSIZE:
                    _send_frame(sock, 0, struct.pack('<q', broker.xp_queue_size))
                elif op == OP_PING:
                    _send_frame(sock, 0)
                else:
                    _send_frame(sock, 2)
        except (ConnectionError, OSError):
            return


class _Server(socketserver.ThreadingMixIn, socketserver.TCPServer):
    daemon_threads = True
    allow_reuse_address = True


class TcpBrokerServer:
    """Serve an :class:`InProcBroker` over TCP (the RabbitMQ-pod equivalent, ks-app/components/rmq.jsonnet)."""

    def __init__(self, host: str = '127.0.0.1', port: int = 0, maxsize: int = 0, drop_oldest: bool = False):
        self.broker = InProcBroker(maxsize=maxsize, drop_oldest=drop_oldest)
        self._srv = _Server((host, port), _Handler)
        self._srv.broker = self.broker
        self.host, self.port = self._srv.server_address
        self._thread = threading.Thread(target=self._srv.serve_forever, daemon=True)

    def start(self):
        self._thread.start()
        return self

    def stop(self):
        self._srv.shutdown()
        self._srv.server_close()


class TcpBroker:
    """Client with the :class:`InProcBroker` interface. Reconnects up to ``max_retries`` times (optimizer.py:88-97)."""

    def __init__(self, host: str = '127.0.0.1', port: int = 5672, max_retries: int = 10, retry_delay: float = 0.5):
        self.host, self.port = host, port
        self.max_retries, self.retry_delay = max_retries, retry_delay
        self._sock: Optional[socket.socket] = None
        self._lock = threading.Lock()
        self._subs: List[Callable] = []
        self._sub_thread = None
        self._stop = threading.Event()
        self.connect()

    def connect(self):
        last = None
        for i in range(self.max_retries):
            try:
                s = socket.create_connection((self.host, self.port), timeout=30)
                s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                s.settimeout(None)
                self._sock = s
                return
            except OSError as e:
                last = e
                logger.error('connection to broker failed, retrying (%d/%d)', i + 1, self.max_retries)
                time.sleep(self.retry_delay)
        raise ConnectionError(f'cannot reach broker {self.host}:{self.port}: {last}')

    def consumer(self) -> 'TcpBroker':
        """A second client on its own connection for a thread that blocks in ``consume_experience`` (the learner's
        decode-ahead thread), so its long polls never hold this client's lock."""
        return TcpBroker(self.host, self.port, self.max_retries, self.retry_delay)

    def _call(self, op, payload=b''):
        with self._lock:
            for attempt in range(2):
                try:
                    _send_frame(self._sock, op, payload)
                    return _recv_frame(self._sock)
                except (ConnectionError, OSError):
                    if attempt:
                        raise
                    logger.error('reconnecting to broker')
                    self.connect()

    def publish_experience(self, body: bytes, timeout=None):
        self._call(OP_PUT_XP, body)

    def consume_experience(self, timeout: Optional[float] = None) -> Optional[bytes]:
        st, body = self._call(OP_GET_XP, struct.pack('<d', -1.0 if timeout is None else float(timeout)))
        return body if st == 0 else None

    @property
    def xp_queue_size(self) -> Optional[int]:
        try:
            st, body = self._call(OP_QSIZE)
            return struct.unpack('<q', body)[0]
        except Exception:
            return None

    def publish_model(self, body: bytes, version: int):
        self._call(OP_PUT_MODEL, struct.pack('<q', int(version)) + body)

    def latest_model(self, newer_than: int = -(1 << 62), timeout: Optional[float] = 0.0):
        st, body = self._call(OP_GET_MODEL, struct.pack('<qd', int(newer_than), float(timeout or 0.0)))
        if st != 0:
            return None
        return struct.unpack_from('<q', body)[0], body[8:]

    def subscribe_model(self, callback: Callable[[int, bytes], None], poll: float = 1.0):
        """Background long-poll subscriber (own connection) invoking ``callback(version, body)``."""
        self._subs.append(callback)
        if self._sub_thread is None:
            def run():
                cli = TcpBroker(self.host, self.port, self.max_retries, self.retry_delay)
                have = -(1 << 62)
                while not self._stop.is_set():
                    try:
                        m = cli.latest_model(newer_than=have, timeout=poll)
                    except Exception:
                        time.sleep(poll)
                        continue
                    if m is not None:
                        have = m[0]
                        for cb in list(self._subs):
                            cb(*m)
                cli.close()
            self._sub_thread = threading.Thread(target=run, daemon=True)
            self._sub_thread.start()

    def close(self):
        self._stop.set()
        th, self._sub_thread = self._sub_thread, None
        if th is not None and th is not threading.current_thread():
            th.join(timeout=30.0)           # its long poll ends within ``poll`` seconds
        if self._sock is not None:
            try:
                self._sock.close()
            except OSError:
                pass


def make_broker(url: Optional[str]):
    """'inproc' / None → InProcBroker; 'tcp://host:port' → TcpBroker; 'shm://name' → shared-memory queue."""
    if url is None or url == 'inproc':
        return InProcBroker()
    if url.startswith('tcp://'):
        host, port = url[6:].rsplit(':', 1)
        return TcpBroker(host, int(port))
    if url.startswith('shm://'):
        from .shm import ShmBroker
        return ShmBroker(url[6:])
    raise ValueError(url)
