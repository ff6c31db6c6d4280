"""Minimal TensorBoard event-file writer (scalars, histograms, images) — no tensorboard/tensorboardX dependency.

The reference logs through tensorboardX (optimizer.py:245, 533-561; agent.py:415-428). Neither tensorboard nor
tensorboardX is installable here, so this module writes the event-file format directly:

    record := u64 length | u32 masked_crc32c(length) | Event bytes | u32 masked_crc32c(Event bytes)
    Event  := {1: wall_time double, 2: step int64, 3: file_version string, 5: Summary}
    Summary.Value := {1: tag, 2: simple_value float, 4: Image, 5: HistogramProto}

The protobuf encoding is written by hand (a handful of fields). Files are named like tensorboardX's
(``events.out.tfevents.<time>.<host>``) so TensorBoard picks them up unchanged.
"""
from __future__ import annotations

import os
import socket
import struct
import time
from typing import Optional

import numpy as np

from .png import encode_png

# ---- crc32c (Castagnoli), table-driven --------------------------------------------------------------------------
_POLY = 0x82F63B78
_TABLE = []
for _i in range(256):
    _c = _i
    for _ in range(8):
        _c = (_c >> 1) ^ _POLY if _c & 1 else _c >> 1
    _TABLE.append(_c)


def crc32c(data: bytes) -> int:
    try:  # native accelerated version when the C++ helper library is built
        from ..native import crc32c as _native
        return _native(data)
    except Exception:
        pass
    crc = 0xFFFFFFFF
    t = _TABLE
    for b in data:
        crc = t[(crc ^ b) & 0xFF] ^ (crc >> 8)
    return crc ^ 0xFFFFFFFF


def masked_crc(data: bytes) -> int:
    c = crc32c(data)
    return (((c >> 15) | (c << 17)) + 0xA282EAD8) & 0xFFFFFFFF


# ---- protobuf wire helpers ---------------------------------------------------------------------------------------
def _varint(v: int) -> bytes:
    out = bytearray()
    v &= (1 << 64) - 1
    while True:
        b = v & 0x7F
        v >>= 7
        if v:
            out.append(b | 0x80)
        else:
            out.append(b)
            return bytes(out)


def _key(field: int, wt: int) -> bytes:
    return _varint((field << 3) | wt)


def _bytes_field(field: int, payload: bytes) -> bytes:
    return _key(field, 2) + _varint(len(payload)) + payload


def _double_field(field: int, v: float) -> bytes:
    return _key(field, 1) + struct.pack('<d', v)


def _float_field(field: int, v: float) -> bytes:
    return _key(field, 5) + struct.pack('<f', v)


def _int_field(field: int, v: int) -> bytes:
    return _key(field, 0) + _varint(int(v))


def _packed_doubles(field: int, vals) -> bytes:
    return _bytes_field(field, struct.pack(f'<{len(vals)}d', *vals))


def _event(step: int, summary_value: bytes, wall_time: Optional[float] = None) -> bytes:
    summary = _bytes_field(1, summary_value)
    return _double_field(1, wall_time or time.time()) + _int_field(2, step) + _bytes_field(5, summary)


class EventWriter:
    def __init__(self, log_dir: str, filename_suffix: str = ''):
        os.makedirs(log_dir, exist_ok=True)
        self.path = os.path.join(log_dir, f'events.out.tfevents.{int(time.time())}.{socket.gethostname()}'
                                          f'{filename_suffix}')
        self._f = open(self.path, 'ab')
        self._write(_double_field(1, time.time()) + _bytes_field(3, b'brain.Event:2'))

    def _write(self, event: bytes):
        hdr = struct.pack('<Q', len(event))
        self._f.write(hdr + struct.pack('<I', masked_crc(hdr)) + event + struct.pack('<I', masked_crc(event)))

    def add_scalar(self, tag: str, value: float, step: int):
        v = _bytes_field(1, tag.encode()) + _float_field(2, float(value))
        self._write(_event(step, v))

    def add_histogram(self, tag: str, values, step: int, bins: int = 30):
        a = np.asarray(values, dtype=np.float64).reshape(-1)
        if a.size == 0:
            return
        counts, edges = np.histogram(a, bins=bins)
        h = (_double_field(1, float(a.min())) + _double_field(2, float(a.max())) + _double_field(3, float(a.size)) +
             _double_field(4, float(a.sum())) + _double_field(5, float((a * a).sum())) +
             _packed_doubles(6, [float(e) for e in edges[1:]]) + _packed_doubles(7, [float(c) for c in counts]))
        v = _bytes_field(1, tag.encode()) + _bytes_field(5, h)
        self._write(_event(step, v))

    def add_image(self, tag: str, img_hwc: np.ndarray, step: int):
        img = np.asarray(img_hwc, dtype=np.uint8)
        H, W, Cc = img.shape
        im = _int_field(1, H) + _int_field(2, W) + _int_field(3, Cc) + _bytes_field(4, encode_png(img))
        v = _bytes_field(1, tag.encode()) + _bytes_field(4, im)
        self._write(_event(step, v))

    def flush(self):
        self._f.flush()

    def close(self):
        self._f.close()


def read_events(path: str):
    """Yield raw Event payloads (verifying CRCs) — used by tests."""
    with open(path, 'rb') as f:
        data = f.read()
    off = 0
    while off < len(data):
        (n,) = struct.unpack_from('<Q', data, off)
        (hc,) = struct.unpack_from('<I', data, off + 8)
        assert hc == masked_crc(data[off:off + 8]), 'header crc'
        ev = data[off + 12: off + 12 + n]
        (dc,) = struct.unpack_from('<I', data, off + 12 + n)
        assert dc == masked_crc(ev), 'data crc'
        yield ev
        off += 12 + n + 4
