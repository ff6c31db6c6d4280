"""Tiny PNG encoder/decoder (8-bit RGB/RGBA/gray) using zlib — replaces the reference's ``pypng`` dependency
(agent.py:740-741 ``Drawing.save``; canvas images in tensorboard, optimizer.py:550)."""
from __future__ import annotations

import struct
import zlib

import numpy as np


def _chunk(tag: bytes, data: bytes) -> bytes:
    return struct.pack('>I', len(data)) + tag + data + struct.pack('>I', zlib.crc32(tag + data) & 0xFFFFFFFF)


def encode_png(img: np.ndarray) -> bytes:
    a = np.asarray(img, dtype=np.uint8)
    if a.ndim == 2:
        a = a[:, :, None]
    H, W, C = a.shape
    ctype = {1: 0, 3: 2, 4: 6}[C]
    raw = b''.join(b'\x00' + a[y].tobytes() for y in range(H))
    return (b'\x89PNG\r\n\x1a\n' + _chunk(b'IHDR', struct.pack('>IIBBBBB', W, H, 8, ctype, 0, 0, 0)) +
            _chunk(b'IDAT', zlib.compress(raw, 6)) + _chunk(b'IEND', b''))


def decode_png(b: bytes) -> np.ndarray:
    """Decoder for the files :func:`encode_png` writes (filter type 0 only)."""
    assert b[:8] == b'\x89PNG\r\n\x1a\n'
    off, idat, W = 8, b'', 0
    while off < len(b):
        (n,) = struct.unpack_from('>I', b, off)
        tag = b[off + 4: off + 8]
        data = b[off + 8: off + 8 + n]
        if tag == b'IHDR':
            W, H, _, ctype = struct.unpack_from('>IIBB', data)
            C = {0: 1, 2: 3, 6: 4}[ctype]
        elif tag == b'IDAT':
            idat += data
        off += 12 + n
    raw = zlib.decompress(idat)
    rows = np.frombuffer(raw, dtype=np.uint8).reshape(H, 1 + W * C)
    assert (rows[:, 0] == 0).all()
    return rows[:, 1:].reshape(H, W, C)


def save_png(path: str, img: np.ndarray):
    with open(path, 'wb') as f:
        f.write(encode_png(img))
