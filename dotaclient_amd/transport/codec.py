"""Experience record and its wire codecs.

The reference ships each rollout as ``pickle.dumps(dict)`` on the ``experience`` queue (agent.py:387-409) with keys
``game_id, team_id, player_id, states{7}, actions{4}, masks{4}, rewards (T,9) f64, weight_version, canvas``
(SURVEY §2.8.4). :class:`Rollout` holds the same content in packed form (one ``(T,U,10)`` unit tensor, flat
``(T, 21+U)`` action/mask vectors) plus the north-star extensions the PPO/LSTM learner needs:

* ``logp`` (T,) — joint log-prob of the sampled action under the behaviour policy (PPO ratio),
* ``values`` (T,) — V(s_t) of the behaviour policy (GAE),
* ``hiddens`` (K, 2, H) — LSTM (h, c) *before* steps 0, stride, 2·stride, … of the rollout (``hidden_stride``), so
  the learner can start every ``seq_len`` chunk from the state the actor actually had (R2D2-style stored state,
  SURVEY §5);
* ``bootstrap_value`` / ``done`` — how the rollout ended (truncated by ``rollout_size`` or terminal).

Codecs:

* :func:`encode` / :func:`decode` — a compact binary format (``DCX2`` magic, JSON header, raw little-endian arrays,
  CRC-32C trailer over everything before it — SSE4.2 in the native module, ≈5× zlib's CRC-32 of the older ``DCX1``
  form, which the decoder still accepts); zero-copy ``np.frombuffer`` on decode, and a corrupted or truncated
  message raises :class:`CorruptMessage` instead of feeding garbage to the learner. ~4× smaller/faster than
  pickling torch tensors.
* :meth:`Rollout.to_reference_dict` / :meth:`Rollout.from_reference_dict` — exact reference message layout, so a
  reference agent's pickled message can be ingested and ours can be read by the reference optimizer.
  Reference pickles are decoded only when explicitly allowed (``decode_any(allow_pickle=True)``, the learner's
  ``--allow-pickle-experience``), and then by a restricted unpickler that can build nothing but dicts, lists,
  strings, numbers and numpy arrays — an unauthenticated broker port must not be a code-execution endpoint.
  Any message that fails to decode (either format) raises :class:`CorruptMessage`.
"""
from __future__ import annotations

import io
import json
import pickle
import struct
import zlib
from dataclasses import dataclass, field
from typing import Dict, Optional, Tuple

import numpy as np

from ..constants import LAYOUT_1V1, UNIT_KEYS, UnitLayout

MAGIC1 = b'DCX1'           # zlib CRC-32 trailer (decode only)
MAGIC2 = b'DCX2'           # CRC-32C trailer
MAGICS = (MAGIC1, MAGIC2)


def _crc32c_prefix(buf, n: int) -> int:
    """CRC-32C of ``buf[:n]``: the native SSE4.2 loop (GIL released), else the table-driven pure-Python one."""
    try:
        from ..native import _native
        return _native.crc32c_buf(buf, n)
    except (ImportError, AttributeError):
        from ..utils.tfevents import crc32c
        return crc32c(bytes(memoryview(buf)[:n]))


def _native_crc() -> bool:
    try:
        from ..native import _native
        return hasattr(_native, 'crc32c_buf')
    except ImportError:
        return False


MAGIC = MAGIC2 if _native_crc() else MAGIC1     # what :func:`encode` writes


class CorruptMessage(ValueError):
    """A DCX1 / DCX2 message failed its CRC / framing checks."""


@dataclass
class Rollout:
    game_id: str
    team_id: int
    player_id: int
    env: np.ndarray                      # (T, 3) f32
    units: Optional[np.ndarray]          # (T, U, 10) f32 (None in a raw rollout: see units_raw)
    actions: np.ndarray                  # (T, 21+U) u8 one-hot per sampled head
    masks: np.ndarray                    # (T, 21+U) u8 selected-heads mask
    rewards: np.ndarray                  # (T, 9) f64 in REWARD_KEYS order
    weight_version: int
    canvas: Optional[np.ndarray] = None  # (256, 256, 3) u8
    logp: Optional[np.ndarray] = None
    values: Optional[np.ndarray] = None
    hiddens: Optional[np.ndarray] = None
    hidden_stride: int = 0
    bootstrap_value: float = 0.0
    done: bool = True
    layout: Tuple[int, ...] = field(default_factory=lambda: LAYOUT_1V1.counts)
    # GPU featurization (features/raw.py, ops/csrc/featurize.hip): a VecEnv(raw=True) actor ships the compact raw unit
    # records (T, U, 8) int32 and the observing hero (T, 4) f32 instead of units; the learner featurizes them on the
    # device at ingest, host consumers through :meth:`ensure_units`
    units_raw: Optional[np.ndarray] = None
    hero: Optional[np.ndarray] = None
    # zero-copy consumption (ShmBroker.claim_experience): the arrays view the message inside the shared ring, and this
    # callable gives its region back; see :meth:`detach_shared`
    release: Optional[object] = field(default=None, repr=False, compare=False)

    @property
    def length(self) -> int:
        return int(self.rewards.shape[0])

    def ensure_units(self) -> 'Rollout':
        """Host features of a raw rollout (the numpy oracle of the device kernel; exact): fills ``units``."""
        if self.units is None and self.units_raw is not None:
            from ..features.raw import featurize_raw_np
            self.units = featurize_raw_np(self.units_raw, self.hero)[0]
        return self

    def detach_shared(self, keep_canvas: bool = False, release: bool = True):
        """Once a ring-resident rollout has been staged (learner/ingest.py): keep private copies of what the learner
        still reads afterwards (rewards for the per-key logs, optionally the canvas), drop the views of the bulk
        arrays — any later read fails loudly instead of reading a recycled ring region — and release the region
        (``release=False``: return the release callable instead, for a caller that releases several at once)."""
        if self.release is None:
            return None
        self.rewards = np.array(self.rewards)
        self.canvas = np.array(self.canvas) if (keep_canvas and self.canvas is not None) else None
        self.env = self.units = self.actions = self.masks = self.logp = self.values = self.hiddens = None
        self.units_raw = self.hero = None
        rel, self.release = self.release, None
        if not release:
            return rel
        rel()
        return None

    def unit_layout(self) -> UnitLayout:
        return UnitLayout(*self.layout)

    # -------------------------------------------------------------------------------------------------
    def to_reference_dict(self) -> Dict:
        """Reference message layout (agent.py:397-407), torch tensors as the reference's pickles carry."""
        import torch
        lay = self.unit_layout()
        self.ensure_units()
        states = {'env': torch.from_numpy(np.ascontiguousarray(self.env))}
        for k, sl in lay.slices().items():
            states[k] = torch.from_numpy(np.ascontiguousarray(self.units[:, sl]))
        heads = {}
        acc = 0
        for k, n in lay.action_counts().items():
            heads[k] = (acc, n)
            acc += n
        actions = {k: torch.from_numpy(np.ascontiguousarray(self.actions[:, o:o + n])) for k, (o, n) in heads.items()}
        masks = {k: torch.from_numpy(np.ascontiguousarray(self.masks[:, o:o + n])) for k, (o, n) in heads.items()}
        return {'game_id': self.game_id, 'team_id': self.team_id, 'player_id': self.player_id, 'states': states,
                'actions': actions, 'masks': masks, 'rewards': self.rewards, 'weight_version': self.weight_version,
                'canvas': self.canvas}

    @classmethod
    def from_reference_dict(cls, d: Dict) -> 'Rollout':
        def npy(x):
            return x.numpy() if hasattr(x, 'numpy') else np.asarray(x)
        states = d['states']
        counts = tuple(int(npy(states[k]).shape[1]) for k in UNIT_KEYS)
        units = np.concatenate([npy(states[k]) for k in UNIT_KEYS], axis=1).astype(np.float32)
        order = ['enum', 'x', 'y', 'target_unit']
        actions = np.concatenate([npy(d['actions'][k]) for k in order], axis=1).astype(np.uint8)
        masks = np.concatenate([npy(d['masks'][k]) for k in order], axis=1).astype(np.uint8)
        return cls(game_id=str(d['game_id']), team_id=int(d['team_id']), player_id=int(d['player_id']),
                   env=npy(states['env']).astype(np.float32), units=units, actions=actions, masks=masks,
                   rewards=np.asarray(d['rewards'], dtype=np.float64), weight_version=int(d['weight_version']),
                   canvas=None if d.get('canvas') is None else np.asarray(d['canvas'], dtype=np.uint8),
                   layout=counts)


_ARRAYS = ['env', 'units', 'actions', 'masks', 'rewards', 'canvas', 'logp', 'values', 'hiddens', 'units_raw', 'hero']


def encode(r: Rollout) -> bytes:
    header = {'game_id': r.game_id, 'team_id': r.team_id, 'player_id': r.player_id,
              'weight_version': r.weight_version, 'bootstrap_value': float(r.bootstrap_value), 'done': bool(r.done),
              'hidden_stride': int(r.hidden_stride),
              'layout': list(r.layout), 'arrays': []}
    blobs = []
    off = 0
    for name in _ARRAYS:
        a = getattr(r, name)
        if a is None:
            continue
        a = np.ascontiguousarray(a)
        b = a.tobytes()
        header['arrays'].append([name, a.dtype.str, list(a.shape), off, len(b)])
        blobs.append(b)
        off += len(b)
    h = json.dumps(header, separators=(',', ':')).encode()
    body = b''.join([MAGIC, struct.pack('<I', len(h)), h] + blobs)
    crc = _crc32c_prefix(body, len(body)) if MAGIC == MAGIC2 else zlib.crc32(body)
    return body + struct.pack('<I', crc)


def decode(buf: bytes, crc_checked: bool = False) -> Rollout:
    """``crc_checked``: the trailer was verified while the message was copied out of the ring
    (``ShmBroker.consume_experience_checked``) — skip the second pass over it."""
    magic = bytes(buf[:4])
    if magic not in MAGICS:
        raise ValueError('not a DCX1 / DCX2 experience message')
    if len(buf) < 12:
        raise CorruptMessage('truncated experience message')
    if not (crc_checked and magic == MAGIC2):
        (crc,) = struct.unpack_from('<I', buf, len(buf) - 4)
        n = len(buf) - 4
        got = _crc32c_prefix(buf, n) if magic == MAGIC2 else zlib.crc32(memoryview(buf)[:n])
        if got != crc:
            raise CorruptMessage('experience message CRC mismatch (corrupted or truncated)')
    (hl,) = struct.unpack_from('<I', buf, 4)
    header = json.loads(bytes(buf[8:8 + hl]))
    base = 8 + hl
    arrays = {}
    mv = memoryview(buf)
    for name, dt, shape, off, n in header['arrays']:
        arrays[name] = np.frombuffer(mv[base + off: base + off + n], dtype=np.dtype(dt)).reshape(shape)
    if arrays.get('units') is None:
        # a raw rollout (GPU featurization): the records and the hero rows must both be there, in their layout
        ur, hr = arrays.get('units_raw'), arrays.get('hero')
        if ur is None or hr is None:
            raise CorruptMessage('experience message without units (or units_raw + hero)')
        if (ur.dtype != np.int32 or ur.ndim != 3 or ur.shape[2] != 8 or hr.dtype != np.float32
                or hr.shape != (ur.shape[0], 4)):
            raise CorruptMessage(f'bad raw unit records {ur.dtype}{ur.shape} / hero {hr.dtype}{hr.shape}')
    return Rollout(game_id=header['game_id'], team_id=header['team_id'], player_id=header['player_id'],
                   weight_version=header['weight_version'], bootstrap_value=header['bootstrap_value'],
                   hidden_stride=header.get('hidden_stride', 0),
                   done=header['done'], layout=tuple(header['layout']), **{k: arrays.get(k) for k in _ARRAYS})


def _storage_from_bytes(b):
    # torch.storage._load_from_bytes would torch.load(weights_only=False) attacker-controlled bytes
    import torch
    return torch.load(io.BytesIO(b), weights_only=True)


def _storage_elements(storage) -> int:
    import torch
    if isinstance(storage, torch.storage.TypedStorage):
        return int(storage._untyped_storage.nbytes()) // torch.empty((), dtype=storage.dtype).element_size()
    return int(storage.nbytes())


def _rebuild_tensor_checked(storage, storage_offset, size, stride, *args, **kwargs):
    """``torch._utils._rebuild_tensor_v2`` restricted to views INSIDE the loaded storage. The stock rebuild calls
    ``set_``, which grows the storage to whatever size/stride the message claims — a crafted message could force an
    allocation of any size. Out-of-range views are rejected as corrupt instead."""
    import torch._utils as tu
    size, stride = tuple(int(x) for x in size), tuple(int(x) for x in stride)
    off = int(storage_offset)
    if len(size) != len(stride) or off < 0 or any(x < 0 for x in size) or any(x < 0 for x in stride):
        raise CorruptMessage(f'invalid tensor view: size={size} stride={stride} offset={off}')
    if all(x > 0 for x in size):
        last = off + sum((n - 1) * st for n, st in zip(size, stride))
        if last >= _storage_elements(storage):
            raise CorruptMessage(f'tensor view size={size} stride={stride} offset={off} exceeds its storage')
    return tu._rebuild_tensor_v2(storage, off, size, stride, *args, **kwargs)


class _ArrayUnpickler(pickle.Unpickler):
    """Unpickler for the reference's experience dicts (numpy arrays and torch tensors in plain containers): only
    array / tensor reconstruction can be resolved — tensor storages through a weights-only ``torch.load``, tensor
    views bounds-checked against their storage — so a crafted message cannot run code or force huge allocations."""
    _ALLOWED = {('numpy.core.multiarray', '_reconstruct'), ('numpy._core.multiarray', '_reconstruct'),
                ('numpy.core.multiarray', 'scalar'), ('numpy._core.multiarray', 'scalar'),
                ('numpy', 'ndarray'), ('numpy', 'dtype'), ('collections', 'OrderedDict')}

    def find_class(self, module, name):
        if (module, name) == ('torch.storage', '_load_from_bytes'):
            return _storage_from_bytes
        if (module, name) == ('torch._utils', '_rebuild_tensor_v2'):
            return _rebuild_tensor_checked
        if (module, name) in self._ALLOWED:
            return super().find_class(module, name)
        raise pickle.UnpicklingError(f'global {module}.{name} is not allowed in an experience message')


def decode_any(buf: bytes, allow_pickle: bool = False, crc_checked: bool = False) -> Rollout:
    """DCX1 binary, or (``allow_pickle``) a reference agent's pickled dict through :class:`_ArrayUnpickler`. Every
    decode failure surfaces as :class:`CorruptMessage` (the learner drops the message and carries on).
    ``crc_checked``: a DCX2 trailer already verified by the ring (:func:`decode`)."""
    try:
        if bytes(buf[:4]) in MAGICS:
            return decode(buf, crc_checked=crc_checked)
        if not allow_pickle:
            raise CorruptMessage('not a DCX1 / DCX2 message (reference pickles need allow_pickle / '
                                 '--allow-pickle-experience)')
        return Rollout.from_reference_dict(_ArrayUnpickler(io.BytesIO(buf)).load())
    except CorruptMessage:
        raise
    except (pickle.UnpicklingError, ValueError, KeyError, TypeError, IndexError, AttributeError, EOFError,
            struct.error, UnicodeDecodeError, RuntimeError, MemoryError, OverflowError) as e:
        raise CorruptMessage(f'undecodable experience message: {e!r}') from e


# ---- model messages -------------------------------------------------------------------------------------------
def encode_state_dict(state_dict) -> bytes:
    """``torch.save(state_dict)`` bytes — the reference's model message / checkpoint format (optimizer.py:699-703)."""
    import torch
    buf = io.BytesIO()
    torch.save(state_dict, buf)
    return buf.getvalue()


def decode_state_dict(b: bytes):
    import torch
    return torch.load(io.BytesIO(b), map_location='cpu', weights_only=True)
