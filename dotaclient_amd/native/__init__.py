"""Native host-side runtime (C++): protobuf featurizer, shared-memory ring, crc32c. Built by ``native/build.py``."""
from __future__ import annotations

try:
    from ._native import ShmRing, copy_jobs, crc32c, featurize_batch, featurize_batch_raw, pack_rows  # noqa: F401
    AVAILABLE = True
except ImportError:  # pragma: no cover - not built yet
    AVAILABLE = False
    ShmRing = copy_jobs = crc32c = featurize_batch = featurize_batch_raw = pack_rows = None
