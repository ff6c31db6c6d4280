"""Artifact store: where checkpoints, metric event files and validation outputs are mirrored off the learner node.

The reference uploads every ``model_%09d.pt`` and the tensorboard events file to the GCS bucket ``dotaservice`` under
the run's ``log_dir`` (optimizer.py:212, 559, 691-715), resumes by listing that bucket prefix (optimizer.py:299-315)
and lets an agent start from a model blob (agent.py:186-193, ``--model``); ``--run-local`` turns all of it off.
Here the same three operations run against a URL-addressed store:

* ``file:///shared/runs`` or a plain directory — a shared filesystem / PVC mount (the usual k8s setup on an MI355X
  cluster without object storage);
* any fsspec URL whose filesystem is importable (``gs://bucket/prefix`` needs ``gcsfs``, ``s3://`` needs ``s3fs``;
  ``memory://`` for tests). A URL whose backend is missing fails loudly at construction.

Uploads run on a background thread with a bounded queue (an upload never stalls an optimizer step; the reference
uploaded synchronously inside the training loop), and ``flush()`` waits for them (called at shutdown).
"""
from __future__ import annotations

import logging
import os
import queue
import shutil
import threading
from typing import List, Optional

logger = logging.getLogger(__name__)


class ArtifactStore:
    """put/get/list of opaque files under a root URL; keys are '/'-separated relative paths."""

    def put(self, local_path: str, key: str):
        raise NotImplementedError

    def get(self, key: str, local_path: str):
        raise NotImplementedError

    def list(self, prefix: str = '') -> List[str]:
        raise NotImplementedError

    def exists(self, key: str) -> bool:
        return key in self.list(os.path.dirname(key))


class LocalStore(ArtifactStore):
    def __init__(self, root: str):
        self.root = os.path.abspath(root)
        os.makedirs(self.root, exist_ok=True)

    def _p(self, key: str) -> str:
        p = os.path.abspath(os.path.join(self.root, key))
        if not p.startswith(self.root):
            raise ValueError(f'key escapes the store root: {key!r}')
        return p

    def put(self, local_path: str, key: str):
        dst = self._p(key)
        os.makedirs(os.path.dirname(dst), exist_ok=True)
        tmp = dst + '.part'
        shutil.copyfile(local_path, tmp)
        os.replace(tmp, dst)                       # readers never see a partial file

    def get(self, key: str, local_path: str):
        os.makedirs(os.path.dirname(os.path.abspath(local_path)), exist_ok=True)
        shutil.copyfile(self._p(key), local_path)

    def list(self, prefix: str = '') -> List[str]:
        base = self._p(prefix) if prefix else self.root
        if not os.path.isdir(base):
            return []
        out = []
        for dirpath, _, files in os.walk(base):
            for f in files:
                if f.endswith('.part'):
                    continue
                out.append(os.path.relpath(os.path.join(dirpath, f), self.root).replace(os.sep, '/'))
        return sorted(out)

    def exists(self, key: str) -> bool:
        return os.path.isfile(self._p(key))


class FsspecStore(ArtifactStore):
    def __init__(self, url: str):
        import fsspec
        self.fs, root = fsspec.core.url_to_fs(url)
        self.root = root.rstrip('/')

    def _p(self, key: str) -> str:
        return f'{self.root}/{key}' if key else self.root

    def put(self, local_path: str, key: str):
        self.fs.put_file(local_path, self._p(key))

    def get(self, key: str, local_path: str):
        os.makedirs(os.path.dirname(os.path.abspath(local_path)), exist_ok=True)
        self.fs.get_file(self._p(key), local_path)

    def list(self, prefix: str = '') -> List[str]:
        base = self._p(prefix)
        if not self.fs.exists(base):
            return []
        files = self.fs.find(base)
        strip = self.root.lstrip('/')
        return sorted(f.lstrip('/')[len(strip):].lstrip('/') for f in files)

    def exists(self, key: str) -> bool:
        return self.fs.exists(self._p(key))


def open_store(url: Optional[str]) -> Optional[ArtifactStore]:
    """``None``/'' → no store; ``file://…`` or a plain path → :class:`LocalStore`; other schemes → fsspec."""
    if not url:
        return None
    if url.startswith('file://'):
        return LocalStore(url[len('file://'):])
    if '://' not in url:
        return LocalStore(url)
    try:
        return FsspecStore(url)
    except (ImportError, ValueError) as e:
        raise RuntimeError(f'artifact store {url!r}: backend not available in this environment ({e})') from e


class Uploader:
    """Background uploads to a store with a bounded queue (back-pressure instead of unbounded memory)."""

    def __init__(self, store: ArtifactStore, maxsize: int = 16):
        self.store = store
        self.q: 'queue.Queue' = queue.Queue(maxsize=maxsize)
        self.errors = 0
        self._t = threading.Thread(target=self._run, name='artifact-uploader', daemon=True)
        self._t.start()

    def _run(self):
        while True:
            item = self.q.get()
            if item is None:
                self.q.task_done()
                return
            local, key = item
            try:
                self.store.put(local, key)
            except Exception as e:  # keep training; the next checkpoint supersedes this one
                self.errors += 1
                logger.warning('artifact upload %s -> %s failed: %s', local, key, e)
            finally:
                self.q.task_done()

    def submit(self, local_path: str, key: str):
        self.q.put((local_path, key))

    def flush(self):
        self.q.join()

    def close(self):
        self.q.put(None)
        self._t.join(timeout=60)


def fetch_latest_checkpoint(store: ArtifactStore, prefix: str, log_dir: str) -> Optional[str]:
    """Resume from the store (reference optimizer.py:299-315 lists the bucket): download the lexicographically latest
    ``model_*.pt`` under ``prefix`` (and its trainer-state sidecar if present) into ``log_dir``; returns the local
    model path or None."""
    from .checkpoint import MODEL_FILENAME_FMT, STATE_FILENAME_FMT, iteration_from_model_filename
    keys = [k for k in store.list(prefix) if os.path.basename(k).startswith('model_') and k.endswith('.pt')]
    if not keys:
        return None
    key = sorted(keys, key=os.path.basename)[-1]
    it = iteration_from_model_filename(key)
    local = os.path.join(log_dir, MODEL_FILENAME_FMT % it)
    store.get(key, local)
    skey = os.path.join(os.path.dirname(key), STATE_FILENAME_FMT % it).replace(os.sep, '/')
    if store.exists(skey):
        store.get(skey, os.path.join(log_dir, STATE_FILENAME_FMT % it))
    return local


def resolve_model_path(spec: str, cache_dir: Optional[str] = None) -> str:
    """A model reference for ``--model``/``--pretrained-model``: a local file, or ``<store-url>#<key>`` /
    ``gs://bucket/path/model.pt`` style URL, downloaded into ``cache_dir`` (reference agent.py:186-193)."""
    if '://' not in spec or spec.startswith('file://') and '#' not in spec:
        return spec[len('file://'):] if spec.startswith('file://') else spec
    if '#' in spec:
        url, key = spec.split('#', 1)
    else:
        url, key = spec.rsplit('/', 1)
    store = open_store(url)
    import tempfile
    cache_dir = cache_dir or tempfile.mkdtemp(prefix='dca_model_')
    local = os.path.join(cache_dir, os.path.basename(key))
    store.get(key, local)
    return local


def mirror_events(uploader: Uploader, prefix: str):
    """A MetricsWriter ``on_flush`` callback that uploads a snapshot of the events and JSONL files after each flush
    (the validation agent's tensorboard output, reference agent.py:97-100, 415-428)."""
    def cb(writer):
        for path in (writer.events_filename,
                     os.path.join(writer.log_dir, 'metrics.jsonl') if writer.log_dir else None):
            if path and os.path.exists(path):
                snap = path + '.snapshot'
                shutil.copyfile(path, snap)
                uploader.submit(snap, f'{prefix}/{os.path.basename(path)}')
    return cb
