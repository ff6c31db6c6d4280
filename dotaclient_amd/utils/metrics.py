"""Metrics sink: JSONL (always) + TensorBoard event files (scalars/histograms/images).

Tag names are the reference's (optimizer.py:500-561; agent.py:415-428) so existing dashboards keep working:
``steps per s``, ``reward_per_sec/{sum,<key>}``, ``loss/{sum,policy,entropy,advantage}``, ``entropy``,
``entropy/<head>``, ``advantage``, ``avg_rollout_len``, ``avg_weight_age``, ``rewards/running_{mean,std}_<team>``,
``mq_size``; histograms ``losses``, ``rollout_lens``, ``weight_age``, ``rewards_per_sec_per_rollout``,
``param/<name>``; image ``canvas``; validation ``game/canvas``, ``game/steps``, ``game/rewards_sum``,
``game/rewards_<key>``. MI355X additions: ``samples per s per gpu``, ``time/<stage>``, ``allreduce_ms``, ...
"""
from __future__ import annotations

import json
import os
import time
from typing import Dict, Optional

import numpy as np

from .tfevents import EventWriter


def _to_float(v):
    try:
        import torch
        if isinstance(v, torch.Tensor):
            return float(v.detach().float().mean().item())
    except ImportError:  # pragma: no cover
        pass
    return float(v)


class MetricsWriter:
    def __init__(self, log_dir: Optional[str], tensorboard: bool = True, jsonl_name: str = 'metrics.jsonl'):
        self.log_dir = log_dir
        self._jsonl = None
        self.tb = None
        self.on_flush = []          # callbacks after every flush (e.g. mirror the events file to an artifact store)
        if log_dir:
            os.makedirs(log_dir, exist_ok=True)
            self._jsonl = open(os.path.join(log_dir, jsonl_name), 'a')
            if tensorboard:
                self.tb = EventWriter(log_dir)

    @property
    def events_filename(self):
        return self.tb.path if self.tb else None

    def add_scalars(self, metrics: Dict[str, float], step: int):
        rec = {'step': int(step), 'time': time.time()}
        for k, v in metrics.items():
            f = _to_float(v)
            rec[k] = f
            if self.tb:
                self.tb.add_scalar(k, f, step)
        if self._jsonl:
            self._jsonl.write(json.dumps(rec) + '\n')

    def add_scalar(self, tag, value, step):
        self.add_scalars({tag: value}, step)

    def add_histogram(self, tag, values, step):
        if self.tb:
            self.tb.add_histogram(tag, np.asarray(values, dtype=np.float64), step)

    def add_image(self, tag, img, step):
        if self.tb and img is not None:
            self.tb.add_image(tag, img, step)

    def flush(self):
        if self._jsonl:
            self._jsonl.flush()
        if self.tb:
            self.tb.flush()
        for cb in self.on_flush:
            cb(self)

    def close(self):
        self.flush()
        if self._jsonl:
            self._jsonl.close()
        if self.tb:
            self.tb.close()


class StageTimer:
    """Per-stage wall timers (ingest / h2d / train / allreduce / publish), reported as ``time/<stage>`` metrics."""

    def __init__(self):
        self.t = {}
        self._t0 = {}

    def start(self, name):
        self._t0[name] = time.perf_counter()

    def stop(self, name):
        self.t[name] = self.t.get(name, 0.0) + time.perf_counter() - self._t0.pop(name)

    def add(self, name, seconds: float):
        """Time measured elsewhere (another thread's stage) reported with this iteration's timers."""
        self.t[name] = self.t.get(name, 0.0) + float(seconds)

    def pop(self) -> Dict[str, float]:
        out = {f'time/{k}': v for k, v in self.t.items()}
        self.t = {}
        return out
