"""Return / advantage computation and running reward statistics (host reference implementations).

* :func:`discount` — reverse linear recurrence ``G_t = r_t + γ G_{t+1}`` (reference optimizer.py:52-53, which uses
  ``scipy.signal.lfilter``; we keep scipy's semantics but do not require it).
* :func:`gae` — generalized advantage estimation (north-star PPO path; SURVEY §2.3 K-return).
* :class:`RunningMeanStd` — per-team EMA of mean/std with factor 0.99 (optimizer.py:213, 335-343).

The device versions are the HIP segmented reverse-scan kernels in ``dotaclient_amd/ops/csrc/scan.hip``; these numpy
versions are their test oracles.
"""
from __future__ import annotations

from typing import Dict, Optional

import numpy as np

from ..constants import EPS


def discount(x: np.ndarray, gamma: float) -> np.ndarray:
    """Discounted cumulative sum along axis 0, returned as float32 (optimizer.py:52-53)."""
    x = np.asarray(x, dtype=np.float64)
    out = np.empty_like(x)
    acc = np.zeros(x.shape[1:], dtype=np.float64)
    for t in range(x.shape[0] - 1, -1, -1):
        acc = x[t] + gamma * acc
        out[t] = acc
    return out.astype(np.float32)


def gae(rewards: np.ndarray, values: np.ndarray, bootstrap_value: float, gamma: float, lam: float,
        done: bool = True):
    """GAE(γ, λ) over one rollout. ``values`` are the behaviour policy's V(s_t).

    Returns (advantages, returns) as float32, with returns = advantages + values.
    ``done`` means the episode terminated after the last step (no bootstrap).
    """
    r = np.asarray(rewards, dtype=np.float64)
    v = np.asarray(values, dtype=np.float64)
    T = r.shape[0]
    adv = np.zeros(T, dtype=np.float64)
    next_v = 0.0 if done else float(bootstrap_value)
    acc = 0.0
    for t in range(T - 1, -1, -1):
        delta = r[t] + gamma * next_v - v[t]
        acc = delta + gamma * lam * acc
        adv[t] = acc
        next_v = v[t]
    return adv.astype(np.float32), (adv + v).astype(np.float32)


class RunningMeanStd:
    """Per-key EMA of batch mean / std (optimizer.py:335-343). The first update initialises the statistics."""

    def __init__(self, factor: float = 0.99):
        self.factor = factor
        self.mean: Dict[int, Optional[float]] = {}
        self.std: Dict[int, Optional[float]] = {}

    def update(self, x: np.ndarray, key: int):
        m, s = float(np.mean(x)), float(np.std(x))
        if self.mean.get(key) is None:
            self.mean[key], self.std[key] = m, s
        else:
            f = self.factor
            self.mean[key] = self.mean[key] * f + m * (1 - f)
            self.std[key] = self.std[key] * f + s * (1 - f)

    def normalize(self, x: np.ndarray, key: int) -> np.ndarray:
        return ((np.asarray(x) - self.mean[key]) / (self.std[key] + EPS)).astype(np.float32)

    def state_dict(self):
        return {'factor': self.factor, 'mean': dict(self.mean), 'std': dict(self.std)}

    def load_state_dict(self, d):
        self.factor = d['factor']
        self.mean = {int(k): v for k, v in d['mean'].items()}
        self.std = {int(k): v for k, v in d['std'].items()}
