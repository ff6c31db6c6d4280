"""Versioned weight store with hot-swap and opponent pool (reference agent.py:161-223, 760-765).

* ``WeightStore`` keeps the last ``maxlen`` (=64, ``MAX_AGE_WEIGHTSTORE``) ``(version, state_dict)`` pairs and a
  ``latest_policy`` that is updated in place whenever a new model arrives — players holding it see new weights
  mid-game, exactly like the reference's synced players (agent.py:293-297).
* ``oldest_weights`` / ``latest_weights`` back the reference's mini-league: with probability
  ``1 − latest_weights_prob`` one team plays the oldest stored weights and does not roll out (agent.py:760-765).
* :class:`~dotaclient_amd.actor.league.League` extends that into a configurable league (BASELINE config 5):
  uniform over history, recency-weighted, or prioritised fictitious self-play from recorded results.
"""
from __future__ import annotations

import threading
from collections import deque
from typing import Optional

import torch

from ..models.policy import Policy
from ..transport.codec import decode_state_dict


class WeightStore:
    def __init__(self, config='compat', maxlen: int = 64, device='cpu'):
        self.config = config
        self.device = device
        self.weights = deque(maxlen=maxlen)
        self.latest_policy = Policy(config).to(device).eval()
        self.latest_policy.weight_version = -1
        self.ready = threading.Event()
        self._lock = threading.Lock()

    def add(self, version: int, state_dict):
        with self._lock:
            self.weights.append((int(version), state_dict))
            self.latest_policy.load_state_dict(state_dict, strict=True)
            self.latest_policy.weight_version = int(version)
        self.ready.set()

    def add_bytes(self, version: int, body: bytes):
        self.add(version, decode_state_dict(body))

    def oldest_weights(self):
        return self.weights[0]

    def latest_weights(self):
        return self.weights[-1]

    def policy_for(self, version_state) -> Policy:
        version, state_dict = version_state
        p = Policy(self.config).to(self.device).eval()
        p.load_state_dict(state_dict, strict=True)
        p.weight_version = version
        return p

    def load_file(self, path: str, version: int = -1):
        self.add(version, torch.load(path, map_location='cpu', weights_only=True))

    def wait_ready(self, timeout: Optional[float] = None) -> bool:
        return self.ready.wait(timeout)
