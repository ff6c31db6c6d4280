"""Fault injection for failure-path testing (kill actor, drop messages, NaN injection).

The reference's failure model is crash-and-restart (agent exceptions end the pod, the optimizer raises on a NaN
loss and k8s restarts it from the last checkpoint — agent.py:896-900, optimizer.py:674-676; optimizer.jsonnet
``restartPolicy: OnFailure``). These hooks let tests (and chaos runs) exercise exactly those paths:

    DCA_FAULTS="drop_xp=0.2,corrupt_xp=0.05,actor_crash=0.001,nan_loss_at=3,seed=1"

* ``drop_xp``      probability an actor silently drops a rollout instead of publishing it (message loss);
* ``corrupt_xp``   probability a published rollout gets a byte flipped (the learner must reject it by CRC);
* ``actor_crash``  probability per actor step of an injected exception (the supervisor must restart the actor);
* ``nan_loss_at``  learner iteration whose loss is replaced by NaN (the learner must raise, then resume).

With ``DCA_FAULTS`` unset every hook is a no-op.
"""
from __future__ import annotations

import os
import random
from typing import Dict, Optional


class Faults:
    def __init__(self, spec: Optional[str] = None):
        self.cfg: Dict[str, float] = {}
        if spec:
            for kv in spec.split(','):
                if kv.strip():
                    k, v = kv.split('=', 1)
                    self.cfg[k.strip()] = float(v)
        self.rng = random.Random(int(self.cfg.get('seed', 0)))
        self.counts: Dict[str, int] = {}

    @property
    def active(self) -> bool:
        return bool(self.cfg)

    def should(self, name: str) -> bool:
        p = self.cfg.get(name, 0.0)
        hit = p > 0 and self.rng.random() < p
        if hit:
            self.counts[name] = self.counts.get(name, 0) + 1
        return hit

    def corrupt(self, body: bytes) -> bytes:
        b = bytearray(body)
        i = self.rng.randrange(len(b))
        b[i] ^= 0xFF
        return bytes(b)

    def nan_loss(self, iteration: int) -> bool:
        at = self.cfg.get('nan_loss_at')
        hit = at is not None and int(at) == int(iteration)
        if hit:
            self.counts['nan_loss'] = self.counts.get('nan_loss', 0) + 1
        return hit


_FAULTS: Optional[Faults] = None


def faults() -> Faults:
    """Process-wide injector configured from ``DCA_FAULTS`` (re-read when the variable changes)."""
    global _FAULTS
    spec = os.environ.get('DCA_FAULTS', '')
    if _FAULTS is None or getattr(_FAULTS, '_spec', None) != spec:
        _FAULTS = Faults(spec)
        _FAULTS._spec = spec
    return _FAULTS
