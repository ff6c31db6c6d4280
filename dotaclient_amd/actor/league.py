"""Opponent league over the weight history (generalises the reference's mini-league, agent.py:760-765).

The reference keeps the last 64 ``(version, state_dict)`` pairs (``MAX_AGE_WEIGHTSTORE``, agent.py:54) and, with
probability ``1 − latest_weights_prob``, lets one random team play the OLDEST of them; that team does not roll out
(agent.py:167-184, 360-362). :class:`League` keeps that behaviour as ``mode='oldest'`` (the default, bit-for-bit
the reference's choice) and adds the sampling schemes BASELINE.json's league config asks for:

* ``uniform`` — any stored snapshot with equal probability (fictitious self-play);
* ``recent`` — geometric preference for recent snapshots, ``p_i ∝ decay^(age_i)``;
* ``pfsp`` — prioritised fictitious self-play: ``p_i ∝ (1 − w_i)^power`` where ``w_i`` is the learner's running
  win rate against snapshot ``i`` (a Beta(1,1)-smoothed estimate), so opponents the learner still loses to are
  played more often.

Results are fed back with :meth:`record` at game end (the actor knows which team used the latest weights).
"""
from __future__ import annotations

import random
from collections import OrderedDict
from typing import Dict, Optional, Tuple

MODES = ('oldest', 'uniform', 'recent', 'pfsp')


class League:
    def __init__(self, store, mode: str = 'oldest', decay: float = 0.9, pfsp_power: float = 2.0,
                 rng: Optional[random.Random] = None, cache_size: int = 4):
        if mode not in MODES:
            raise ValueError(f'league mode must be one of {MODES}, got {mode!r}')
        self.store = store
        self.mode = mode
        self.decay = float(decay)
        self.pfsp_power = float(pfsp_power)
        self.rng = rng or random.Random()
        self.wins: Dict[int, float] = {}
        self.games: Dict[int, float] = {}
        self.results: Dict[int, list] = {}     # per opponent version: every game's result (1 / 0 / 0.5), in order
        self._cache: 'OrderedDict[int, object]' = OrderedDict()
        self.cache_size = cache_size

    # ------------------------------------------------------------------------------------------------
    def weights(self):
        """Sampling weights over ``store.weights`` (oldest first)."""
        hist = list(self.store.weights)
        n = len(hist)
        if n == 0:
            return []
        if self.mode == 'oldest':
            return [1.0] + [0.0] * (n - 1)
        if self.mode == 'uniform':
            return [1.0] * n
        if self.mode == 'recent':
            return [self.decay ** (n - 1 - i) for i in range(n)]
        out = []
        for version, _ in hist:
            w = self.win_rate(version)
            out.append(max(1e-3, (1.0 - w) ** self.pfsp_power))
        return out

    def sample(self) -> Tuple[int, dict]:
        hist = list(self.store.weights)
        if not hist:
            raise RuntimeError('league: the weight store is empty')
        w = self.weights()
        return self.rng.choices(hist, weights=w, k=1)[0]

    def policy(self, version_state):
        """A (cached) eval-mode Policy for a snapshot — games against the same snapshot share it."""
        version = int(version_state[0])
        p = self._cache.get(version)
        if p is None:
            p = self.store.policy_for(version_state)
            self._cache[version] = p
            while len(self._cache) > self.cache_size:
                self._cache.popitem(last=False)
        else:
            self._cache.move_to_end(version)
        return p

    # ------------------------------------------------------------------------------------------------
    def record(self, opponent_version: int, learner_result: float):
        """``learner_result`` = 1 win, 0 loss, 0.5 draw/timeout for the team that used the latest weights."""
        v = int(opponent_version)
        self.wins[v] = self.wins.get(v, 0.0) + float(learner_result)
        self.games[v] = self.games.get(v, 0.0) + 1.0
        self.results.setdefault(v, []).append(float(learner_result))

    def win_rate(self, version: int) -> float:
        v = int(version)
        return (self.wins.get(v, 0.0) + 1.0) / (self.games.get(v, 0.0) + 2.0)

    def stats(self):
        return {v: (self.win_rate(v), int(self.games.get(v, 0))) for v, _ in self.store.weights}
