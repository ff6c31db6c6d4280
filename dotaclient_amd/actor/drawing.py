"""Trajectory canvas shipped with each experience message (reference agent.py:719-741)."""
from __future__ import annotations

import numpy as np

from ..protos import TEAM_DIRE, TEAM_RADIANT, UnitType
from ..utils.png import save_png


class Drawing:
    TEAM_COLORS = {TEAM_DIRE: [255, 0, 0], TEAM_RADIANT: [0, 255, 0]}

    def __init__(self, size: int = 256):
        self.size = size
        self.sizeh = size / 2.
        self.canvas = np.ones((size, size, 3), dtype=np.uint8) * 255
        self.ratio = self.sizeh / 8000.

    def normalize_location(self, l):
        x = int((l.x * self.ratio) + self.sizeh)
        y = int(self.size - (l.y * self.ratio) - self.sizeh)
        return min(max(x, 0), self.size - 1), min(max(y, 0), self.size - 1)

    def step(self, state, team_id: int, player_id: int):
        for unit in state.units:
            if unit.unit_type == UnitType.HERO and unit.player_id == player_id:
                x, y = self.normalize_location(unit.location)
                self.canvas[y, x] = self.TEAM_COLORS[team_id]

    def save(self, stem: str):
        save_png(f'{stem}.png', self.canvas)
