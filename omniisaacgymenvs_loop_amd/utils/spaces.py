"""Minimal gym.spaces stand-ins (gym is not a dependency of the hot path).

Same attributes rl_games reads: Box.low/.high/.shape/.dtype, Dict.spaces
(rl_games/rl_games/common/experience.py:300-330, a2c_common.py:210-215)."""
from __future__ import annotations

import numpy as np


class Box:
    def __init__(self, low, high, shape=None, dtype=np.float32):
        if shape is not None:
            low = np.full(shape, low, dtype=dtype)
            high = np.full(shape, high, dtype=dtype)
        self.low = np.asarray(low, dtype=dtype)
        self.high = np.asarray(high, dtype=dtype)
        self.shape = tuple(self.low.shape)
        self.dtype = np.dtype(dtype)

    def __repr__(self):
        return f"Box({self.low.min()}, {self.high.max()}, {self.shape}, {self.dtype})"


class DictSpace:
    def __init__(self, spaces):
        self.spaces = dict(spaces)

    def __getitem__(self, k):
        return self.spaces[k]

    def __repr__(self):
        return f"Dict({self.spaces})"
