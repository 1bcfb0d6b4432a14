"""BoardConfig: board shape + token bit layout + action-id codec.

Drop-in for ``match3tile.boardConfig.BoardConfig`` of ThorLL/Element-Crush-Gym
(reference match3tile/boardConfig.py:5-69): same constructor fields, same
derived attributes and values, same decode/encode results (including the
truncating ``int()`` in decode and the adjacency assertion in encode).

Token layout for T tile types, with k = ceil(log2(T + 1)):
  type_mask         TM = 2^k - 1          (tile type lives in the low k bits)
  h_line            H  = 2^k
  v_line            V  = 2^(k+1)
  bomb              B  = 3 * 2^k          (== special_type_mask)
  mega_token        M  = 2^(k+2)
e.g. 9x9x6 -> TM 7, H 8, V 16, B 24, M 32; 16x16x8 -> TM 15, H 16, V 32, B 48, M 64.
"""
from __future__ import annotations

import math
from dataclasses import dataclass, field

import numpy as np


def _token_layout(types: int) -> dict:
    k = math.ceil(math.log2(types + 1))
    tm = (1 << k) - 1
    stm = (1 << (k + 1)) + (1 << k)          # == 2^(k+1) + 1 + tm
    return dict(type_mask=tm, special_type_mask=stm, h_line=tm + 1, v_line=2 * (tm + 1),
                bomb=stm, mega_token=tm + stm + 1)


def _trunc_div(x: int, d: int) -> int:
    """Python's int(x / d) for the small integers used here (truncates toward 0)."""
    q = abs(x) // d
    return q if x >= 0 else -q


@dataclass(frozen=True)
class BoardConfig:
    seed: int = None
    rows: int = 9
    columns: int = 9
    types: int = 6

    shape: tuple = field(init=False)
    action_space: int = field(init=False)
    actions: dict = field(init=False)
    type_mask: int = field(init=False)
    special_type_mask: int = field(init=False)
    h_line: int = field(init=False)
    v_line: int = field(init=False)
    bomb: int = field(init=False)
    mega_token: int = field(init=False)

    def __post_init__(self):
        put = object.__setattr__
        # A falsy seed draws one from numpy's global RNG, exactly like the
        # reference (seed=0 therefore means "random").
        if not self.seed:
            put(self, "seed", np.random.randint(0, 2 ** 31 - 1))
        put(self, "shape", (self.rows, self.columns))
        n_actions = 2 * self.rows * (self.columns - 1)
        put(self, "action_space", n_actions)
        put(self, "actions", {a: self.decode(a) for a in range(n_actions)})
        for name, value in _token_layout(self.types).items():
            put(self, name, value)

    def decode(self, action):
        """Action id -> ((row1, col1), (row2, col2)); row r owns ids r*(2C-1)...,
        first the C-1 horizontal swaps then the C vertical ones."""
        stride = 2 * self.columns - 1
        n_h = self.columns - 1
        offset = action - stride * int(action / stride)
        if offset < n_h:
            col = action % stride
            row = _trunc_div(action - col, stride)
            return (row, col), (row, col + 1)
        col = action % stride - n_h
        row = _trunc_div(action - 3 - col, stride)
        return (row, col), (row + 1, col)

    def encode(self, tile1, tile2):
        """Adjacent cell pair -> action id (inverse of decode)."""
        (r1, c1), (r2, c2) = tile1, tile2
        vertical = c1 == c2 and abs(r1 - r2) == 1
        horizontal = r1 == r2 and abs(c1 - c2) == 1
        assert vertical or horizontal, 'source and target must be adjacent'
        base = min(r1, r2) * (2 * self.columns - 1) + min(c1, c2)
        return base + (self.columns - 1 if c1 == c2 else 0)
