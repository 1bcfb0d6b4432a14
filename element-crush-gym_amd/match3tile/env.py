"""Match3Env: the gym-style single-board environment.

Drop-in for ``match3tile.env.Match3Env`` (reference match3tile/env.py:8-82,
usage README.md:18-31). The reference class does not run at the snapshot
(``BoardV2(..., seed=...)`` has no such keyword, env.py:38,64, and
``apply_action`` returns a board, not ``(score, event)``, env.py:50), so this
is the intended behaviour restated:

  step(a): reward = board'.reward - board.reward; score += reward;
           moves_taken += 1; truncated = score >= env_goal;
           done = truncated or moves_taken == num_moves;
           returns (board'.array, reward, done, truncated, {})
  reset(seed=None): keeps the reference's seed arithmetic
           ((1 + seed) % 2**32 - 1, i.e. the same seed again).

``action_space`` / ``observation_space`` are gymnasium spaces when gymnasium
is importable, else small duck-typed stand-ins with ``n``/``shape``/
``sample()``/``contains()``. Rendering (pygame in the reference) is out of
scope; ``render_mode='human'`` prints the board as text.
"""
from __future__ import annotations

from random import randint

import numpy as np

from .boardConfig import BoardConfig
from .boardv2 import BoardV2

try:  # optional dependency, pinned by the reference (requirements.txt:9)
    from gymnasium import spaces as _spaces
except Exception:  # pragma: no cover - gymnasium is not installed in this image
    _spaces = None


class Discrete:
    def __init__(self, n: int):
        self.n = int(n)
        self.shape = ()
        self.dtype = np.int64

    def sample(self) -> int:
        return int(np.random.randint(self.n))

    def contains(self, x) -> bool:
        return isinstance(x, (int, np.integer)) and 0 <= int(x) < self.n

    def __repr__(self):
        return f"Discrete({self.n})"


class Box:
    def __init__(self, low, high, shape, dtype=np.int64):
        self.low, self.high, self.shape, self.dtype = low, high, tuple(shape), dtype

    def sample(self):
        return np.random.randint(self.low, self.high + 1, size=self.shape).astype(self.dtype)

    def contains(self, x) -> bool:
        x = np.asarray(x)
        return x.shape == self.shape and bool(((x >= self.low) & (x <= self.high)).all())

    def __repr__(self):
        return f"Box({self.low}, {self.high}, {self.shape}, {np.dtype(self.dtype).name})"


class Match3Env:
    metadata = {"render_modes": ["human"], "render_fps": 60, "animation_speed": 1}

    def __init__(self, width: int = 9, height: int = 9, num_types: int = 6, num_moves: int = 20,
                 env_goal: int = 500, seed: int = None, render_mode: str = None):
        self.seed = seed if seed is not None else randint(0, 2 ** 32 - 1)
        assert width >= 3 and height >= 3, "Board size too small: min size: 3x3"
        assert render_mode is None or render_mode in self.metadata["render_modes"]
        self.width, self.height, self.num_types = width, height, num_types
        self.env_goal, self.num_moves = env_goal, num_moves
        self.render_mode = render_mode
        self.score, self.moves_taken = 0, 0
        self.actions = []
        self.board = self._new_board()
        # env.py:36 counts adjacent cell pairs; it equals BoardConfig.action_space (the id
        # range apply_action accepts) on square boards only -- kept as the reference has it
        n_act = height * (width - 1) + width * (height - 1)
        if _spaces is not None:
            self.action_space = _spaces.Discrete(n_act)
            self.observation_space = _spaces.Box(0, self.board.cfg.mega_token, (height, width), np.int64)
        else:
            self.action_space = Discrete(n_act)
            self.observation_space = Box(0, self.board.cfg.mega_token, (height, width), np.int64)

    def _new_board(self) -> BoardV2:
        cfg = BoardConfig(seed=self.seed, rows=self.height, columns=self.width, types=self.num_types)
        return BoardV2(self.num_moves, cfg)

    def init(self):
        return self.board.array

    def step(self, action: int):
        self.actions = self.board.legal_actions
        before = self.board.reward
        self.board = self.board.apply_action(action)
        reward = self.board.reward - before
        self.score += reward
        self.moves_taken += 1
        truncated = self.score >= self.env_goal
        done = truncated or self.num_moves == self.moves_taken
        return self.board.array, reward, done, truncated, {}

    def reset(self, seed=None):
        self.seed = seed if seed is not None else (1 + self.seed) % 2 ** 32 - 1
        self.score, self.moves_taken = 0, 0
        self.board = self._new_board()
        return self.board.array, {}

    def render(self):
        if self.render_mode is None:
            return None
        text = "\n".join(" ".join(f"{v:3d}" for v in row) for row in self.board.array)
        print(text)
        return text
