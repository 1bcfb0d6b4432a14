"""BoardV2: the reference's immutable board state, computed on the MI355X.

Drop-in for ``match3tile.boardv2.BoardV2`` (reference match3tile/boardv2.py:
11-226) as used by mctslib (State interface), samplerTasks.py and dataset.py:
constructor ``BoardV2(n_actions, cfg=BoardConfig(), array=None)``, attributes
``cfg``, ``n_actions``, ``array`` (int64 [rows, columns]), properties
``legal_actions``/``is_terminal``/``reward``/``greedy_action``, methods
``apply_action``/``clone``, plus ``random_action()`` (README.md:23).

Every rule evaluation (initial board, apply_action, legal_actions) runs in the
HIP kernels of libm3.so. What stays on the host is bookkeeping the reference
also does in Python, including its *side effect on numpy's global RNG*: the
reference reseeds ``np.random`` with ``cfg.seed`` inside apply_action and
consumes draws from it, and callers (samplerTasks.random_task, MCTS.rollout)
sample their next action from that global stream. The kernels report how many
raw MT19937 outputs were consumed since the last reseed, and the facade
replays the same state into numpy's global generator, so those callers make
exactly the choices they make with the reference.
"""
from __future__ import annotations

from typing import List

import numpy as np

from . import _native
from .boardConfig import BoardConfig
from .state import State


def _sync_global_rng(seed: int, draws: int) -> None:
    """numpy global RNG := seed(seed) advanced by `draws` raw 32-bit outputs."""
    np.random.seed(seed)
    if draws:
        np.random.mtrand._rand._bit_generator.random_raw(int(draws))


def _ctx(cfg: BoardConfig) -> _native.Context:
    return _native.context(cfg.rows, cfg.columns, cfg.types)


def _ids_past_board(cfg: BoardConfig) -> None:
    """rows < columns: the last action ids decode to a swap with row `rows` (boardConfig.py:27,45-59),
    so the reference's legal_actions -- called by every apply_action too (boardv2.py:188) -- raises
    numpy's IndexError. Same here (the kernels refuse such a shape for anything but a reset)."""
    if cfg.rows < cfg.columns:
        raise IndexError(f"index {cfg.rows} is out of bounds for axis 0 with size {cfg.rows}")


class BoardV2(State):
    # the reference's default argument is built once, at import (boardv2.py:12)
    def __init__(self, n_actions: int, cfg=BoardConfig(), array: np.ndarray = None):
        self.cfg = cfg
        self.n_actions = n_actions
        self._reward = 0
        if array is None:
            np.random.seed(cfg.seed)  # boardv2.py:20 -- raises ValueError outside [0, 2**32) like the reference
            boards, draws, _ = _ctx(cfg).init_boards([int(cfg.seed) & 0xFFFFFFFF])
            self.array = boards[0].astype(np.int64)
            _sync_global_rng(cfg.seed, int(draws[0]))       # boardv2.py:20-27 leave the RNG here
        else:
            self.array = array
        self._actions = []

    # ---- State interface -------------------------------------------------------
    @property
    def legal_actions(self) -> List[int]:
        _ids_past_board(self.cfg)
        if len(self._actions) == 0:                          # cached only while non-empty
            self._actions = _ctx(self.cfg).legal_actions(self.array)
        return self._actions

    def clone(self) -> "BoardV2":
        other = BoardV2(self.n_actions, self.cfg, np.copy(self.array))
        other._reward = self._reward
        other._actions = self._actions
        return other

    def apply_action(self, action) -> "BoardV2":
        if self.is_terminal:
            return self
        if action not in self.cfg.actions:                   # reseed happens before the KeyError
            np.random.seed(self.cfg.seed)
            raise KeyError(action)
        if self.cfg.rows < self.cfg.columns:
            np.random.seed(self.cfg.seed)
            _ids_past_board(self.cfg)
        res = _ctx(self.cfg).apply_actions(self.array, int(self.cfg.seed) & 0xFFFFFFFF, self.n_actions,
                                           int(action))
        _sync_global_rng(self.cfg.seed, int(res["draws"][0]))
        nxt = BoardV2(self.n_actions - 1, self.cfg, res["boards"][0].astype(np.int64))
        nxt._reward = self._reward + int(res["reward"][0])
        return nxt

    @property
    def is_terminal(self) -> bool:
        return self.n_actions < 1

    @property
    def reward(self) -> float:
        return self._reward

    # ---- extras used by callers ----------------------------------------------------
    @property
    def greedy_action(self) -> int:
        """Best one-step legal action (boardv2.py:209-218), all candidates in ONE launch."""
        legal = self.legal_actions
        if not legal:
            return None
        n = len(legal)
        res = _ctx(self.cfg).apply_actions(np.broadcast_to(self.array, (n,) + self.array.shape),
                                           int(self.cfg.seed) & 0xFFFFFFFF, self.n_actions, legal)
        best, best_reward = None, -1
        for a, r in zip(legal, res["reward"]):
            if self._reward + int(r) > best_reward:          # first maximum wins, as in the loop
                best_reward, best = self._reward + int(r), a
        if not self.is_terminal:  # a terminal board's apply_action never touches the RNG
            _sync_global_rng(self.cfg.seed, int(res["draws"][-1]))  # state after the last apply_action
        return best

    def random_action(self) -> int:
        """env.board.random_action() of README.md:23: np.random.choice(legal_actions)."""
        return int(np.random.choice(self.legal_actions))
