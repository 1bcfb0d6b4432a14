"""MCTS consumer of the step, host side, on CPU.

* The oracle's restatement of ``MCTS.rollout`` (mctslib/standard/mcts.py:14-19,
  oracle/m3_oracle.c m3o_rollout) against rollouts the real reference played
  (tests/golden/gen_golden_mcts.py -> mcts.npz): return, step count, the global
  numpy stream's final position.
* ``match3tile.mcts.MCTS`` -- the search the device rollouts plug into -- run
  over oracle-backed states with oracle rollouts must return exactly the
  reference's (action, value, policies) for the same Python ``random`` seed,
  over two consecutive calls (root re-use).
"""
import random

import numpy as np
import pytest

from conftest import SHAPES
from match3tile.boardConfig import BoardConfig
from match3tile.mcts import MCTS
from oracle import Oracle


@pytest.mark.parametrize("tag", list(SHAPES))
def test_oracle_rollouts_match_reference(golden, tag):
    g = golden("mcts")
    o = Oracle(*SHAPES[tag])
    R, C, _ = SHAPES[tag]
    k = f"ro_{tag}_"
    res = o.rollouts(g[k + "board"].astype(np.int32).reshape(-1, R * C), g[k + "seed"], g[k + "n_actions"],
                     g[k + "rseed"], threads=4)
    assert (res["gain"] == g[k + "gain"]).all()
    assert (res["steps"] == g[k + "steps"]).all()
    assert (res["draws"] == g[k + "draws"]).all()
    assert (res["flags"] & 0x08 == 0).all()
    assert (g[k + "steps"] == 0).any() and (g[k + "steps"] >= 20).any()  # terminal and full-length cases


class OracleBoard:
    """Test-only State over the CPU oracle: the surface MCTS touches (mctslib/abc/mcts.py:8-30)."""

    def __init__(self, n_actions, cfg, oracle, array=None, reward=0):
        self.cfg, self.n_actions, self._o = cfg, n_actions, oracle
        self.array = oracle.init_board(cfg.seed)[0] if array is None else array
        self._reward = reward
        self._actions = []

    @property
    def legal_actions(self):
        if not self._actions:
            self._actions = self._o.legal_actions(self.array)
        return self._actions

    def apply_action(self, a):
        if self.is_terminal:
            return self
        nb, r, _, _ = self._o.apply_action(self.array, self.cfg.seed, a, self.n_actions)
        return OracleBoard(self.n_actions - 1, self.cfg, self._o, nb, self._reward + r)

    def clone(self):
        c = OracleBoard(self.n_actions, self.cfg, self._o, np.copy(self.array), self._reward)
        c._actions = self._actions
        return c

    @property
    def is_terminal(self):
        return self.n_actions < 1

    @property
    def reward(self):
        return self._reward


def oracle_rollouts(o):
    def run(states, seeds):
        res = o.rollouts(np.stack([s.array for s in states]), [s.cfg.seed for s in states],
                         [s.n_actions for s in states], seeds, threads=1)
        return np.array([s.reward for s in states]) + res["gain"]
    return run


def test_search_matches_reference(golden):
    g = golden("mcts")
    o = Oracle(9, 9, 6)
    for i in range(len(g["se_seed"])):
        seed, sims, pyseed, c = int(g["se_seed"][i]), int(g["se_sims"][i]), int(g["se_pyseed"][i]), float(g["se_c"][i])
        root = OracleBoard(20, BoardConfig(seed=seed), o)
        random.seed(pyseed)
        m = MCTS(root, c, sims, False, rollout_fn=oracle_rollouts(o))
        for call in range(2):
            a, v, p = m()
            n = int(g[f"se{call}_npol"][i])
            assert a == g[f"se{call}_action"][i], (i, call)
            assert v == g[f"se{call}_value"][i], (i, call)
            assert np.array_equal(np.array(p), g[f"se{call}_policies"][i][:n]), (i, call)


def test_leaf_rollouts_average(golden):
    """leaf_rollouts=k backs up the mean of k rollouts with k consecutive random seeds."""
    o = Oracle(9, 9, 6)
    root = OracleBoard(5, BoardConfig(seed=77), o)
    seen = []

    def fn(states, seeds):
        seen.append(list(seeds))
        return oracle_rollouts(o)(states, seeds)

    random.seed(5)
    m = MCTS(root, 1.0, 6, False, leaf_rollouts=4, rollout_fn=fn)
    m()
    random.seed(5)
    want = [random.randint(0, 2**31 - 1) for _ in range(24)]
    assert [s for batch in seen for s in batch] == want
    assert all(len(b) == 4 for b in seen)


def test_oracle_greedy_episodes_match_reference(golden):
    """samplerTasks.greedy_test (boardv2.py:209-218 every move) restated over the oracle."""
    g = golden("mcts")
    o = Oracle(9, 9, 6)
    for seed, acts, total in zip(g["gr_seed"], g["gr_actions"], g["gr_reward"]):
        board, _ = o.init_board(int(seed))
        reward, na = 0, 20
        for m in range(20):
            best, best_r, best_b = None, -1, None
            for a in o.legal_actions(board):
                nb, r, _, _ = o.apply_action(board, int(seed), a, na)
                if reward + r > best_r:
                    best, best_r, best_b = a, reward + r, nb
            assert best == acts[m]
            board, reward, na = best_b, best_r, na - 1
        assert reward == total
