"""MCTS over the device step: drop-in for ``mctslib.standard.mcts.MCTS`` with batched rollouts.

The reference's MCTS (mctslib/abc/mcts.py:71-128, mctslib/standard/mcts.py)
spends nearly all of its time in ``rollout``: a Python loop of
``np.random.choice(legal_actions)`` + ``apply_action`` until the state is
terminal (mcts.py:14-19), ~20 steps of ~0.74 ms each on 9x9x6. Here a rollout
is one lane of ``k_rollout`` (libm3.so, ``m3_rollouts``): the whole random
playout runs on the GPU and returns the summed reward, and many rollouts share
one launch.

``MCTS`` keeps the reference's search exactly -- node bookkeeping, expansion
order (``untried_actions.pop()``), UCB1 with the node's ``n_actions`` as the
exploration weight during selection (mctslib/abc/mcts.py:96), the rollout
seed drawn from Python's ``random`` (mcts.py:15), root re-use between calls --
so with ``leaf_rollouts=1`` it returns the same (action, value, policies) as
the reference for the same Python ``random`` state. ``leaf_rollouts=k > 1``
is the batched extension: each simulation plays k rollouts from the leaf in
ONE launch (seeds k consecutive ``random.randint`` draws) and backs up their
mean.

``rollouts(states, rollout_seeds)`` is the raw batched call for any set of
BoardV2 states that share a board shape.
"""
from __future__ import annotations

import math
import random
from typing import Callable, Optional, Sequence

import numpy as np

from . import _native

SEED_BOUND = 2**31 - 1  # random.randint(0, 2 ** 31 - 1) (mcts.py:15)


def _sync_global_rng(seed: int, draws: int) -> None:
    np.random.seed(int(seed) & 0xFFFFFFFF)
    if draws:
        np.random.mtrand._rand._bit_generator.random_raw(int(draws))


def rollouts(states: Sequence, rollout_seeds) -> dict:
    """MCTS.rollout for every state in one launch (states: BoardV2 of one board shape).

    Returns ``returns`` (state.reward + the rollout's summed step rewards, what
    mcts.py:19 returns) and the raw per-rollout gain/steps/draws/flags. Raises
    ValueError where the reference raises (no legal action to sample)."""
    states = list(states)
    if not states:
        return dict(returns=np.zeros(0, np.int64), gain=np.zeros(0, np.int32), steps=np.zeros(0, np.int32),
                     draws=np.zeros(0, np.uint32), flags=np.zeros(0, np.uint32))
    cfg = states[0].cfg
    shape = (cfg.rows, cfg.columns, cfg.types)
    if any((s.cfg.rows, s.cfg.columns, s.cfg.types) != shape for s in states):
        raise ValueError("rollouts() needs states of one board shape")
    ctx = _native.context(*shape)
    boards = np.stack([np.asarray(s.array) for s in states])
    seeds = np.array([int(s.cfg.seed) & 0xFFFFFFFF for s in states], dtype=np.uint32)
    n_actions = np.array([s.n_actions for s in states], dtype=np.int32)
    res = ctx.rollouts(boards, seeds, n_actions, np.asarray(rollout_seeds, dtype=np.uint32))
    if (res["flags"] & _native.FLAG_NO_LEGAL).any():
        raise ValueError("a rollout reached a board with no legal action (np.random.choice of an empty list)")
    base = np.array([s.reward for s in states], dtype=np.int64)
    res["returns"] = base + res["gain"]
    return res


def device_rollout(state, rollout_seed: int) -> int:
    """MCTS.rollout(state) (mcts.py:14-19) with numpy's global RNG left where the reference leaves it."""
    res = rollouts([state], [rollout_seed])
    last_seed = state.cfg.seed if res["steps"][0] > 0 else rollout_seed
    _sync_global_rng(last_seed, int(res["draws"][0]))
    return int(res["returns"][0])


class Node:
    """Search-tree node (mctslib/abc/mcts.py:33-76 + standard/mcts.py:22-43)."""

    __slots__ = ("state", "parent", "children", "visits", "reward", "untried_actions")

    def __init__(self, state, parent: Optional["Node"] = None):
        self.state = state.clone()
        self.parent = parent
        self.children: dict = {}           # insertion order = expansion order (max() tie-breaks on it)
        self.visits = 0
        self.reward = 0
        self.untried_actions = list(state.legal_actions)

    @property
    def is_fully_expanded(self) -> bool:
        return not self.untried_actions

    def expand(self) -> "Node":
        action = self.untried_actions.pop()          # last untried action first
        child = Node(self.state.apply_action(action), self)
        self.children[action] = child
        return child

    def update(self, reward) -> None:
        self.visits += 1
        self.reward += reward

    def ucb1(self, c: float) -> float:
        if self.visits == 0:
            return float("inf")
        return self.reward / self.visits + c * math.sqrt(math.log(self.parent.visits) / (1 + self.visits))

    def best_child(self, c: float) -> "Node":
        best, best_v = None, None
        for ch in self.children.values():            # first maximum wins, as max()
            v = ch.ucb1(c)
            if best is None or v > best_v:
                best, best_v = ch, v
        return best

    @property
    def exploitation(self) -> float:
        return self.reward / self.visits

    @property
    def policies(self):
        return [ch.visits / self.visits for ch in self.children.values()]


class MCTS:
    """``mctslib.standard.mcts.MCTS(state, exploration_weight, simulations, verbose, deterministic)``.

    ``rollout_fn(states, seeds) -> returns`` replaces the device rollout (tests
    use the CPU oracle to check the search logic without a GPU)."""

    def __init__(self, state, exploration_weight: float, simulations: int, verbose: bool = False,
                 deterministic: bool = False, leaf_rollouts: int = 1,
                 rollout_fn: Optional[Callable] = None, rng=None):
        if leaf_rollouts < 1:
            raise ValueError("leaf_rollouts must be >= 1")
        self._root = Node(state)
        self._simulations = simulations
        self._verbose = verbose
        self._exploration_weight = exploration_weight  # kept for parity; selection uses n_actions (abc:96)
        self.deterministic = deterministic
        self.leaf_rollouts = leaf_rollouts
        self._rollout_fn = rollout_fn
        self._rng = random if rng is None else rng     # source of rollout seeds (mcts.py:15)
        self._root.expand()                            # abc/mcts.py:84

    def _seed(self, state) -> int:
        return state.seed if self.deterministic else self._rng.randint(0, SEED_BOUND)

    def rollout(self, state) -> float:
        """mcts.py:14-19 on the device; with leaf_rollouts > 1 the mean of that many."""
        seeds = [self._seed(state) for _ in range(self.leaf_rollouts)]
        if self._rollout_fn is not None:
            rets = np.asarray(self._rollout_fn([state] * len(seeds), seeds))
        elif len(seeds) == 1:
            return device_rollout(state, seeds[0])
        else:
            rets = rollouts([state] * len(seeds), seeds)["returns"]
        return int(rets[0]) if len(seeds) == 1 else float(rets.mean())

    # ---- one simulation, split so that many searches can share a launch ------
    def select_leaf(self) -> Node:
        """Selection + expansion (abc/mcts.py:94-101)."""
        node = self._root
        while not node.state.is_terminal and node.is_fully_expanded:
            node = node.best_child(node.state.n_actions)
        if not node.state.is_terminal and not node.is_fully_expanded:
            node = node.expand()
        return node

    @staticmethod
    def backpropagate(node: Node, reward) -> None:
        while node is not None:                        # abc/mcts.py:106-109
            node.update(reward)
            node = node.parent

    def finish(self):
        """Most-visited root child, root policies, greedy-line value; re-root (abc/mcts.py:115-128)."""
        root = self._root
        best_action, best = None, None
        for a, ch in root.children.items():
            if best is None or ch.visits > best.visits:
                best_action, best = a, ch
        policies = root.policies
        node = root
        while not node.state.is_terminal and node.is_fully_expanded:
            node = node.best_child(0)
        value = node.state.reward
        best.parent = None
        self._root = best
        return best_action, value, policies

    def __call__(self):
        pbar = None
        if self._verbose:
            from tqdm import tqdm

            pbar = tqdm(total=self._simulations)
        for _ in range(self._simulations):
            node = self.select_leaf()
            self.backpropagate(node, self.rollout(node.state))
            if pbar is not None:
                pbar.update(1)
        if pbar is not None:
            pbar.close()
        return self.finish()


def search_lockstep(searches: Sequence[MCTS]):
    """Run one ``__call__`` of every search with the simulations in lockstep.

    Simulation i of all searches shares ONE rollout launch (every search's
    leaf, in order); each search draws its rollout seed from its own ``rng``,
    so search g returns what ``searches[g]()`` alone would. All leaves must
    share a board shape. Returns [(action, value, policies)] per search."""
    searches = list(searches)
    if not searches:
        return []
    sims = searches[0]._simulations
    if any(m._simulations != sims for m in searches):
        raise ValueError("lockstep searches need the same number of simulations")
    for _ in range(sims):
        leaves, seeds, owner = [], [], []
        for gi, m in enumerate(searches):
            leaf = m.select_leaf()
            for _k in range(m.leaf_rollouts):
                leaves.append(leaf)
                seeds.append(m._seed(leaf.state))
                owner.append(gi)
            m._leaf = leaf
        if searches[0]._rollout_fn is not None:
            rets = np.asarray(searches[0]._rollout_fn([n.state for n in leaves], seeds))
        else:
            rets = rollouts([n.state for n in leaves], seeds)["returns"]
        pos = 0
        for m in searches:
            k = m.leaf_rollouts
            r = rets[pos:pos + k]
            pos += k
            m.backpropagate(m._leaf, int(r[0]) if k == 1 else float(np.mean(r)))
            m._leaf = None
    return [m.finish() for m in searches]
