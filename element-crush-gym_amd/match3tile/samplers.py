"""Episode scorers of the reference's ``samplerTasks.py`` over the device step, and batched greedy.

``random_task`` / ``greedy_test`` / ``mcts_task`` restate samplerTasks.py:9-32
(the NN variant, :35-42, needs the JAX model and is out of scope). The
reference functions take no arguments and draw the board seed from numpy's
global RNG (``BoardConfig()``, boardConfig.py:34); here ``seed`` may be given
to make an episode reproducible, and ``None`` keeps the reference behaviour.

``greedy_actions(states)`` is ``[s.greedy_action for s in states]``
(boardv2.py:209-218) for many boards in ONE launch: every legal action of
every state is applied by one ``m3_apply_actions`` call and each state keeps
its first maximum, as the reference loop does.
"""
from __future__ import annotations

from typing import List, Sequence

import numpy as np

from . import _native
from .boardConfig import BoardConfig
from .boardv2 import BoardV2, _sync_global_rng
from .mcts import MCTS


def _start(seed, moves=20):
    state = BoardV2(moves, BoardConfig(seed=seed))
    np.random.seed(state.cfg.seed)                                # samplerTasks.py:11
    return state


def random_task(seed=None) -> int:
    """samplerTasks.py:9-14: seeded random actions until terminal; returns the episode reward."""
    state = _start(seed)
    while not state.is_terminal:
        state = state.apply_action(np.random.choice(state.legal_actions))
    return state.reward


def greedy_test(seed=None) -> int:
    """samplerTasks.py:17-22: the best one-step action every move."""
    state = _start(seed)
    while not state.is_terminal:
        state = state.apply_action(state.greedy_action)
    return state.reward


def mcts_task(seed=None, exploration_weight=2, simulations=100) -> int:
    """samplerTasks.py:25-32: MCTS(state, 2, 100) every move, device rollouts."""
    state = _start(seed)
    search = MCTS(state, exploration_weight, simulations, False, deterministic=False)
    while not state.is_terminal:
        action, _, _ = search()
        state = state.apply_action(action)
    return state.reward


def greedy_actions(states: Sequence[BoardV2], sync_rng: bool = False) -> List:
    """``greedy_action`` of every state (one board shape) with all candidates in one launch.

    sync_rng=True leaves numpy's global RNG as the LAST state's greedy_action would."""
    states = list(states)
    if not states:
        return []
    cfg = states[0].cfg
    shape = (cfg.rows, cfg.columns, cfg.types)
    if any((s.cfg.rows, s.cfg.columns, s.cfg.types) != shape for s in states):
        raise ValueError("greedy_actions() needs states of one board shape")
    legal = [s.legal_actions for s in states]
    counts = np.array([len(x) for x in legal])
    owner = np.repeat(np.arange(len(states)), counts)
    if len(owner) == 0:
        return [None] * len(states)
    acts = np.concatenate([np.asarray(x, dtype=np.int32) for x in legal if len(x)])
    boards = np.stack([np.asarray(states[i].array) for i in owner])
    seeds = np.array([int(states[i].cfg.seed) & 0xFFFFFFFF for i in owner], dtype=np.uint32)
    n_act = np.array([states[i].n_actions for i in owner], dtype=np.int32)
    res = _native.context(*shape).apply_actions(boards, seeds, n_act, acts)
    out, pos = [], 0
    for i, s in enumerate(states):
        k = int(counts[i])
        if k == 0:
            out.append(None)
            continue
        totals = s.reward + res["reward"][pos:pos + k].astype(np.int64)
        out.append(int(acts[pos + int(np.argmax(totals))]))   # argmax = first maximum, as the loop
        pos += k
    if sync_rng and counts[-1] and not states[-1].is_terminal:
        _sync_global_rng(states[-1].cfg.seed, int(res["draws"][-1]))
    return out
