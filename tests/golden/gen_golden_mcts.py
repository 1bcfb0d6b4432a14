#!/usr/bin/env python3
"""Golden vectors for the MCTS consumer of the step, from the REAL reference.

    PYTHONPATH=/root/reference python3 -B tests/golden/gen_golden_mcts.py

Runs in this container only (the reference never travels). Writes
``tests/golden/mcts.npz``:

  rollouts   ``MCTS.rollout(state)`` (mctslib/standard/mcts.py:14-19) on states
             reached by seeded random play, per shape: input board, cfg.seed,
             n_actions, the rollout seed the call drew from Python's ``random``
             (deterministic=False), and the outputs -- return,
             number of apply_action calls and the global numpy stream's draws
             since its last seed;
  searches   ``MCTS(state, c, simulations)()`` (mctslib/abc/mcts.py:71-128) on
             9x9x6 roots: Python ``random`` seed, simulations, the returned
             (action, value, policies) of two consecutive calls;
  greedy     ``samplerTasks.greedy_test`` episodes (greedy_action every move,
             boardv2.py:209-218) for board seeds 1..32: actions and reward.

Only data is committed -- no reference source.
"""
from __future__ import annotations

import os
import random
import signal
import sys
from multiprocessing import Pool

sys.dont_write_bytecode = True
REF = os.environ.get("M3_REFERENCE", "/root/reference")
if REF not in sys.path:
    sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.boardv2 import BoardV2  # noqa: E402
from mctslib.standard.mcts import MCTS  # noqa: E402

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
from gen_golden import draws_since_seed  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))


class _Rollout:
    deterministic = False


def _alarm(signum, frame):
    raise TimeoutError


def _rollout_case(args):
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(60)                          # a dead board whose shuffle cycles hangs the reference
    try:
        return _rollout_case_inner(args)
    except TimeoutError:
        return None
    finally:
        signal.alarm(0)


def _rollout_case_inner(args):
    R, C, T, seed, depth, n_actions, pyseed = args
    cfg = BoardConfig(seed=seed, rows=R, columns=C, types=T)
    state = BoardV2(n_actions, cfg)
    np.random.seed(seed)
    for _ in range(depth):                    # seeded random play to a mid-episode state
        if state.is_terminal or not state.legal_actions:
            break
        state = state.apply_action(int(np.random.choice(state.legal_actions)))
    random.seed(pyseed)
    rseed = random.randint(0, 2**31 - 1)      # what mcts.py:15 will draw
    random.seed(pyseed)
    ret = MCTS.rollout(_Rollout(), state)
    steps = state.n_actions if state.n_actions > 0 else 0
    last_seed = seed if steps > 0 else rseed
    return (state.array.astype(np.int8).ravel(), seed, state.n_actions, rseed, int(ret) - int(state.reward),
            steps, draws_since_seed(last_seed))


def gen_rollouts(pool):
    out = {}
    for (R, C, T), n in (((9, 9, 6), 1200), ((16, 16, 8), 160)):
        rng = np.random.default_rng(R * 1000 + T)
        cases = []
        for i in range(n):
            seed = int(rng.integers(1, 2**31 - 1))
            n_act = int(rng.choice([20, 20, 20, 5, 1, 0, 30]))
            depth = int(rng.integers(0, max(1, n_act)))
            cases.append((R, C, T, seed, depth, n_act, int(rng.integers(0, 2**31))))
        res = [r for r in pool.map(_rollout_case, cases, chunksize=8) if r is not None]
        tag = f"{R}x{C}x{T}"
        out[f"ro_{tag}_board"] = np.stack([r[0] for r in res])
        for k, j in (("seed", 1), ("n_actions", 2), ("rseed", 3), ("gain", 4), ("steps", 5), ("draws", 6)):
            out[f"ro_{tag}_{k}"] = np.array([r[j] for r in res], dtype=np.int64)
    return out


def _search_case(args):
    seed, sims, pyseed, c = args
    cfg = BoardConfig(seed=seed)
    root = BoardV2(20, cfg)
    random.seed(pyseed)
    np.random.seed(seed)
    m = MCTS(root, c, sims, False)
    res = []
    for _ in range(2):                         # a second call continues from the kept subtree
        a, v, p = m()
        res.append((int(a), float(v), np.array(p, dtype=np.float64)))
    return res


def gen_searches(pool):
    cases = [(s, sims, 1000 + s, c) for s, sims, c in ((3, 24, 1.4), (11, 40, 1.0), (29, 60, 2.0), (101, 33, 0.5))]
    res = pool.map(_search_case, cases)
    out = {"se_seed": np.array([c[0] for c in cases]), "se_sims": np.array([c[1] for c in cases]),
           "se_pyseed": np.array([c[2] for c in cases]), "se_c": np.array([c[3] for c in cases])}
    for call in range(2):
        out[f"se{call}_action"] = np.array([r[call][0] for r in res])
        out[f"se{call}_value"] = np.array([r[call][1] for r in res])
        pol = [r[call][2] for r in res]
        width = max(len(p) for p in pol)
        out[f"se{call}_npol"] = np.array([len(p) for p in pol])
        out[f"se{call}_policies"] = np.stack([np.pad(p, (0, width - len(p)), constant_values=-1) for p in pol])
    return out


def _greedy_case(seed):
    """samplerTasks.greedy_test (samplerTasks.py:17-22) with a fixed board seed."""
    state = BoardV2(20, BoardConfig(seed=seed))
    np.random.seed(state.cfg.seed)
    acts = []
    while not state.is_terminal:
        a = state.greedy_action
        acts.append(int(a))
        state = state.apply_action(a)
    return acts, int(state.reward)


def gen_greedy(pool):
    seeds = list(range(1, 33))
    res = pool.map(_greedy_case, seeds)
    return {"gr_seed": np.array(seeds), "gr_actions": np.array([r[0] for r in res], dtype=np.int32),
            "gr_reward": np.array([r[1] for r in res], dtype=np.int64)}


def main():
    with Pool(8) as pool:
        out = gen_rollouts(pool)
        out.update(gen_searches(pool))
        out.update(gen_greedy(pool))
    np.savez_compressed(os.path.join(OUT, "mcts.npz"), **out)
    print({k: v.shape for k, v in out.items()})


if __name__ == "__main__":
    main()
