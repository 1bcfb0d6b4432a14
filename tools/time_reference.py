#!/usr/bin/env python3
"""Time the reference's own Python step path on this container's host cores.

Runs the reference's samplerTasks.random_task loop (samplerTasks.py:9-14:
BoardV2(20, BoardConfig(seed)) then apply_action(np.random.choice(legal_actions))
until terminal) for seeded 9x9x6 boards, one process per core, and prints one
JSON line. Only for DESIGN.md's "reference Python path" row: the reference does
not exist on the GPU box, so bench.py's cpu_baseline times the C oracle instead.

    PYTHONPATH=/root/reference python3 -B tools/time_reference.py [--procs 8 --seconds 20]
"""
import argparse
import json
import multiprocessing as mp
import os
import time


def worker(args):
    first_seed, seconds = args
    import numpy as np
    from match3tile.boardConfig import BoardConfig
    from match3tile.boardv2 import BoardV2

    steps = episodes = 0
    seed = first_seed
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        state = BoardV2(20, BoardConfig(seed=seed))
        np.random.seed(state.cfg.seed)
        while not state.is_terminal:
            state = state.apply_action(np.random.choice(state.legal_actions))
            steps += 1
        episodes += 1
        seed += 1
    return steps, episodes, time.perf_counter() - t0


def rollout_worker(args):
    """mctslib MCTS.rollout (mctslib/standard/mcts.py:14-19) from fresh 20-move boards."""
    first_seed, seconds = args
    import random

    from match3tile.boardConfig import BoardConfig
    from match3tile.boardv2 import BoardV2
    from mctslib.standard.mcts import MCTS

    class _R:
        deterministic = False

    random.seed(first_seed)
    n = steps = 0
    seed = first_seed
    t0 = time.perf_counter()
    while time.perf_counter() - t0 < seconds:
        state = BoardV2(20, BoardConfig(seed=seed))
        MCTS.rollout(_R(), state)
        n += 1
        steps += 20
        seed += 1
    return n, steps, time.perf_counter() - t0


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--procs", type=int, default=os.cpu_count() or 1)
    ap.add_argument("--seconds", type=float, default=20.0)
    ap.add_argument("--rollouts", action="store_true", help="time MCTS.rollout instead of random_task")
    a = ap.parse_args()
    if a.rollouts:
        res = {}
        for procs in sorted({1, a.procs}):
            with mp.Pool(procs) as pool:
                out = pool.map(rollout_worker, [(1 + 1_000_000 * i, a.seconds) for i in range(procs)])
            wall = max(o[2] for o in out)
            res[procs] = {"rollouts_per_s": sum(o[0] for o in out) / wall,
                          "env_steps_per_s": sum(o[1] for o in out) / wall, "seconds": wall}
        print(json.dumps({"what": "reference mctslib MCTS.rollout from fresh 9x9x6 20-move boards",
                          "host": "build container", "cpus": os.cpu_count(), "by_processes": res}))
        return
    res = {}
    for procs in sorted({1, a.procs}):
        with mp.Pool(procs) as pool:
            out = pool.map(worker, [(1 + 1_000_000 * i, a.seconds) for i in range(procs)])
        steps = sum(o[0] for o in out)
        wall = max(o[2] for o in out)
        res[procs] = {"env_steps_per_s": steps / wall, "steps": steps, "episodes": sum(o[1] for o in out),
                      "seconds": wall}
    print(json.dumps({"what": "reference samplerTasks.random_task loop (BoardV2.apply_action), 9x9x6, 20 moves",
                      "host": "build container", "cpus": os.cpu_count(), "by_processes": res}))


if __name__ == "__main__":
    main()
