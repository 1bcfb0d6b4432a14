#!/usr/bin/env python3
"""Per-call latency of the batch-1 facade path (unchanged mctslib / samplerTasks callers).

    python3 tools/latency.py [--calls 300] [--out gpurun_out/latency.json]

The reference's MCTS expands and rolls out one node at a time
(mctslib/standard/mcts.py:14-19,31-42): every BoardV2.apply_action /
legal_actions is one call on one board. Times, on the MI355X box, the median
(and p10 / p90) wall time per call of:
  * BoardV2.apply_action through the facade (ctypes + m3_apply_actions + the
    numpy global-RNG replay), and the bare C-ABI call for one board;
  * BoardV2.legal_actions (uncached: a fresh board each call) and m3_legal_actions;
  * BoardV2(20, cfg) (reset, m3_init_boards);
  * MCTS.rollout of one state (m3_rollouts, 19 moves);
beside the reference's own per-call CPU times measured in the build container
(apply_action 0.74 ms, legal_actions 0.34 ms, __init__ 0.35 ms at 9x9x6).
"""
import argparse
import json
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd"))

import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402
from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.boardv2 import BoardV2  # noqa: E402

REFERENCE_MS = {"apply_action": 0.740, "legal_actions": 0.34, "init": 0.349}  # SURVEY.md §6, 9x9x6, 1 core


def timeit(fn, calls, warm=20):
    for _ in range(warm):
        fn()
    t = np.empty(calls)
    for i in range(calls):
        t0 = time.perf_counter()
        fn()
        t[i] = time.perf_counter() - t0
    return {"median_us": float(np.median(t) * 1e6), "p10_us": float(np.percentile(t, 10) * 1e6),
            "p90_us": float(np.percentile(t, 90) * 1e6), "calls": calls}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--calls", type=int, default=300)
    ap.add_argument("--out", default=None)
    a = ap.parse_args()
    cfg = BoardConfig(seed=12345)
    b0 = BoardV2(20, cfg)
    ctx = _native.context(9, 9, 6)
    seeds = np.array([cfg.seed], np.uint32)
    boards = b0.array.astype(np.int8)[None]
    legal = b0.legal_actions
    act = int(legal[0])
    res = {}
    res["facade_apply_action"] = timeit(lambda: b0.apply_action(act), a.calls)
    res["abi_apply_actions_n1"] = timeit(lambda: ctx.apply_actions(boards, seeds, 20, act), a.calls)
    fresh = [BoardV2(20, cfg, b0.array.copy()) for _ in range(a.calls + 20)]
    it = iter(fresh)
    res["facade_legal_actions_uncached"] = timeit(lambda: next(it).legal_actions, a.calls)
    res["abi_legal_actions_n1"] = timeit(lambda: ctx.legal_bits(boards), a.calls)
    res["facade_init"] = timeit(lambda: BoardV2(20, cfg), a.calls)
    res["abi_rollouts_n1"] = timeit(lambda: ctx.rollouts(boards, seeds, 19, np.array([7], np.uint32)), a.calls)
    out = {"what": "per-call wall time, batch 1, 9x9x6, MI355X (tools/latency.py)",
           "reference_python_ms": REFERENCE_MS, "results": res,
           "vs_reference": {"apply_action": REFERENCE_MS["apply_action"] * 1e3 / res["facade_apply_action"]["median_us"],
                            "legal_actions": REFERENCE_MS["legal_actions"] * 1e3
                            / res["facade_legal_actions_uncached"]["median_us"],
                            "init": REFERENCE_MS["init"] * 1e3 / res["facade_init"]["median_us"]}}
    s = json.dumps(out, indent=1)
    print(s)
    if a.out:
        with open(a.out, "w") as f:
            f.write(s)


if __name__ == "__main__":
    main()
