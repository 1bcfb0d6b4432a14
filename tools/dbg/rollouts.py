"""debug: frame rollouts vs oracle, mismatch detail and determinism"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from match3tile import _native
from oracle import Oracle
for (R, C, T) in [(10, 8, 5), (9, 9, 6), (16, 16, 8), (7, 7, 3)]:
    ctx = _native.Context(R, C, T)
    seeds = np.arange(1, 4097, dtype=np.uint32)
    boards, _, _ = ctx.init_boards(seeds)
    rs = (np.arange(4096, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    ro = ctx.rollouts(boards, seeds, 20, rs)
    ro2 = ctx.rollouts(boards, seeds, 20, rs)
    want = Oracle(R, C, T).rollouts(boards.astype(np.int32), seeds, 20, rs, threads=4)
    bad = np.flatnonzero((ro["gain"] != want["gain"]) | (ro["steps"] != want["steps"]) | (ro["draws"] != want["draws"]))
    det = np.flatnonzero((ro["gain"] != ro2["gain"]) | (ro["draws"] != ro2["draws"]))
    print((R, C, T), "mismatch", len(bad), "nondet", len(det), flush=True)
    for i in bad[:8]:
        print("  ", i, "gpu", ro["gain"][i], ro["steps"][i], ro["draws"][i], hex(ro["flags"][i]),
              "ref", want["gain"][i], want["steps"][i], want["draws"][i], "rerun", ro2["gain"][i], ro2["draws"][i])
    for i in bad[:3]:
        r1 = ctx.rollouts(boards[i:i + 1], seeds[i:i + 1], 20, rs[i:i + 1])
        print("   single", i, r1["gain"][0], r1["steps"][0], r1["draws"][0], hex(r1["flags"][0]))
    ctx.close()
