"""debug (round 5): characterise the frame-kernel lane interference on a given library (M3_LIB).

For each shape: 4096 seeded rollouts vs the oracle -> failing boards and their lane (index % 64);
then, for the first failing board, the board alone at several lane positions with the other lanes
idle (n_actions 0) or busy (other boards), and with its wave's real neighbours.
"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402
from oracle import Oracle  # noqa: E402

N = 4096
for shape in sys.argv[1:] or ["12x12x7", "10x8x5", "10x8x9"]:
    R, C, T = (int(x) for x in shape.split("x"))
    ctx = _native.Context(R, C, T)
    o = Oracle(R, C, T)
    seeds = np.arange(1, N + 1, dtype=np.uint32)
    boards, _, _ = ctx.init_boards(seeds)
    rs = (np.arange(N, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    na = np.full(N, 20, np.int32)
    g = ctx.rollouts(boards, seeds, na, rs)
    w = o.rollouts(boards.astype(np.int32), seeds, na, rs, threads=16)
    bad = np.nonzero((g["gain"] != w["gain"]) | (g["draws"] != w["draws"]) | (g["steps"] != w["steps"]))[0]
    print(shape, "failing", len(bad), "of", N, "lanes", sorted(set((bad % 64).tolist()))[:40], flush=True)
    print("   boards", bad[:24].tolist(), flush=True)
    if not len(bad):
        continue
    b = int(bad[0])
    ref = (int(w["gain"][b]), int(w["draws"][b]), int(w["steps"][b]))

    def run(idx, nav, label):
        idx = np.asarray(idx)
        gg = ctx.rollouts(boards[idx], seeds[idx], np.asarray(nav, np.int32), rs[idx])
        pos = [i for i, x in enumerate(idx) if x == b and nav[i] > 0]
        res = [(int(gg["gain"][i]), int(gg["draws"][i]), int(gg["steps"][i])) for i in pos]
        print(f"   {label:34s} board {b} at lanes {pos}: ok={[r == ref for r in res]}", flush=True)

    run([b], [20], "alone (lane 0)")
    wave = list(range(b - b % 64, b - b % 64 + 64))
    run(wave, [20] * 64, "its own wave")
    for L in (0, 1, 17, 40, 63):
        idx = [b if i == L else (b + 1 + i) % N for i in range(64)]
        run(idx, [20 if i == L else 0 for i in range(64)], f"lane {L}, others idle")
        run(idx, [20] * 64, f"lane {L}, others busy")
    run([b] * 64, [20] * 64, "64 copies")
