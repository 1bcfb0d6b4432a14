"""debug: locate the first diverging rollout step of a failing lane"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from match3tile import _native
from oracle import Oracle
R, C, T = 12, 12, 7
ctx = _native.Context(R, C, T)
o = Oracle(R, C, T)
seeds = np.arange(1, 4097, dtype=np.uint32)
boards, _, _ = ctx.init_boards(seeds)
rs = (np.arange(4096, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
def cmp(idx, na, label):
    idx = np.asarray(idx)
    nav = np.asarray(na, np.int32)
    g = ctx.rollouts(boards[idx], seeds[idx], nav, rs[idx], final_boards=True)
    w = o.rollouts(boards[idx].astype(np.int32), seeds[idx], nav, rs[idx], threads=1)
    ok = (g["gain"] == w["gain"]) & (g["draws"] == w["draws"])
    print(label, idx.tolist(), list(nav), "gpu", g["gain"].tolist(), g["draws"].tolist(), "ref", w["gain"].tolist(), w["draws"].tolist(), "ok", ok.tolist(), flush=True)
    return ok, g
cmp([2918, 2919], [20, 20], "pair")
cmp([2919, 2918], [20, 20], "swapped")
cmp([2919, 2919], [20, 20], "same")
cmp([2918, 2919], [0, 20], "lane0-idle")
cmp([2919], [20], "alone")
for k in range(1, 21):
    ok, g = cmp([2918, 2919], [20, k], f"k={k}")
    if not ok[1]:
        print("first bad step", k)
        break
cmp(list(range(2880, 2944)), [20] * 64, "wave45")
