import sys, os
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path[:0] = [ROOT + "/tests", ROOT + "/element-crush-gym_amd", ROOT + "/oracle"]
import numpy as np
from match3tile import _native
from oracle import Oracle
from test_gpu_mcts import start_states
tag = sys.argv[1] if len(sys.argv) > 1 else "16x16x8"
R, C, T = (int(x) for x in tag.split("x"))
o = Oracle(R, C, T)
c = _native.Context(R, C, T)
for n, fb in ((160, False), (768, False), (768, True), (64, True)):
    boards, seeds, na, rs = start_states(o, n, 1000 + 768)
    boards, seeds, na, rs = boards[:n], seeds[:n], na[:n], rs[:n]
    want = o.rollouts(boards, seeds, na, rs, threads=8)
    got = c.rollouts(boards.astype(np.int8), seeds, na, rs, final_boards=fb)
    bad = np.flatnonzero(got["gain"] != want["gain"])
    print(n, fb, "bad", len(bad), "got steps sum", got["steps"].sum(), "want", want["steps"].sum(),
          "got gain sum", got["gain"].sum(), "flags", np.unique(got["flags"]), np.unique(want["flags"]))
    for i in bad[:5]:
        print("  ", i, na[i], got["gain"][i], want["gain"][i], got["steps"][i], want["steps"][i], got["draws"][i], want["draws"][i], got["flags"][i], want["flags"][i])
