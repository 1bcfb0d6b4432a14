"""debug (round 5): how many rollouts of a 4096-board batch are already wrong after k steps (all lanes
n_actions = k), on the library in M3_LIB; and the first-step inputs of a failing board through the
stateless k_apply kernel in the same company."""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402
from oracle import Oracle  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "10x8x9"
R, C, T = (int(x) for x in shape.split("x"))
N = 4096
ctx = _native.Context(R, C, T)
o = Oracle(R, C, T)
seeds = np.arange(1, N + 1, dtype=np.uint32)
boards, _, _ = ctx.init_boards(seeds)
rs = (np.arange(N, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
for k in (1, 2, 3, 5, 20):
    na = np.full(N, k, np.int32)
    g = ctx.rollouts(boards, seeds, na, rs, final_boards=True)
    w = o.rollouts(boards.astype(np.int32), seeds, na, rs, threads=16)
    fb = (g["final"].reshape(N, -1) != w["final"].reshape(N, -1)).any(1)
    bad = fb | (g["gain"] != w["gain"]) | (g["draws"] != w["draws"]) | (g["steps"] != w["steps"])
    print(f"k={k}: wrong {int(bad.sum())} (board {int(fb.sum())}, gain {int((g['gain'] != w['gain']).sum())}, "
          f"draws {int((g['draws'] != w['draws']).sum())}, steps {int((g['steps'] != w['steps']).sum())}, "
          f"flags {int((g['flags'] != w['flags']).sum())})", flush=True)
    if k == 1 and bad.any():
        # the first action of a rollout: choice(legal) on the rollout seed's stream; find which action the
        # GPU applied by trying every legal action through the oracle
        for b in np.nonzero(bad)[0][:5]:
            legal = o.legal_actions(boards[b])
            st = np.random.RandomState(int(rs[b]))
            want_a = int(legal[st.randint(0, len(legal))])
            got_a = [int(a) for a in legal
                     if (o.apply_action(boards[b], int(seeds[b]), int(a), 1)[0].reshape(-1) == g["final"][b].reshape(-1)).all()]
            print(f"   board {b}: oracle first action {want_a}, GPU board matches actions {got_a}; "
                  f"gain gpu {g['gain'][b]} ref {w['gain'][b]} draws gpu {g['draws'][b]} ref {w['draws'][b]}", flush=True)
