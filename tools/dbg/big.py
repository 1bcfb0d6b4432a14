"""debug: 32x32x8 apply_actions mismatches vs fixture, split by draw count (chain reach 227)"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd"))
import numpy as np
from match3tile import _native
g = np.load(os.path.join(ROOT, "tests/golden/big.npz"))
for tag in ("32x32x8", "24x17x5", "20x20x6"):
    R, C, T = (int(x) for x in tag.split("x"))
    ctx = _native.Context(R, C, T)
    ok = g["step_draws_" + tag] != -2
    r = ctx.apply_actions(g["step_board_" + tag][ok], g["step_seed_" + tag][ok], g["step_n_actions_" + tag][ok],
                          g["step_action_" + tag][ok])
    good = (r["boards"] == g["step_next_" + tag][ok]).reshape(ok.sum(), -1).all(axis=1) & (r["reward"] == g["step_reward_" + tag][ok])
    d = g["step_draws_" + tag][ok]
    print(tag, "bad", (~good).sum(), "of", len(good), "| bad with draws>=227:", (~good & (d >= 227)).sum(),
          "draws>=227 total:", (d >= 227).sum(), "| bad draws sample", d[~good][:10].tolist(), flush=True)
    # one at a time: the first few bad ones alone
    for i in np.flatnonzero(~good)[:3]:
        idx = np.flatnonzero(ok)[i]
        r1 = ctx.apply_actions(g["step_board_" + tag][idx:idx + 1], g["step_seed_" + tag][idx:idx + 1],
                               g["step_n_actions_" + tag][idx:idx + 1], g["step_action_" + tag][idx:idx + 1])
        print("   alone", i, (r1["boards"][0] == g["step_next_" + tag][idx]).all(), r1["reward"][0], g["step_reward_" + tag][idx], r1["draws"][0], d[i], hex(r1["flags"][0]), flush=True)
    ctx.close()
