"""Match3Env host logic without a GPU: spaces, and the env.npz fixture's own bookkeeping.

The GPU test (test_gpu_env.py) replays the fixture through the HIP kernels; here
the A.8 bookkeeping recorded in it is re-derived from its rewards alone (score,
truncation at env_goal, done at num_moves, reset seeds incl. the env.py:62
quirk), and the duck-typed spaces used when gymnasium is absent are checked.
"""
import numpy as np

from match3tile.env import Box, Discrete


def test_spaces_stand_ins():
    d = Discrete(144)
    assert d.n == 144 and d.contains(0) and d.contains(np.int64(143)) and not d.contains(144)
    np.random.seed(0)
    assert all(d.contains(d.sample()) for _ in range(100))
    b = Box(0, 32, (9, 9), np.int64)
    assert b.shape == (9, 9) and b.contains(np.full((9, 9), 32)) and not b.contains(np.full((9, 9), 33))
    assert not b.contains(np.zeros((9, 8)))
    assert b.sample().shape == (9, 9)


def test_env_fixture_bookkeeping(golden):
    g = golden("env")
    tags = sorted({k[len("moves_"):] for k in g.files if k.startswith("moves_")})
    for tag in tags:
        R, C, T = (int(x) for x in tag.split("x"))
        assert int(g["action_space_" + tag]) == R * (C - 1) + C * (R - 1)
        for i in range(len(g["seed_" + tag])):
            moves, goal = int(g["moves_" + tag][i]), int(g["goal_" + tag][i])
            seed, score, taken = int(g["seed_" + tag][i]), 0, 0
            for t in range(g["action_" + tag].shape[1]):
                score += int(g["reward_" + tag][i, t])
                taken += 1
                tr = score >= goal
                dn = tr or taken == moves
                assert bool(g["trunc_" + tag][i, t]) == tr and bool(g["done_" + tag][i, t]) == dn
                arg = int(g["reset_arg_" + tag][i, t])
                assert (arg != -2) == dn
                if dn:
                    seed = arg if arg >= 0 else (1 + seed) % 2**32 - 1
                    score, taken = 0, 0
                assert int(g["seed_after_" + tag][i, t]) == seed
