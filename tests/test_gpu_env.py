"""Match3Env driven exactly as the reference README.md:18-31 does.

    env = Match3Env(...)
    action = env.board.random_action()
    obs, reward, done, won, info = env.step(action)
    if done: obs, info = env.reset()

The reference Match3Env cannot run at its snapshot (env.py:38,64,50), so
tests/golden/env.npz holds runs of that loop with the Match3Env bookkeeping
 restated over the REAL reference BoardV2 / numpy global RNG
(tests/golden/gen_golden.py: gen_env). Every observation, reward, done and
truncated flag, every reset (seeded, and the reset() seed quirk of env.py:62)
and the spaces are compared bit for bit; the boards come from the HIP kernels.
"""
import os

import numpy as np
import pytest

from conftest import GOLDEN

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.env import Match3Env  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


def _fixture_tags(g):
    return sorted({k[len("moves_"):] for k in g.files if k.startswith("moves_")})


with np.load(os.path.join(GOLDEN, "env.npz")) as _g:
    ENV_TAGS = _fixture_tags(_g)  # 9x9x6, 16x16x8 and the frame shapes (8x8x5, 10x8x5, 5x3x3, ...)


def test_env_fixture_covers_both_headline_shapes(golden):
    tags = _fixture_tags(golden("env"))
    assert "9x9x6" in tags and "16x16x8" in tags


def test_env_fixture_covers_frame_shapes():
    assert {"8x8x5", "10x8x5", "5x3x3", "12x12x7"} <= set(ENV_TAGS)


@pytest.mark.parametrize("tag", ENV_TAGS)
def test_match3env_readme_loop_golden(golden, tag):
    g = golden("env")
    R, C, T = (int(x) for x in tag.split("x"))
    runs = len(g["seed_" + tag])
    n_steps = g["action_" + tag].shape[1]
    seen_trunc = seen_quirk = seen_seeded = 0
    for i in range(runs):
        env = Match3Env(width=C, height=R, num_types=T, num_moves=int(g["moves_" + tag][i]),
                        env_goal=int(g["goal_" + tag][i]), seed=int(g["seed_" + tag][i]))
        assert env.action_space.n == int(g["action_space_" + tag])  # env.py:36
        if R == C:
            assert env.action_space.n == R * (C - 1) * 2
        assert tuple(env.observation_space.shape) == (R, C)
        assert env.observation_space.low == 0 and env.observation_space.high == env.board.cfg.mega_token
        assert (env.init() == g["init_" + tag][i]).all() and env.init().dtype == np.int64
        for t in range(n_steps):
            action = env.board.random_action()                      # README.md:23
            assert action == g["action_" + tag][i, t], (i, t)
            obs, reward, done, won, info = env.step(action)          # README.md:24
            assert obs.dtype == np.int64 and obs.shape == (R, C)
            assert env.observation_space.contains(obs)
            assert (obs == g["obs_" + tag][i, t]).all(), (i, t)
            assert reward == g["reward_" + tag][i, t], (i, t)
            assert bool(done) == bool(g["done_" + tag][i, t]) and bool(won) == bool(g["trunc_" + tag][i, t])
            assert info == {}
            if done:
                arg = int(g["reset_arg_" + tag][i, t])
                obs, info = env.reset() if arg < 0 else env.reset(seed=arg)   # README.md:30
                assert (obs == g["reset_obs_" + tag][i, t]).all(), (i, t)
                assert env.score == 0 and env.moves_taken == 0
                seen_trunc += bool(won)
                seen_quirk += arg < 0
                seen_seeded += arg >= 0
            assert env.seed == g["seed_after_" + tag][i, t]
    assert seen_quirk and seen_seeded  # reset() and reset(seed) exercised
    if tag in ("9x9x6", "16x16x8"):
        assert seen_trunc  # env_goal truncation


def test_reset_without_seed_replays_the_episode():
    """env.py:62: (1 + seed) % 2**32 - 1 == seed, so reset() restarts the same board and stream."""
    env = Match3Env(seed=4242, num_moves=5)
    first = [env.step(env.board.random_action())[:2] for _ in range(5)]
    obs, _ = env.reset()
    assert env.seed == 4242
    again = [env.step(env.board.random_action())[:2] for _ in range(5)]
    for (o1, r1), (o2, r2) in zip(first, again):
        assert (o1 == o2).all() and r1 == r2


def test_reset_quirk_at_the_top_seed_raises_like_the_reference():
    """seed 2**32 - 1: reset() computes -1, and the reference's np.random.seed(-1) raises ValueError."""
    env = Match3Env(seed=2**32 - 1, num_moves=3)
    with pytest.raises(ValueError):
        env.reset()


def test_terminal_board_after_num_moves_is_a_no_op():
    """Stepping past num_moves without a reset: BoardV2 is terminal, apply_action returns it unchanged."""
    env = Match3Env(seed=99, num_moves=2, env_goal=10**9)
    for _ in range(2):
        env.step(env.board.random_action())
    before = env.board.array.copy()
    obs, r, done, tr, _ = env.step(0)
    assert (obs == before).all() and r == 0 and not done  # moves_taken 3 != num_moves 2
