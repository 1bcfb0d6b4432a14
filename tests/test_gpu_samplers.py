"""samplerTasks drop-ins and batched greedy on the MI355X against the reference's episodes.

random_task (samplerTasks.py:9-14) vs the reference-generated seeded episodes
(episodes.npz); greedy_test (:17-22) vs reference greedy episodes (mcts.npz
gr_*); greedy_actions() over many states in one launch == per-state
greedy_action.
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.boardv2 import BoardV2  # noqa: E402
from match3tile.samplers import greedy_actions, greedy_test, random_task  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


def test_random_task_matches_reference(golden):
    g = golden("episodes")
    for i in range(24):
        assert random_task(int(g["seeds_9x9x6"][i])) == int(g["rewards_9x9x6"][i].sum())


def test_greedy_test_matches_reference(golden):
    g = golden("mcts")
    for seed, total in zip(g["gr_seed"][:12], g["gr_reward"][:12]):
        assert greedy_test(int(seed)) == int(total)


def test_batched_greedy_equals_per_state(golden):
    g = golden("mcts")
    states = []
    for seed, acts in zip(g["gr_seed"], g["gr_actions"]):
        s = BoardV2(20, BoardConfig(seed=int(seed)))
        for a in acts[: int(seed) % 7]:          # states at various depths
            s = s.apply_action(int(a))
        states.append(s)
    states.append(BoardV2(0, BoardConfig(seed=5)))  # terminal: the first legal action wins
    got = greedy_actions(states)
    want = [s.greedy_action for s in states]
    assert got == want
    # the batched result continues the reference's greedy episodes
    for seed, acts in zip(g["gr_seed"], g["gr_actions"]):
        d = int(seed) % 7
        assert got[int(seed) - 1] == acts[d]
