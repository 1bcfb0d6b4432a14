"""Self-play producer on the MI355X against the reference's mcts_task output.

``mcts_task`` (device MCTS, one rollout launch per simulation) and
``play_games`` (all games in lockstep, one launch per simulation round) must
both reproduce the reference's observations, policy vectors and values for the
same (cfg seed, Python random seed) -- tests/golden/gen_golden_dataset.py.
"""
import random

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.dataset import mcts_task, play_games  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def need_gpu():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


def _check(got, g, i):
    assert np.array_equal(np.array(got["observations"]), g[f"task{i}_obs"])
    assert np.array_equal(np.array(got["policies"]), g[f"task{i}_pol"])
    assert np.array_equal(np.array(got["values"]), g[f"task{i}_val"])


def test_mcts_task_matches_reference(golden):
    g = golden("dataset")
    moves = int(g["task_moves"])
    for i in range(len(g["task_seed"])):
        random.seed(int(g["task_pyseed"][i]))
        (got,) = mcts_task(((lambda: None, (BoardConfig(seed=int(g["task_seed"][i])), moves)), moves - 1))
        _check(got, g, i)


def test_lockstep_games_match_reference(golden):
    g = golden("dataset")
    moves = int(g["task_moves"])
    k = len(g["task_seed"])
    cfgs = [BoardConfig(seed=int(g["task_seed"][i])) for i in range(k)]
    got = play_games(cfgs, moves, [int(g["task_pyseed"][i]) for i in range(k)])
    for i in range(k):
        part = {key: v[i * moves:(i + 1) * moves] for key, v in got.items()}
        _check(part, g, i)
