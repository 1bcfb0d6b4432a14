"""Device rollouts (k_rollout via m3_rollouts) and the MCTS facade on the MI355X.

Bar: bit-exact gain / step count / global-stream draws / terminal boards
against the reference's rollouts (tests/golden/mcts.npz) and against the C
oracle on thousands of states (fresh boards, mid-episode boards with
specials, terminal states, 1-move states); the device-backed MCTS returns the
reference's (action, value, policies).
"""
import random

import numpy as np
import pytest

from conftest import SHAPES

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.boardv2 import BoardV2  # noqa: E402
from match3tile.mcts import MCTS, device_rollout, rollouts  # noqa: E402
from oracle import Oracle  # noqa: E402


@pytest.fixture(scope="module")
def ctxs():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return {tag: _native.Context(*shape) for tag, shape in SHAPES.items()}


@pytest.mark.parametrize("tag", list(SHAPES))
def test_rollouts_golden(golden, ctxs, tag):
    g = golden("mcts")
    k = f"ro_{tag}_"
    r = ctxs[tag].rollouts(g[k + "board"], g[k + "seed"], g[k + "n_actions"], g[k + "rseed"])
    assert (r["gain"] == g[k + "gain"]).all()
    assert (r["steps"] == g[k + "steps"]).all()
    assert (r["draws"] == g[k + "draws"]).all()
    assert (r["flags"] & _native.FLAG_NO_LEGAL == 0).all()


def start_states(o, n, seed0):
    """Fresh boards and boards after 1..12 seeded random moves (specials present)."""
    rng = np.random.default_rng(seed0)
    seeds = (np.arange(n, dtype=np.uint32) + np.uint32(seed0)).astype(np.uint32)
    depth = rng.integers(0, 13, n)
    ep = o.batch_episodes(seeds, num_moves=12, threads=8)
    boards = np.empty((n, o.R * o.C), np.int32)
    for i in range(n):
        if depth[i] == 0 or ep["moves"][i] == 0:
            boards[i] = o.init_board(int(seeds[i]))[0].ravel()
        else:
            boards[i] = ep["final"][i]
    n_actions = rng.choice([0, 1, 2, 7, 20, 20, 20, 25], n).astype(np.int32)
    rseeds = rng.integers(0, 2**31, n).astype(np.uint32)
    return boards, seeds, n_actions, rseeds


@pytest.mark.parametrize("tag,n", [("9x9x6", 8192), ("16x16x8", 768)])
def test_rollouts_vs_oracle(ctxs, tag, n):
    o = Oracle(*SHAPES[tag])
    boards, seeds, na, rs = start_states(o, n, 1000 + n)
    want = o.rollouts(boards, seeds, na, rs, threads=16)
    got = ctxs[tag].rollouts(boards.astype(np.int8), seeds, na, rs, final_boards=True)
    assert (got["gain"] == want["gain"]).all()
    assert (got["steps"] == want["steps"]).all()
    assert (got["draws"] == want["draws"]).all()
    assert (got["flags"] == want["flags"]).all()
    assert (got["final"].reshape(n, -1) == want["final"]).all()


def test_rollouts_ragged_and_empty(ctxs):
    o = Oracle(9, 9, 6)
    c = ctxs["9x9x6"]
    for n in (1, 63, 65, 130):
        boards, seeds, na, rs = start_states(o, n, 7 + n)
        want = o.rollouts(boards, seeds, na, rs, threads=4)
        got = c.rollouts(boards.astype(np.int8), seeds, na, rs)
        assert (got["gain"] == want["gain"]).all() and (got["draws"] == want["draws"]).all()
    empty = c.rollouts(np.zeros((0, 81), np.int8), [], [], [])
    assert len(empty["gain"]) == 0


def test_device_rollout_global_rng(golden):
    """device_rollout leaves numpy's global RNG where the reference's rollout leaves it."""
    g = golden("mcts")
    k = "ro_9x9x6_"
    for i in range(40):
        cfg = BoardConfig(seed=int(g[k + "seed"][i]))
        st = BoardV2(int(g[k + "n_actions"][i]), cfg, g[k + "board"][i].reshape(9, 9).astype(np.int64))
        ret = device_rollout(st, int(g[k + "rseed"][i]))
        assert ret == g[k + "gain"][i]
        last = cfg.seed if g[k + "steps"][i] > 0 else int(g[k + "rseed"][i])
        rs = np.random.RandomState(last)
        rs._bit_generator.random_raw(int(g[k + "draws"][i]))
        assert np.random.randint(0, 2**31 - 1) == rs.randint(0, 2**31 - 1)


def test_batched_rollouts_facade():
    states = [BoardV2(20, BoardConfig(seed=s)) for s in range(1, 33)]
    res = rollouts(states, list(range(100, 132)))
    o = Oracle(9, 9, 6)
    want = o.rollouts(np.stack([s.array for s in states]), [s.cfg.seed for s in states], 20, list(range(100, 132)))
    assert (res["returns"] == want["gain"]).all()


def test_search_matches_reference(golden):
    g = golden("mcts")
    for i in range(len(g["se_seed"])):
        root = BoardV2(20, BoardConfig(seed=int(g["se_seed"][i])))
        random.seed(int(g["se_pyseed"][i]))
        m = MCTS(root, float(g["se_c"][i]), int(g["se_sims"][i]), False)
        for call in range(2):
            a, v, p = m()
            n = int(g[f"se{call}_npol"][i])
            assert a == g[f"se{call}_action"][i]
            assert v == g[f"se{call}_value"][i]
            assert np.array_equal(np.array(p), g[f"se{call}_policies"][i][:n])


def test_rollouts_through_dead_boards_vs_oracle(ctxs):
    """Rollouts whose board goes dead mid-rollout (no legal move once settled, ~1e-5 of steps: the
    row shuffle, boardFunctions.py:16-23, inside the rollout loop): enough rollouts that dozens take
    that path; every one of them, and a random sample of the rest, equal the oracle's."""
    o = Oracle(9, 9, 6)
    c = ctxs["9x9x6"]
    n = 1 << 18
    seeds = (np.arange(n, dtype=np.uint64) * 7919 + 11).astype(np.uint32)
    boards, _, _ = c.init_boards(seeds)
    rs = (np.arange(n, dtype=np.uint64) * 104729 + 3).astype(np.uint32)
    got = c.rollouts(boards, seeds, 20, rs, final_boards=True)
    shuffled = np.flatnonzero(got["flags"] & _native.FLAG_SHUFFLED)
    assert len(shuffled) >= 5, len(shuffled)
    idx = np.union1d(shuffled, np.random.default_rng(3).choice(n, 1024, replace=False))
    want = o.rollouts(boards[idx].reshape(len(idx), -1).astype(np.int32), seeds[idx], 20, rs[idx], threads=16)
    for k in ("gain", "steps", "draws", "flags"):
        assert (got[k][idx] == want[k]).all(), k
    assert (got["final"][idx].reshape(len(idx), -1) == want["final"]).all()
