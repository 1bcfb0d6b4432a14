"""The CPU oracle (oracle/m3_oracle.c) against the reference's own outputs.

Every fixture in tests/golden was produced by running the real reference
(tests/golden/gen_golden.py). These tests pin the oracle; the oracle then pins
the HIP path at sizes the fixtures cannot reach.
"""
import numpy as np
import pytest

from conftest import SHAPES
from oracle import FLAG_SHUFFLE_CAP, FLAG_SHUFFLED, Oracle


def test_prng_raw_streams(golden):
    g = golden("prng")
    o = Oracle()
    for s, r in zip(g["seeds"], g["raw"]):
        assert (o.mt_raw(int(s), len(r)) == r).all(), int(s)


@pytest.mark.parametrize("tag", list(SHAPES))
def test_get_matches_and_spawn(golden, tag):
    g = golden("matches")
    o = Oracle(*SHAPES[tag])
    for tb, mk, sp, ng in zip(g["tb_" + tag], g["mask_" + tag], g["spawn_" + tag], g["ngroups_" + tag]):
        mask, spawn, n = o.get_matches(tb.astype(np.int32))
        assert (mask == mk.astype(bool)).all()
        assert (spawn == sp).all()
        assert n == ng


@pytest.mark.parametrize("tag", list(SHAPES))
def test_legal_actions(golden, tag):
    g = golden("legal")
    o = Oracle(*SHAPES[tag])
    for b, lb in zip(g["boards_" + tag], g["legal_" + tag]):
        bits = np.zeros(o.A, np.uint8)
        bits[o.legal_actions(b.astype(np.int32))] = 1
        assert (bits == lb).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_init_boards(golden, tag):
    g = golden("init")
    o = Oracle(*SHAPES[tag])
    for s, b, d in zip(g["seeds_" + tag], g["boards_" + tag], g["draws_" + tag]):
        bb, dd = o.init_board(int(s))
        assert (bb == b).all() and dd == d, int(s)


@pytest.mark.parametrize("tag", list(SHAPES))
def test_step_transitions(golden, tag):
    g = golden("steps")
    o = Oracle(*SHAPES[tag])
    cols = [g[k + "_" + tag] for k in ("board", "seed", "n_actions", "action", "next", "reward", "draws")]
    for b, s, na, a, nx, r, d in zip(*cols):
        nb, rr, dd, f = o.apply_action(b.astype(np.int32), int(s), int(a), int(na))
        assert (nb == nx).all() and rr == r
        if d >= 0:
            assert dd == d


@pytest.mark.parametrize("tag", list(SHAPES))
def test_seeded_episodes(golden, tag):
    g = golden("episodes")
    o = Oracle(*SHAPES[tag])
    for i, s in enumerate(g["seeds_" + tag]):
        e = o.random_episode(int(s))
        assert (e["actions"] == g["actions_" + tag][i]).all()
        assert (e["rewards"] == g["rewards_" + tag][i]).all()
        assert (e["draws"] == g["draws_" + tag][i]).all()
        assert (e["final"] == g["final_" + tag][i]).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_shuffle_path(golden, tag):
    g = golden("shuffle")
    o = Oracle(*SHAPES[tag])
    n_shuffled = 0
    for b, s, a, nx, r, d, t in zip(*[g[k + "_" + tag] for k in
                                       ("board", "seed", "action", "next", "reward", "draws", "terminates")]):
        nb, rr, dd, f = o.apply_action(b.astype(np.int32), int(s), int(a), 20)
        if t:
            assert (nb == nx).all() and rr == r and dd == d and not (f & FLAG_SHUFFLE_CAP)
        else:
            assert f & FLAG_SHUFFLE_CAP
        n_shuffled += bool(f & FLAG_SHUFFLED)
    assert n_shuffled > 100


@pytest.mark.parametrize("fixture", ["shapes", "types2", "big"])
def test_other_board_configs(golden, fixture):
    """Every other BoardConfig the fixtures hold (shapes.npz: square, rows > columns, 3 and 15
    types; types2.npz: two tile types; big.npz: sides 17..32 and types 20 / 31), through the
    oracle: resets, legal sets, transitions and seeded episodes."""
    g = golden(fixture)
    tags = sorted({k[len("init_seeds_"):] for k in g.files if k.startswith("init_seeds_")})
    assert tags
    for tag in tags:
        o = Oracle(*(int(x) for x in tag.split("x")))
        for s, b, d in zip(g["init_seeds_" + tag][::4], g["init_boards_" + tag][::4], g["init_draws_" + tag][::4]):
            bb, dd = o.init_board(int(s))
            assert (bb == b).all() and dd == d, (tag, int(s))
        for b, lb in zip(g["legal_boards_" + tag], g["legal_" + tag]):
            bits = np.zeros(o.A, np.uint8)
            bits[o.legal_actions(b.astype(np.int32))] = 1
            assert (bits == lb).all(), tag
        if "step_board_" + tag not in g.files:
            continue
        cols = [g["step_" + k + "_" + tag] for k in ("board", "seed", "n_actions", "action", "next", "reward", "draws")]
        for b, s, na, a, nx, r, d in zip(*cols):
            if d == -2:  # the reference hangs (cycling shuffle)
                continue
            nb, rr, dd, f = o.apply_action(b.astype(np.int32), int(s), int(a), int(na))
            assert (nb == nx).all() and rr == r, tag
            if d >= 0:
                assert dd == d, tag
        for i, s in enumerate(g["ep_seeds_" + tag][:16]):
            e = o.random_episode(int(s))
            assert (e["actions"] == g["ep_actions_" + tag][i]).all(), tag
            assert (e["rewards"] == g["ep_rewards_" + tag][i]).all(), tag
            assert (e["final"] == g["ep_final_" + tag][i]).all(), tag
