"""Host-side mirror of BoardConfig (match3tile/boardConfig.py) against the oracle and known constants."""
import numpy as np
import pytest

from conftest import SHAPES
from match3tile.boardConfig import BoardConfig
from oracle import Oracle


@pytest.mark.parametrize("tag", list(SHAPES))
def test_constants_and_codec(tag):
    R, C, T = SHAPES[tag]
    cfg = BoardConfig(seed=5, rows=R, columns=C, types=T)
    o = Oracle(R, C, T)
    oc = o.cfg
    assert (cfg.type_mask, cfg.special_type_mask, cfg.h_line, cfg.v_line, cfg.bomb, cfg.mega_token) == \
        (oc.TM, oc.STM, oc.H, oc.V, oc.B, oc.M)
    assert cfg.action_space == oc.A == R * (C - 1) * 2
    for a in range(cfg.action_space):
        assert cfg.actions[a] == o.decode(a)
        assert cfg.encode(*cfg.decode(a)) == a


def test_known_layouts():
    c = BoardConfig(seed=1)
    assert (c.type_mask, c.h_line, c.v_line, c.bomb, c.mega_token) == (7, 8, 16, 24, 32)
    c = BoardConfig(seed=1, rows=16, columns=16, types=8)
    assert (c.type_mask, c.h_line, c.v_line, c.bomb, c.mega_token) == (15, 16, 32, 48, 64)


def test_seed_zero_means_random_from_numpy_global():
    np.random.seed(123)
    expect = np.random.randint(0, 2 ** 31 - 1)
    np.random.seed(123)
    assert BoardConfig(seed=0).seed == expect


def test_encode_rejects_non_adjacent():
    with pytest.raises(AssertionError):
        BoardConfig(seed=1).encode((0, 0), (2, 0))
