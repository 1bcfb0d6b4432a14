"""The device rule code (m3_rules.hpp), compiled for the HOST by a test-only harness
(tests/hostcore), differential-tested against the reference fixtures and the oracle.
This checks the bitboard logic without a GPU; the HIP path itself is covered by the
-m gpu tests."""
import os
import sys

import numpy as np
import pytest

from conftest import ROOT, SHAPES
from oracle import Oracle

sys.path.insert(0, os.path.join(ROOT, "tests", "hostcore"))
from hostcore import HostCore, lib  # noqa: E402


def test_chain_mt_matches_numpy_stream(golden):
    g = golden("prng")
    for s, r in zip(g["seeds"], g["raw"]):
        for k in (0, 1, 226, 227, 453, 454, 622, 623):
            assert lib().hc_chain_draw(int(s), k) == r[k]
        assert lib().hc_chain_draw(int(s), 624) == 0xFFFFFFFF  # beyond the first block: overflow


def test_chain2_equals_numpy_stream_over_two_blocks():
    """ChainMT2 (register-only, 16x16x8 resets) == numpy's MT19937 raw stream for draws 0..1247,
    including the level changes at 227 / 454 / 624 / 851 / 1078 and the mt''[623] wrap."""
    import ctypes

    o = Oracle()
    for s in (1, 2, 12345, 4242, 2**31 - 1, 2**32 - 1):
        want = o.mt_raw(s, 1248)
        got = np.zeros(1249, np.uint32)
        assert lib().hc_chain2_raw(ctypes.c_uint32(s), 1248, got.ctypes.data_as(ctypes.c_void_p)) == 0
        assert (got[:1248] == want).all(), (s, int(np.flatnonzero(got[:1248] != want)[0]))
        assert lib().hc_chain2_raw(ctypes.c_uint32(s), 1249, got.ctypes.data_as(ctypes.c_void_p)) == -1
