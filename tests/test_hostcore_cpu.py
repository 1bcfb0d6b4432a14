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


@pytest.mark.parametrize("shape", [(9, 9, 6), (16, 16, 8), (7, 7, 3), (9, 9, 2), (12, 5, 4)],
                         ids=lambda s: "x".join(map(str, s)))
def test_fast_match_mask_equals_scan(shape):
    """BoardV2.__init__'s match mask (boardv2.py:23-27) by the union-of-runs fast path equals the
    sequential get_matches scan on dense random boards (few types: many L / T / crossing runs,
    so the dropped-arm fallback is exercised too), the mask of the reset and its fixtures."""
    R, C, T = shape
    hc = HostCore(R, C, T)
    rng = np.random.default_rng(7)
    b = rng.integers(1, T + 1, size=(20000, R * C)).astype(np.int8)
    assert hc.mask_mismatches(b) == 0


@pytest.mark.parametrize("shape", [(9, 9, 6), (16, 16, 8), (10, 8, 5), (12, 12, 7), (7, 7, 3), (9, 9, 20)],
                         ids=lambda s: "x".join(map(str, s)))
def test_fast_matches_equal_scan(shape):
    """get_matches' loop-free path (M3_FAST_MATCH, m3_rules.hpp) equals the sequential scan of
    boardFunctions.py:121-169 -- mask, spawn values and result -- on 100,000+ boards per shape:
    uniform random boards with specials, typed values and holes (many crossing runs: the scan
    path), boards with few repeats (the loop-free path), and boards with planted straight runs of
    3..7 both ways (spawn centres, runs of 6+ back on the scan)."""
    R, C, T = shape
    hc = HostCore(R, C, T)
    rng = np.random.default_rng(R * 100 + C + T)
    N = R * C
    n = 40000
    dense = rng.integers(1, T + 1, size=(n, N))
    sparse = rng.integers(1, T + 1, size=(n, N))
    sparse[:, 1::2] = rng.integers(1, T + 1, size=(n, (N + 0) // 2))  # (a second draw: fewer runs per board)
    planted = rng.integers(1, T + 1, size=(n, N))
    for i in range(n):
        for _ in range(2):
            L = int(rng.integers(3, min(8, C) + 1))
            if rng.random() < 0.5:
                r, c = int(rng.integers(0, R)), int(rng.integers(0, C - min(L, C) + 1))
                planted[i, r * C + c:r * C + c + min(L, C)] = planted[i, r * C + c]
            else:
                L = min(L, R)
                r, c = int(rng.integers(0, R - L + 1)), int(rng.integers(0, C))
                planted[i, (r + np.arange(L)) * C + c] = planted[i, r * C + c]
    boards = np.concatenate([dense, sparse, planted]).astype(np.int8)
    sp = rng.random(boards.shape)
    TM = (1 << max(1, int(T).bit_length())) - 1
    boards[sp < 0.03] = 0
    boards[(sp >= 0.03) & (sp < 0.05)] = TM + 1 + 2
    bad, fast = hc.fast_match_mismatches(boards)
    assert bad == 0
    assert fast > len(boards) // 10, fast  # the loop-free path is exercised


@pytest.mark.parametrize("tag", list(SHAPES))
def test_roundtrip_planes(tag):
    hc = HostCore(*SHAPES[tag])
    b = np.random.default_rng(1).integers(0, 128, size=(500, hc.N)).astype(np.int8)
    assert (hc.roundtrip(b) == b).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_matches_legal_init_steps_golden(golden, tag):
    hc = HostCore(*SHAPES[tag])
    m = golden("matches")
    mask, sp, fd = hc.matches(m["tb_" + tag])
    assert (mask == m["mask_" + tag].reshape(len(mask), -1)).all()
    assert (sp == m["spawn_" + tag].reshape(len(sp), -1)).all()
    assert ((fd > 0) == (m["ngroups_" + tag] > 0)).all()
    lg = golden("legal")
    bits = np.unpackbits(hc.legal(lg["boards_" + tag]).view(np.uint8), axis=1, bitorder="little")
    assert (bits[:, :lg["legal_" + tag].shape[1]] == lg["legal_" + tag]).all()
    ini = golden("init")
    out, drw, _, _ = hc.init(ini["seeds_" + tag])
    assert (out == ini["boards_" + tag].reshape(len(out), -1)).all() and (drw == ini["draws_" + tag]).all()
    st = golden("steps")
    out, rew, drw, flg, _, _ = hc.apply(st["board_" + tag], st["seed_" + tag], st["n_actions_" + tag],
                                        st["action_" + tag])
    assert (out == st["next_" + tag].reshape(len(out), -1)).all()
    assert (rew == st["reward_" + tag]).all()
    live = st["draws_" + tag] >= 0
    assert (drw[live] == st["draws_" + tag][live]).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_episodes_golden(golden, tag):
    hc = HostCore(*SHAPES[tag])
    e = golden("episodes")
    seeds = e["seeds_" + tag].astype(np.uint32)
    b, _, _, act = hc.init(seeds)
    for m in range(20):
        assert (act == e["actions_" + tag][:, m]).all()
        b, rew, drw, _, _, act = hc.apply(b, seeds, 20 - m, act)
        assert (rew == e["rewards_" + tag][:, m]).all()
        assert (drw == e["draws_" + tag][:, m]).all()
    assert (b == e["final_" + tag].reshape(len(b), -1)).all()


def test_random_states_vs_oracle():
    """Boards with random specials/typed values and random (incl. illegal) actions."""
    rng = np.random.default_rng(11)
    hc, o = HostCore(), Oracle()
    n = 3000
    seeds = rng.integers(1, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    boards, _, _, _ = hc.init(seeds)
    sprinkle = rng.random((n, 81)) < 0.06
    vals = rng.choice([8, 16, 24, 32, 11, 19, 27, 40, 56, 0, 127], size=(n, 81))
    boards = np.where(sprinkle, vals, boards).astype(np.int8)
    acts = rng.integers(0, 144, size=n)
    out, rew, drw, flg, legal, nxt = hc.apply(boards, seeds, 20, acts)
    for i in range(n):
        ob, orr, od, of = o.apply_action(boards[i].astype(np.int32), int(seeds[i]), int(acts[i]))
        assert (ob.reshape(-1) == out[i]).all() and orr == rew[i] and od == drw[i], i
        bits = np.zeros(144, np.uint8)
        bits[o.legal_actions(ob)] = 1
        assert (np.unpackbits(legal[i].view(np.uint8), bitorder="little")[:144] == bits).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_group_overflow_fallback_is_exact(golden, tag):
    """A 1-group table overflows on every multi-group match; the recompute must give identical results."""
    hc = HostCore(*SHAPES[tag])
    st = golden("steps")
    args = (st["board_" + tag], st["seed_" + tag], st["n_actions_" + tag], st["action_" + tag])
    a = hc.apply(*args)
    b = hc.apply(*args, small=True)
    assert hc.recomputed > 10
    for x, y in zip(a, b):
        assert (x == y).all()


def test_chain_init_fallback_counts(golden):
    """Reset runs on the register-only MT19937 chain; seeds needing >= 624 draws are recomputed exactly."""
    for tag in SHAPES:
        hc = HostCore(*SHAPES[tag])
        ini = golden("init")
        out, drw, _, _ = hc.init(ini["seeds_" + tag])
        assert (out == ini["boards_" + tag].reshape(len(out), -1)).all() and (drw == ini["draws_" + tag]).all()
        assert hc.recomputed == int((ini["draws_" + tag] > 623).sum())


def _check_steps(hc, g, tag, small):
    ok = g["terminates_" + tag] if "terminates_" + tag in g else np.ones(len(g["seed_" + tag]), bool)
    na = g["n_actions_" + tag] if "n_actions_" + tag in g else 20
    out, rew, drw, flg, _, _ = hc.apply(g["board_" + tag], g["seed_" + tag], na, g["action_" + tag], small=small)
    ok = ok.astype(bool)
    assert (out[ok] == g["next_" + tag].reshape(len(out), -1)[ok]).all()
    assert (rew[ok] == g["reward_" + tag][ok]).all()
    live = ok & (g["draws_" + tag] >= 0)
    assert (drw[live] == g["draws_" + tag][live]).all()


def test_one_level_chain_fallback_is_exact(golden):
    """The 16x16 env step runs the one-level MT chain (draws < 227): steps past it -- near-full-board
    refills such as mega+mega (256 cells) -- must be redone exactly (rare-branch test, forced by the
    golden combo cases)."""
    hc = HostCore(16, 16, 8)
    st = golden("steps")
    args = (st["board_16x16x8"], st["seed_16x16x8"], st["n_actions_16x16x8"], st["action_16x16x8"])
    a = hc.apply(*args)
    b = hc.apply(*args, small=32)
    assert hc.recomputed > 0
    for x, y in zip(a, b):
        assert (x == y).all()
    _check_steps(hc, st, "16x16x8", 32)


@pytest.mark.parametrize("tag", list(SHAPES))
@pytest.mark.parametrize("pause", [0, 1, 2, 3])
def test_paused_cascade_resumes_exactly(golden, tag, pause):
    """The env kernel's bounded cascade: a step paused before inner iteration pause + 1, its state
    serialized through Cont (the continuation record) and resumed from the words, must give the
    uninterrupted step's board, reward, draws, flags, legal set and next action -- on every step,
    shuffle and combo fixture and on random boards with specials."""
    import ctypes

    R, C, T = SHAPES[tag]
    hc = HostCore(R, C, T)
    cases = []
    for g in (golden("steps"), golden("shuffle")):
        na = g["n_actions_" + tag] if "n_actions_" + tag in g else np.full(len(g["seed_" + tag]), 20)
        ok = g["terminates_" + tag].astype(bool) if "terminates_" + tag in g else np.ones(len(na), bool)
        cases.append((g["board_" + tag][ok], g["seed_" + tag][ok], na[ok], g["action_" + tag][ok]))
    rng = np.random.default_rng(17 + pause)
    n = 1500 if R == 9 else 300
    seeds = rng.integers(1, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    boards, _, _, _ = hc.init(seeds)
    vals = {"9x9x6": (8, 16, 24, 32, 11, 19, 27, 0), "16x16x8": (16, 32, 48, 64, 19, 35, 0)}[tag]
    boards = np.where(rng.random((n, R * C)) < 0.05, rng.choice(vals, size=(n, R * C)), boards).astype(np.int8)
    cases.append((boards, seeds, np.full(n, 20), rng.integers(0, R * (C - 1) * 2, size=n)))
    lib().hc_paused.restype = ctypes.c_long
    lib().hc_paused(1)
    for b, s, na, a in cases:
        want = hc.apply(b, s, na, a)
        got = hc.apply(b, s, na, a, small=100 + pause)
        for x, y in zip(want, got):
            assert (x == y).all()
    assert lib().hc_paused(1) > (200 if pause < 2 else 20)  # the pause path really ran


# ---- the 16 x 16 frame (FCfg): every BoardConfig other than the two specialised shapes ----------
FRAME_SHAPES = [(3, 3, 3), (5, 3, 3), (7, 7, 4), (8, 8, 5), (10, 8, 5), (12, 12, 7), (16, 3, 4), (16, 15, 15),
                (6, 5, 9), (9, 9, 5), (4, 4, 3), (11, 7, 6)]


@pytest.mark.parametrize("tag", list(SHAPES))
def test_frame_form_on_headline_fixtures(golden, tag):
    """The frame form of the rule code (walls around the board, run-time shape) reproduces every
    9x9x6 / 16x16x8 reference fixture, like the specialised form."""
    hc = HostCore(*SHAPES[tag], frame=True)
    b = np.random.default_rng(1).integers(0, 128, size=(200, hc.N)).astype(np.int8)
    assert (hc.roundtrip(b) == b).all()
    m = golden("matches")
    mask, sp, fd = hc.matches(m["tb_" + tag])
    assert (mask == m["mask_" + tag].reshape(len(mask), -1)).all()
    assert (sp == m["spawn_" + tag].reshape(len(sp), -1)).all()
    lg = golden("legal")
    bits = np.unpackbits(hc.legal(lg["boards_" + tag]).view(np.uint8), axis=1, bitorder="little")
    assert (bits[:, :lg["legal_" + tag].shape[1]] == lg["legal_" + tag]).all()
    ini = golden("init")
    out, drw, _, _ = hc.init(ini["seeds_" + tag])
    assert (out == ini["boards_" + tag].reshape(len(out), -1)).all() and (drw == ini["draws_" + tag]).all()
    _check_steps(hc, golden("steps"), tag, 32)
    _check_steps(hc, golden("shuffle"), tag, 32)
    e = golden("episodes")
    seeds = e["seeds_" + tag].astype(np.uint32)
    b, _, _, act = hc.init(seeds)
    for mv in range(20):
        assert (act == e["actions_" + tag][:, mv]).all()
        b, rew, drw, _, _, act = hc.apply(b, seeds, 20 - mv, act, small=32)
        assert (rew == e["rewards_" + tag][:, mv]).all() and (drw == e["draws_" + tag][:, mv]).all()
    assert (b == e["final_" + tag].reshape(len(b), -1)).all()


@pytest.mark.parametrize("shape", FRAME_SHAPES, ids=lambda s: "x".join(map(str, s)))
def test_frame_random_states_vs_oracle(shape):
    """Frame form vs the C oracle on seeded boards with specials / typed values / holes, random
    (incl. illegal) actions, the env kernels' fast tables (one-level MT chain, 4-group table) with the
    exact recompute behind them, and 20-move seeded episodes. Includes columns = 3 (the decode quirk
    of boardConfig.py:50) and rows > columns (ids ending inside the last row)."""
    R, C, T = shape
    rng = np.random.default_rng(R * 1000 + C * 10 + T)
    hc, o = HostCore(R, C, T), Oracle(R, C, T, episode_shuffle_cap=1024)
    assert hc.frame
    n = 200
    seeds = rng.integers(1, 2**32, size=n, dtype=np.uint64).astype(np.uint32)
    boards, draws, _, first = hc.init(seeds)
    for i in range(0, n, 9):
        ob, od = o.init_board(int(seeds[i]))
        assert (ob.reshape(-1) == boards[i]).all() and od == draws[i]
    cf = o.cfg
    vals = [cf.H, cf.V, cf.B, cf.M, 0, cf.H + 1, min(127, cf.M + 3)]
    boards = np.where(rng.random((n, R * C)) < 0.07, rng.choice(vals, size=(n, R * C)), boards).astype(np.int8)
    A = R * (C - 1) * 2
    acts = rng.integers(0, A, size=n)
    out, rew, drw, flg, legal, nxt = hc.apply(boards, seeds, 20, acts, small=32)
    for i in range(n):
        ob, orr, od, of = o.apply_action(boards[i].astype(np.int32), int(seeds[i]), int(acts[i]))
        assert (ob.reshape(-1) == out[i]).all() and orr == rew[i] and od == drw[i] and (of & 0x1F) == (flg[i] & 0x1F), i
        bits = np.zeros(A, np.uint8)
        bits[o.legal_actions(ob)] = 1
        assert (np.unpackbits(legal[i].view(np.uint8), bitorder="little")[:A] == bits).all(), i
    e = o.batch_episodes(seeds[:64], 20, 2**31 - 1, threads=2)
    b, _, _, act = hc.init(seeds[:64])
    for mv in range(20):
        live = e["moves"] > mv
        assert (act[live] == e["actions"][live, mv]).all()
        b, rw, dr, _, _, act = hc.apply(b, seeds[:64], 20 - mv, act, small=32)
        assert (rw[live] == e["rewards"][live, mv]).all() and (dr[live] == e["draws"][live, mv]).all()


def test_frame_shapes_golden(golden):
    """Reference fixtures of the other BoardConfigs (tests/golden/shapes.npz) through the frame form:
    init, legal sets, apply_action transitions, seeded episodes."""
    g = golden("shapes")
    tags = sorted({k[len("init_seeds_"):] for k in g.files if k.startswith("init_seeds_")})
    assert len(tags) >= 6
    for tag in tags:
        R, C, T = (int(x) for x in tag.split("x"))
        hc = HostCore(R, C, T)
        out, drw, _, _ = hc.init(g["init_seeds_" + tag].astype(np.uint32))
        assert (out == g["init_boards_" + tag].reshape(len(out), -1)).all() and (drw == g["init_draws_" + tag]).all()
        bits = np.unpackbits(hc.legal(g["legal_boards_" + tag]).view(np.uint8), axis=1, bitorder="little")
        assert (bits[:, :hc.A] == g["legal_" + tag]).all(), tag
        ok = g["step_draws_" + tag] != -2
        out, rew, drw, _, _, _ = hc.apply(g["step_board_" + tag][ok], g["step_seed_" + tag][ok],
                                          g["step_n_actions_" + tag][ok], g["step_action_" + tag][ok], small=32)
        assert (out == g["step_next_" + tag][ok].reshape(len(out), -1)).all(), tag
        assert (rew == g["step_reward_" + tag][ok]).all(), tag
        live = g["step_draws_" + tag][ok] >= 0
        assert (drw[live] == g["step_draws_" + tag][ok][live]).all(), tag
        seeds = g["ep_seeds_" + tag].astype(np.uint32)
        b, _, _, act = hc.init(seeds)
        for mv in range(20):
            assert (act == g["ep_actions_" + tag][:, mv]).all(), (tag, mv)
            b, rew, drw, _, _, act = hc.apply(b, seeds, 20 - mv, act, small=32)
            assert (rew == g["ep_rewards_" + tag][:, mv]).all() and (drw == g["ep_draws_" + tag][:, mv]).all()
        assert (b == g["ep_final_" + tag].reshape(len(b), -1)).all(), tag


def test_frame_rows_below_columns_reset_only(golden):
    g = golden("shapes")
    for tag in ("8x10x5", "3x5x3"):
        R, C, T = (int(x) for x in tag.split("x"))
        out, drw, _, _ = HostCore(R, C, T).init(g["wide_seeds_" + tag].astype(np.uint32))
        assert (out == g["wide_boards_" + tag].reshape(len(out), -1)).all() and (drw == g["wide_draws_" + tag]).all()


def test_wide_frame_big_boards_golden(golden):
    """The 32 x 32 frame (boards with a side > 16) on the host against tests/golden/big.npz:
    resets, legal sets, apply_action transitions and seeded episodes of 20x20x6, 24x17x5, 17x17x3
    and 32x32x8, and the 5-bit token layouts of 9x9x20 and 12x12x31 (types 16..31)."""
    g = golden("big")
    for tag in ("20x20x6", "24x17x5", "17x17x3", "32x32x8", "9x9x20", "12x12x31"):
        R, C, T = (int(x) for x in tag.split("x"))
        hc = HostCore(R, C, T)
        assert hc.frame
        out, drw, _, _ = hc.init(g["init_seeds_" + tag].astype(np.uint32))
        assert (out == g["init_boards_" + tag].reshape(len(out), -1)).all() and (drw == g["init_draws_" + tag]).all()
        bits = np.unpackbits(hc.legal(g["legal_boards_" + tag]).view(np.uint8), axis=1, bitorder="little")
        assert (bits[:, :hc.A] == g["legal_" + tag]).all(), tag
        ok = g["step_draws_" + tag] != -2
        out, rew, drw, _, _, _ = hc.apply(g["step_board_" + tag][ok], g["step_seed_" + tag][ok],
                                          g["step_n_actions_" + tag][ok], g["step_action_" + tag][ok], small=32)
        assert (out == g["step_next_" + tag][ok].reshape(len(out), -1)).all(), tag
        assert (rew == g["step_reward_" + tag][ok]).all(), tag
        live = g["step_draws_" + tag][ok] >= 0
        assert (drw[live] == g["step_draws_" + tag][ok][live]).all(), tag
        seeds = g["ep_seeds_" + tag].astype(np.uint32)
        if not len(seeds):
            continue
        b, _, _, act = hc.init(seeds)
        for mv in range(20):
            assert (act == g["ep_actions_" + tag][:, mv]).all(), (tag, mv)
            b, rew, drw, _, _, act = hc.apply(b, seeds, 20 - mv, act, small=32)
            assert (rew == g["ep_rewards_" + tag][:, mv]).all() and (drw == g["ep_draws_" + tag][:, mv]).all()
        assert (b == g["ep_final_" + tag].reshape(len(b), -1)).all(), tag


@pytest.mark.parametrize("shape", [(10, 8, 9), (10, 8, 5), (12, 12, 7), (9, 9, 6), (16, 16, 8)],
                         ids=lambda s: "x".join(map(str, s)))
def test_rollouts_vs_oracle_on_host(shape):
    """k_rollout's rollout_one, compiled for the host, against the oracle's MCTS.rollout
    (mctslib/standard/mcts.py:14-19) on the shapes whose frame rollouts came out wrong on the GPU
    only with busy neighbour lanes (round 4/5 lane interference): the composed rule code
    is exact here after 1, 2, 5 and 20 moves, so the GPU failure was not in the source's logic
    (the MSan run of the same harness, tests/hostcore msan target, checks for uninitialised reads)."""
    R, C, T = shape
    hc, o = HostCore(R, C, T), Oracle(R, C, T, episode_shuffle_cap=1024)
    n = 256
    seeds = np.arange(1, n + 1, dtype=np.uint32)
    boards, _, _, _ = hc.init(seeds)
    rs = (np.arange(n, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    for k in (1, 2, 5, 20):
        g = hc.rollouts(boards, seeds, k, rs)
        w = o.rollouts(boards.astype(np.int32), seeds, k, rs, threads=4)
        ok = g["gain"] >= 0  # (chain overflow: replayed on the GPU by k_rollout_fix)
        assert ok.mean() > 0.95
        assert (g["gain"][ok] == w["gain"][ok]).all() and (g["steps"][ok] == w["steps"][ok]).all()
        assert (g["draws"][ok].astype(np.int64) == w["draws"][ok]).all()
        assert ((g["flags"][ok] & 0x1F) == (w["flags"][ok] & 0x1F)).all()
