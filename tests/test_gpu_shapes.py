"""Every other BoardConfig through the same C-ABI: the frame kernels (FCfg, m3_rules.hpp).

Reference fixtures (tests/golden/shapes.npz, gen_golden.py: gen_shapes) for square boards,
rows > columns, columns = 3 (boardConfig.py:50's literal 3 sends vertical ids of row r to row
r - 1), three and fifteen tile types; the oracle for large batches; and rows < columns, where
the reference resets fine but its legal_actions / apply_action raise IndexError."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.batched import BatchedMatch3Env  # noqa: E402
from oracle import Oracle  # noqa: E402

BIG = 2**31 - 1


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


def _tags(g, prefix):
    return sorted({k[len(prefix):] for k in g.files if k.startswith(prefix)})


def _shape(tag):
    return tuple(int(x) for x in tag.split("x"))


def unpack(words, A):
    return np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), axis=-1, bitorder="little")[..., :A]


def test_fixture_covers_the_asked_shapes(golden):
    g = golden("shapes")
    tags = _tags(g, "init_seeds_")
    for t in ("7x7x4", "8x8x5", "10x8x5", "5x3x3", "12x12x7"):
        assert t in tags
    assert set(_tags(g, "wide_seeds_")) == {"8x10x5", "3x5x3"}


def _check_golden_shape(g, tag):
    """init / legal / apply_action / seeded-episode fixtures of one BoardConfig through the C-ABI"""
    R, C, T = _shape(tag)
    ctx = _native.Context(R, C, T)
    A = ctx.A
    boards, draws, _ = ctx.init_boards(g["init_seeds_" + tag].astype(np.uint32))
    assert (boards == g["init_boards_" + tag]).all(), tag
    assert (draws == g["init_draws_" + tag]).all(), tag
    bits = unpack(ctx.legal_bits(g["legal_boards_" + tag]), A)
    assert (bits == g["legal_" + tag]).all(), tag
    ok = g["step_draws_" + tag] != -2  # (-2: the reference hangs in a cycling shuffle)
    r = ctx.apply_actions(g["step_board_" + tag][ok], g["step_seed_" + tag][ok], g["step_n_actions_" + tag][ok],
                          g["step_action_" + tag][ok])
    assert (r["boards"] == g["step_next_" + tag][ok]).all(), tag
    assert (r["reward"] == g["step_reward_" + tag][ok]).all(), tag
    live = g["step_draws_" + tag][ok] >= 0
    assert (r["draws"][live] == g["step_draws_" + tag][ok][live]).all(), tag
    # seeded random_task episodes through the batched env (its step / reset / random-action kernels)
    seeds = g["ep_seeds_" + tag].astype(np.uint32)
    if len(seeds):
        env = BatchedMatch3Env(len(seeds), R, C, T, num_moves=20, env_goal=BIG, seeds=seeds, autoreset=False)
        assert (env.observations() == g["ep_init_" + tag]).all(), tag
        for m in range(20):
            assert (env.next_actions() == g["ep_actions_" + tag][:, m]).all(), (tag, m)
            env.step()
            assert (env.rewards() == g["ep_rewards_" + tag][:, m]).all(), (tag, m)
            assert (env.draws() == g["ep_draws_" + tag][:, m]).all(), (tag, m)
        assert (env.observations() == g["ep_final_" + tag]).all(), tag
        env.close()
    ctx.close()


def test_frame_shapes_golden(golden):
    g = golden("shapes")
    for tag in _tags(g, "init_seeds_"):
        _check_golden_shape(g, tag)


def test_big_boards_golden(golden):
    """Boards past 16 x 16 (the 32 x 32 frame, FCfg<BITS, 32>): 20x20x6, 24x17x5, 17x17x3 and
    32x32x8, and types 16..31 (5 token bits, FCfg<5>): 9x9x20, 12x12x31, against
    tests/golden/big.npz (gen_golden.py: gen_big). 17x17x3 has no episodes: the
    reference's seeded play there runs into cascades it does not finish within the generator's
    5 s per episode."""
    g = golden("big")
    tags = _tags(g, "init_seeds_")
    assert {"20x20x6", "24x17x5", "32x32x8", "17x17x3", "9x9x20", "12x12x31"} <= set(tags)
    for tag in tags:
        _check_golden_shape(g, tag)


def test_big_boards_rollouts_vs_oracle():
    """MCTS rollouts on 20x20x6 (one 32 x 32-frame board per lane, whole waves) against the oracle."""
    R, C, T = 20, 20, 6
    ctx = _native.Context(R, C, T)
    seeds = np.arange(1, 257, dtype=np.uint32)
    boards, _, _ = ctx.init_boards(seeds)
    rs = (np.arange(256, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    ro = ctx.rollouts(boards, seeds, 20, rs)
    want = Oracle(R, C, T).rollouts(boards.astype(np.int32), seeds, 20, rs, threads=4)
    assert (ro["gain"] == want["gain"]).all() and (ro["steps"] == want["steps"]).all()
    assert (ro["draws"] == want["draws"]).all()
    ctx.close()


def test_rows_below_columns_reset_but_do_not_step(golden):
    """rows < columns: BoardV2.__init__ as the reference; legal_actions / apply_action raise IndexError
    there (and here) -- the C-ABI refuses them with M3_ERR_INVALID."""
    from match3tile.boardConfig import BoardConfig
    from match3tile.boardv2 import BoardV2
    from match3tile.env import Match3Env

    g = golden("shapes")
    for tag in _tags(g, "wide_seeds_"):
        R, C, T = _shape(tag)
        assert list(g["wide_errors_" + tag]) == ["IndexError"]
        ctx = _native.Context(R, C, T)
        boards, draws, _ = ctx.init_boards(g["wide_seeds_" + tag].astype(np.uint32))
        assert (boards == g["wide_boards_" + tag]).all() and (draws == g["wide_draws_" + tag]).all()
        with pytest.raises(_native.M3Error) as e:
            ctx.legal_bits(boards[:1])
        assert e.value.code == -1
        with pytest.raises(_native.M3Error):
            ctx.apply_actions(boards[:1], [1], 20, 0)
        b = BoardV2(20, BoardConfig(seed=1, rows=R, columns=C, types=T))
        assert (b.array == g["wide_boards_" + tag][0]).all()
        with pytest.raises(IndexError):
            b.legal_actions
        with pytest.raises(IndexError):
            b.apply_action(0)
        env = Match3Env(width=C, height=R, num_types=T, seed=3)
        with pytest.raises(IndexError):
            env.step(0)
        ctx.close()


@pytest.mark.parametrize("shape", [(12, 12, 7), (8, 8, 5), (5, 3, 3)], ids=lambda s: "x".join(map(str, s)))
def test_frame_env_large_batch_vs_oracle(shape):
    """262,144 boards (C4-sized batch) of a frame shape, 20 seeded moves with autoreset off: size-
    independent checks on all, every move of a 2,048-board sample against the oracle."""
    R, C, T = shape
    n = 1 << 18
    env = BatchedMatch3Env(n, R, C, T, num_moves=20, env_goal=BIG, seed_base=11, autoreset=False, shards=2)
    total = np.zeros(n, np.int64)
    idx = np.random.default_rng(0).choice(n, 2048, replace=False)
    rews, acts = [], []
    for _ in range(20):
        acts.append(env.next_actions()[idx])
        env.step()
        r = env.rewards()
        assert (r >= 0).all()
        total += r
        rews.append(r[idx])
    assert (env.scores() == total).all() and (env.moves() == 20).all()
    cap = (env.flags() & (_native.FLAG_SHUFFLE_CAP | _native.FLAG_CASCADE_CAP)) != 0
    o = Oracle(R, C, T, episode_shuffle_cap=1024).batch_episodes((idx + 11).astype(np.uint32), 20, BIG)
    ok = (o["moves"] == 20) & ~cap[idx]
    assert ok.mean() > 0.95
    assert (np.array(acts).T[ok] == o["actions"][ok]).all()
    assert (np.array(rews).T[ok] == o["rewards"][ok]).all()
    assert (env.observations().reshape(n, -1)[idx][ok] == o["final"][ok]).all()
    env.close()


@pytest.mark.parametrize("shape", [(10, 8, 5), (12, 12, 7), (10, 10, 6), (10, 8, 9), (16, 16, 15), (10, 8, 3),
                                   (12, 12, 20)],
                         ids=lambda s: "x".join(map(str, s)))
def test_frame_rollouts_vs_oracle(shape):
    """MCTS rollouts (f3) of 4096 states, 64 lanes a wave, on frame shapes of every token width.
    Regression guard for the round-4 lane interference: a value live out of a
    divergent loop (the RNG position after the cascade) came back as garbage for lanes that had
    left the loop early, in kernels that spilled VGPRs -- a board was exact alone and wrong only
    with busy neighbours. Token widths 2..5 bits. Fails on the pre-fix library (build/libm3_pre.so: 55 / 70 / 1,662 of
    4,096 wrong on 12x12x7 / 10x8x5 / 10x8x9, profiles/r05_lane_regression.txt), passes now."""
    R, C, T = shape
    ctx = _native.Context(R, C, T)
    seeds = np.arange(1, 4097, dtype=np.uint32)
    boards, _, _ = ctx.init_boards(seeds)
    rs = (np.arange(4096, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    ro = ctx.rollouts(boards, seeds, 20, rs)
    want = Oracle(R, C, T).rollouts(boards.astype(np.int32), seeds, 20, rs, threads=4)
    assert (ro["gain"] == want["gain"]).all() and (ro["steps"] == want["steps"]).all()
    assert (ro["draws"] == want["draws"]).all()
    ctx.close()


def test_frame_autoreset_vs_oracle():
    """Same-step autoreset (f1) on a frame shape."""
    R, C, T = 10, 8, 5
    ctx = _native.Context(R, C, T)
    n = 2048
    env = BatchedMatch3Env(n, R, C, T, num_moves=5, env_goal=BIG, seed_base=100, autoreset=True, seed_stride=n)
    for _ in range(5):
        env.step()
    assert env.dones().all()
    fresh, _, first = ctx.init_boards(np.arange(100 + n, 100 + 2 * n, dtype=np.uint32))
    assert (env.observations() == fresh).all() and (env.next_actions() == first).all()
    env.close()
    ctx.close()


def test_two_types_golden(golden):
    """BoardConfig(types=2) against tests/golden/types2.npz: resets and legal sets on 4x4 .. 12x7,
    apply_action transitions and seeded random_task episodes on 4x4, 5x5 and 6x6 (where the
    reference's cascade returns)."""
    g = golden("types2")
    tags = _tags(g, "init_seeds_")
    assert {"4x4x2", "5x5x2", "6x6x2", "9x9x2", "12x7x2"} <= set(tags)
    for tag in tags:
        R, C, T = _shape(tag)
        ctx = _native.Context(R, C, T)
        boards, draws, _ = ctx.init_boards(g["init_seeds_" + tag].astype(np.uint32))
        assert (boards == g["init_boards_" + tag]).all(), tag
        assert (draws == g["init_draws_" + tag]).all(), tag
        assert (unpack(ctx.legal_bits(g["legal_boards_" + tag]), ctx.A) == g["legal_" + tag]).all(), tag
        if "step_board_" + tag in g.files:
            ok = g["step_draws_" + tag] != -2
            r = ctx.apply_actions(g["step_board_" + tag][ok], g["step_seed_" + tag][ok],
                                  g["step_n_actions_" + tag][ok], g["step_action_" + tag][ok])
            assert (r["boards"] == g["step_next_" + tag][ok]).all(), tag
            assert (r["reward"] == g["step_reward_" + tag][ok]).all(), tag
            live = g["step_draws_" + tag][ok] >= 0
            assert (r["draws"][live] == g["step_draws_" + tag][ok][live]).all(), tag
            seeds = g["ep_seeds_" + tag].astype(np.uint32)
            env = BatchedMatch3Env(len(seeds), R, C, T, num_moves=20, env_goal=BIG, seeds=seeds, autoreset=False)
            assert (env.observations() == g["ep_init_" + tag]).all(), tag
            for m in range(20):
                assert (env.next_actions() == g["ep_actions_" + tag][:, m]).all(), (tag, m)
                env.step()
                assert (env.rewards() == g["ep_rewards_" + tag][:, m]).all(), (tag, m)
            assert (env.observations() == g["ep_final_" + tag]).all(), tag
            env.close()
        ctx.close()


def test_two_types_large_board_steps_return_flagged(golden):
    """9x9x2: the reference's first move of seeded play mostly never returns (types2.npz records
    which of seeds 1..16 did within 3 s); here every step returns, and a step whose cascade ran
    into the 65,536-refill cap says so (M3_FLAG_CASCADE_CAP, parity undefined there; 6x6x2 steps of the
    fixture need up to ~10,000 refills, which the cap leaves exact)."""
    g = golden("types2")
    assert g["first_move_returns_9x9x2"].sum() < 16  # the reference hangs on some
    n = 512
    env = BatchedMatch3Env(n, 9, 9, 2, num_moves=20, env_goal=BIG, seed_base=1, autoreset=False)
    env.step()
    f = env.flags()
    capped = (f & _native.FLAG_CASCADE_CAP) != 0
    assert capped.any() and env.observations().shape == (n, 9, 9)
    obs = env.observations()
    assert np.isin(obs[~capped], [1, 2, 4, 8, 12, 16]).all()  # tiles 1..2, H 4, V 8, B 12, M 16 (TM 3)
    assert np.isin(obs[capped], [0, 1, 2, 4, 8, 12, 16]).all()  # (a capped cascade stops with its holes)
    env.close()


@pytest.mark.parametrize("shape", [(6, 6, 5), (9, 9, 7), (11, 11, 8), (13, 13, 9), (16, 16, 12), (16, 9, 7),
                                   (10, 3, 4), (12, 12, 20)], ids=lambda s: "x".join(map(str, s)))
def test_frame_full_waves_episodes_and_rollouts_vs_oracle(shape):
    """Every lane of every wave busy (4,096 boards): 20 seeded random-action env moves and then a
    20-move rollout from each final board, against the oracle -- the lane-interference guard of
    DESIGN.md §4 ("SGPR spills") on frame shapes of every token width (tools/dbg/frame_sweep.py
    runs 24 shapes)."""
    R, C, T = shape
    n = 4096
    seeds = np.arange(1, n + 1, dtype=np.uint32)
    env = BatchedMatch3Env(n, R, C, T, num_moves=20, env_goal=BIG, seeds=seeds, autoreset=False)
    acts, rews = [], []
    for _ in range(20):
        acts.append(env.next_actions())
        env.step()
        rews.append(env.rewards())
    o = Oracle(R, C, T, episode_shuffle_cap=1024).batch_episodes(seeds, 20, BIG)
    cap = (env.flags() & (_native.FLAG_SHUFFLE_CAP | _native.FLAG_CASCADE_CAP)) != 0
    ok = (o["moves"] == 20) & ~cap
    assert ok.mean() > 0.85
    assert (np.array(acts).T[ok] == o["actions"][ok]).all()
    assert (np.array(rews).T[ok] == o["rewards"][ok]).all()
    fin = env.observations().reshape(n, R, C).astype(np.int8)
    assert (fin.reshape(n, -1)[ok] == o["final"][ok]).all()
    env.close()
    ctx = _native.Context(R, C, T)
    rs = (np.arange(n, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    ro = ctx.rollouts(fin, seeds, 20, rs)
    want = Oracle(R, C, T).rollouts(fin.astype(np.int32), seeds, 20, rs)
    assert (ro["gain"] == want["gain"]).all() and (ro["steps"] == want["steps"]).all()
    assert (ro["draws"] == want["draws"]).all()
    ctx.close()


def _has_match(b):
    b = np.asarray(b)
    h = (b[:, :-2] == b[:, 1:-1]) & (b[:, 1:-1] == b[:, 2:]) & (b[:, :-2] > 0)
    v = (b[:-2, :] == b[1:-1, :]) & (b[1:-1, :] == b[2:, :]) & (b[:-2, :] > 0)
    return bool(h.any() or v.any())


def test_reset_cap_flag_reaches_callers_16x16x2():
    """16x16x2 resets need 0.4 M - 7.5 M draws (oracle, seeds 1..8), past the 16,384-round cap for
    most seeds: a reset stopped there returns a board that still has a match, and every caller must
    see M3_FLAG_RESET_CAP -- m3_init_boards_ex's flags (m3_init_boards refuses with M3_ERR_CAP), and
    the env's flags for an autoreset episode (the prefetched slot's flag)."""
    R, C, T = 16, 16, 2
    ctx = _native.Context(R, C, T)
    seeds = np.arange(1, 65, dtype=np.uint32)
    boards, draws, _, flags = ctx.init_boards(seeds, flags=True)
    capped = (flags & _native.FLAG_RESET_CAP) != 0
    assert capped.any() and (~capped).any()
    assert [_has_match(b) for b in boards] == list(capped)
    o = Oracle(R, C, T)
    for i in np.nonzero(~capped)[0][:3]:  # the ones that finished: the reference's board
        want, wdraws = o.init_board(int(seeds[i]))[:2]
        assert (boards[i].reshape(-1) == want.reshape(-1)).all() and int(draws[i]) == int(wdraws)
    with pytest.raises(_native.M3Error) as e:
        ctx.init_boards(seeds)
    assert e.value.code == -7  # M3_ERR_CAP
    n = 64
    env = BatchedMatch3Env(n, R, C, T, num_moves=1, env_goal=BIG, seed_base=1, autoreset=True, seed_stride=n)
    for _ in range(2):
        env.step()  # every episode is one move long: every board starts a new episode each step
        obs = env.observations()
        got = (env.flags() & _native.FLAG_RESET_CAP) != 0
        assert [_has_match(b) for b in obs] == list(got)
    env.close()
    ctx.close()
