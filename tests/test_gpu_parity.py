"""HIP path (libm3.so on the MI355X) vs the reference's golden vectors and the C oracle.

Bar: bit-exact boards, rewards, raw-draw counts, flags, legal sets and seeded
random actions. Sizes: every golden fixture, 65,536 boards x 20 moves against
the oracle (config C2), the 16x16x8 shape (C4 sample), and size-independent
properties at 1,048,576 boards (C3).
"""
import numpy as np
import pytest

from conftest import SHAPES

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.batched import BatchedMatch3Env  # noqa: E402
from oracle import FLAG_SHUFFLE_CAP, Oracle  # noqa: E402

BIG = 2**31 - 1


@pytest.fixture(scope="module")
def ctxs():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")
    return {tag: _native.Context(*shape) for tag, shape in SHAPES.items()}


def unpack(words, A):
    return np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), axis=-1,
                         bitorder="little")[..., :A]


@pytest.mark.parametrize("tag", list(SHAPES))
def test_init_boards_golden(golden, ctxs, tag):
    g = golden("init")
    boards, draws, _ = ctxs[tag].init_boards(g["seeds_" + tag].astype(np.uint32))
    assert (boards == g["boards_" + tag]).all()
    assert (draws == g["draws_" + tag]).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_legal_golden(golden, ctxs, tag):
    g = golden("legal")
    bits = unpack(ctxs[tag].legal_bits(g["boards_" + tag]), ctxs[tag].A)
    assert (bits == g["legal_" + tag]).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_apply_action_golden(golden, ctxs, tag):
    g = golden("steps")
    r = ctxs[tag].apply_actions(g["board_" + tag], g["seed_" + tag], g["n_actions_" + tag], g["action_" + tag])
    assert (r["boards"] == g["next_" + tag]).all()
    assert (r["reward"] == g["reward_" + tag]).all()
    live = g["draws_" + tag] >= 0
    assert (r["draws"][live] == g["draws_" + tag][live]).all()
    term = g["n_actions_" + tag] < 1
    assert (r["flags"][term] & _native.FLAG_TERMINAL).all()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_shuffle_golden(golden, ctxs, tag):
    g = golden("shuffle")
    r = ctxs[tag].apply_actions(g["board_" + tag], g["seed_" + tag], 20, g["action_" + tag])
    t = g["terminates_" + tag] == 1
    assert (r["boards"][t] == g["next_" + tag][t]).all()
    assert (r["reward"][t] == g["reward_" + tag][t]).all()
    assert (r["draws"][t] == g["draws_" + tag][t]).all()
    assert not (r["flags"][t] & FLAG_SHUFFLE_CAP).any()
    assert (r["flags"][~t] & FLAG_SHUFFLE_CAP).all()
    assert (r["flags"] & _native.FLAG_SHUFFLED).sum() > 100


def run_env_episodes(shape, seeds, moves=20, goal=BIG):
    env = BatchedMatch3Env(len(seeds), *shape, num_moves=moves, env_goal=goal, seeds=seeds, autoreset=False)
    acts, rews, drws, dones = [], [], [], []
    for _ in range(moves):
        acts.append(env.next_actions())
        env.step()
        rews.append(env.rewards())
        drws.append(env.draws())
        dones.append(env.dones())
    out = dict(actions=np.array(acts).T, rewards=np.array(rews).T, draws=np.array(drws).T, done=np.array(dones).T,
               final=env.observations().reshape(len(seeds), -1), flags=env.flags(), scores=env.scores())
    env.close()
    return out


@pytest.mark.parametrize("tag", list(SHAPES))
def test_seeded_episodes_golden(golden, tag):
    g = golden("episodes")
    e = run_env_episodes(SHAPES[tag], g["seeds_" + tag].astype(np.uint32))
    assert (e["actions"] == g["actions_" + tag]).all()
    assert (e["rewards"] == g["rewards_" + tag]).all()
    assert (e["draws"] == g["draws_" + tag]).all()
    assert (e["final"] == g["final_" + tag].reshape(len(e["final"]), -1)).all()


def test_c2_65536_boards_vs_oracle():
    """Config C2: 65,536 parallel 9x9x6 boards, 20 seeded moves, every move bit-exact."""
    seeds = (np.arange(65536, dtype=np.uint64) * 2654435761 + 1).astype(np.uint32)
    e = run_env_episodes((9, 9, 6), seeds, goal=500)
    o = Oracle(9, 9, 6).batch_episodes(seeds, 20, 500)
    m = o["moves"]
    mask = np.arange(20)[None, :] < m[:, None]
    assert (e["actions"][mask] == o["actions"][mask]).all()
    assert (e["rewards"][mask] == o["rewards"][mask]).all()
    assert (e["draws"][mask] == o["draws"][mask]).all()
    # done flags: the env reports done at the oracle's last move
    assert (e["done"][np.arange(len(m)), m - 1] == 1).all()
    # boards that ran all 20 moves end on the oracle's final board
    full = m == 20
    assert (e["final"][full] == o["final"][full]).all()
    assert full.mean() > 0.3


def test_c4_16x16_sample_vs_oracle():
    seeds = (np.arange(4096, dtype=np.uint64) * 40503 + 7).astype(np.uint32)
    e = run_env_episodes((16, 16, 8), seeds)
    o = Oracle(16, 16, 8).batch_episodes(seeds, 20)
    assert (e["actions"] == o["actions"]).all()
    assert (e["rewards"] == o["rewards"]).all()
    assert (e["final"] == o["final"]).all()


@pytest.mark.parametrize("shape", [(9, 9, 6), (16, 16, 8)], ids=["9x9x6", "16x16x8"])
def test_env_legal_sets_derived_and_eager(shape):
    """M3_ENV_LEGAL is derived: m3_env_get computes it from the boards (lazy), and after
    m3_env_device_ptr of it every step writes it (eager, for device consumers) -- through steps
    autoresets (10-move episodes, 25 steps) both equal the stateless legal kernel on the boards."""
    R, C, T = shape
    n = 8192
    lazy = BatchedMatch3Env(n, R, C, T, num_moves=10, env_goal=BIG, seed_base=3, autoreset=True, seed_stride=n)
    eager = BatchedMatch3Env(n, R, C, T, num_moves=10, env_goal=BIG, seed_base=3, autoreset=True, seed_stride=n)
    assert eager.device_ptr(_native.ENV_LEGAL) != 0
    for t in range(25):
        lazy.step()
        eager.step()
        if t % 4 == 3 or t == 24:
            want = lazy.ctx.legal_bits(lazy.observations())
            assert (lazy.legal_bits() == want).all(), t
            assert (eager.observations() == lazy.observations()).all(), t
            assert (eager.legal_bits() == want).all(), t
    lazy.close()
    eager.close()


def test_c3_1m_boards_properties():
    """Config C3 size: 1,048,576 boards. Size-independent checks + a sampled oracle check."""
    n = 1 << 20
    env = BatchedMatch3Env(n, num_moves=20, env_goal=BIG, seed_base=1, autoreset=False)
    ctx = env.ctx
    obs0 = env.observations().reshape(n, -1)
    legal0 = env.legal_bits()
    # legal bitset kept by the env == stateless legal kernel on the same boards
    idx = np.random.default_rng(0).choice(n, 4096, replace=False)
    assert (ctx.legal_bits(obs0[idx]) == legal0[idx]).all()
    total = np.zeros(n, np.int64)
    shuffled = np.zeros(n, bool)
    for _ in range(20):
        env.step()
        r = env.rewards()
        assert (r >= 0).all()
        total += r
        shuffled |= (env.flags() & _native.FLAG_SHUFFLED) != 0
    obs = env.observations().reshape(n, -1)
    allowed = np.array([1, 2, 3, 4, 5, 6, 8, 16, 24, 32], np.int8)
    assert np.isin(obs, allowed).all()
    assert (env.moves() == 20).all() and env.dones().all()
    assert (env.scores() == total).all()
    # sampled boards, and every board that went dead (its step continued in k_env_cont at the
    # row shuffle, ~1e-5 of steps: ~150 boards here), replayed through the oracle
    assert shuffled.sum() >= 10, shuffled.sum()
    idx = np.union1d(idx, np.flatnonzero(shuffled))
    o = Oracle().batch_episodes((idx + 1).astype(np.uint32), 20)
    assert (o["final"] == obs[idx]).all()
    assert (o["rewards"].sum(1) == total[idx]).all()
    env.close()


@pytest.mark.parametrize("tag", list(SHAPES))
def test_autoreset_matches_fresh_episodes(tag):
    """After autoreset, a board continues with seed + stride exactly like a fresh episode.
    (5-move episodes: the second episode's cells come from fill_next_slots' explicit reset; the
    prefetch path of later episodes is test_autoreset_prefetched_episodes_16x16x8.)"""
    n = 2048
    env = BatchedMatch3Env(n, *SHAPES[tag], num_moves=5, env_goal=BIG, seed_base=100, autoreset=True, seed_stride=n)
    for _ in range(5):
        env.step()
    assert env.dones().all()
    assert (env.seeds() == np.arange(100 + n, 100 + 2 * n, dtype=np.uint32)).all()
    fresh_boards, _, fresh_first = _native.Context(*SHAPES[tag]).init_boards(np.arange(100 + n, 100 + 2 * n, dtype=np.uint32))
    assert (env.observations() == fresh_boards).all()
    assert (env.next_actions() == fresh_first).all()
    assert (env.moves() == 0).all() and (env.scores() == 0).all()
    # the second episode steps like a fresh env on those seeds (the reset's per-board RNG state)
    fresh = BatchedMatch3Env(n, *SHAPES[tag], num_moves=5, env_goal=BIG,
                             seeds=np.arange(100 + n, 100 + 2 * n, dtype=np.uint32), autoreset=False)
    for _ in range(4):
        env.step()
        fresh.step()
        assert (env.rewards() == fresh.rewards()).all()
        assert (env.observations() == fresh.observations()).all()
    fresh.close()
    env.close()


def test_autoreset_prefetched_episodes_16x16x8():
    """The step's own prefetch resets, checked on their output: with one-move episodes
    every step autoresets every board, so steps 4.. swap in episodes that the two-stage 16x16x8 reset
    (k_reset_stream + k_reset_tiles, the rare sixth-round boards deferred to k_init_coop) built
    during the run. After each of 10 steps the boards, first actions and seeds must equal an
    explicit reset of seed_base + b + k * n (k_init_fix_lane), and a sample the oracle's
    BoardV2.__init__ (boardv2.py:17-27). 8,192 boards: ~33 per episode need the sixth round."""
    n, base = 8192, 100
    shape = (16, 16, 8)
    env = BatchedMatch3Env(n, *shape, num_moves=1, env_goal=BIG, seed_base=base, autoreset=True, seed_stride=n)
    ctx = _native.Context(*shape)
    o = Oracle(*shape)
    pick = np.random.RandomState(5).choice(n, 48, replace=False)
    for k in range(1, 11):
        env.step()
        assert env.dones().all()
        seeds = np.arange(base + k * n, base + (k + 1) * n, dtype=np.uint32)
        assert (env.seeds() == seeds).all(), f"step {k}: seeds"
        want, _, want_first = ctx.init_boards(seeds)
        obs = env.observations()
        bad = (obs.reshape(n, -1) != want.reshape(n, -1)).any(1)
        assert not bad.any(), f"step {k}: {int(bad.sum())} boards differ from a fresh reset (first {np.nonzero(bad)[0][:5]})"
        assert (env.next_actions() == want_first).all(), f"step {k}: first actions"
        assert (env.moves() == 0).all() and (env.scores() == 0).all()
        assert not (env.flags() & _native.FLAG_RESET_CAP).any()
        for i in pick[(k - 1) * 4:k * 4 + 4]:
            ob, _ = o.init_board(int(seeds[i]))
            assert (ob == obs[i]).all(), f"step {k}: board {i} vs the oracle"
    ctx.close()
    env.close()


def test_determinism_and_checksum():
    a = run_env_episodes((9, 9, 6), np.arange(1, 20001, dtype=np.uint32))
    b = run_env_episodes((9, 9, 6), np.arange(1, 20001, dtype=np.uint32))
    for k in ("actions", "rewards", "final"):
        assert (a[k] == b[k]).all()


def test_edge_inputs(ctxs):
    c = ctxs["9x9x6"]
    # empty batch
    r = c.apply_actions(np.zeros((0, 9, 9), np.int8), [], [], [])
    assert r["boards"].shape == (0, 9, 9)
    # bad action ids and terminal boards leave the board untouched
    b, _, _ = c.init_boards([5, 6, 7, 8])
    r = c.apply_actions(b, [5, 6, 7, 8], [20, 20, 0, -1], [-1, 144, 3, 3])
    assert (r["boards"] == b).all() and (r["reward"] == 0).all()
    assert (r["flags"][:2] & _native.FLAG_BAD_ACTION).all()
    assert (r["flags"][2:] & _native.FLAG_TERMINAL).all()
    # out-of-range cell values are rejected on the host
    with pytest.raises(ValueError):
        c.apply_actions(np.full((1, 9, 9), 200), [1], [20], [0])
    # ragged tail: batch sizes that are not a multiple of the 256-board workgroup
    for n in (1, 255, 257, 1000):
        seeds = np.arange(1, n + 1, dtype=np.uint32)
        bb, _, fa = c.init_boards(seeds)
        r = c.apply_actions(bb, seeds, 20, fa)
        o = Oracle()
        for i in (0, n // 2, n - 1):
            ob, orr, od, _ = o.apply_action(bb[i].astype(np.int32), int(seeds[i]), int(fa[i]))
            assert (r["boards"][i] == ob).all() and r["reward"][i] == orr and r["draws"][i] == od


def test_shards_do_not_change_results():
    """Boards split over 1, 3 or 8 HIP streams step identically (autoreset on, env_goal 500)."""
    n = 300_000
    outs = []
    for shards in (1, 3, 8):
        env = BatchedMatch3Env(n, num_moves=20, env_goal=500, seed_base=7, autoreset=True, shards=shards)
        acc = np.zeros(n, np.int64)
        for _ in range(25):
            env.step()
            acc = acc * 3 + env.rewards()
        outs.append((env.observations().copy(), acc, env.seeds().copy(), env.next_actions().copy()))
        env.close()
    for o in outs[1:]:
        for x, y in zip(outs[0], o):
            assert (x == y).all()


def test_explicit_actions_match_stateless_apply():
    """env.step(actions) == BoardV2.apply_action on the same boards (host actions path)."""
    n = 4096
    env = BatchedMatch3Env(n, num_moves=20, env_goal=BIG, seed_base=11, autoreset=False, shards=2)
    ctx = env.ctx
    rng = np.random.default_rng(3)
    for m in range(5):
        obs = env.observations()
        acts = rng.integers(0, 144, size=n).astype(np.int32)
        ref = ctx.apply_actions(obs, env.seeds(), 20 - m, acts)
        env.step(acts)
        assert (env.observations() == ref["boards"]).all()
        assert (env.rewards() == ref["reward"]).all()
    env.close()


def test_c4_262144_boards_autoreset_properties():
    """Config C4 at its stated size: 262,144 x 16x16x8 boards, 20 steps of seeded random play with
    same-step autoreset (env_goal 500, so truncated episodes restart mid-run). Every board, every
    step: values in {1..8, 16, 32} (clip(0, 32), boardv2.py:163: bombs 48 and megas 64 become 32),
    rewards >= 0, score == sum of the episode's rewards, done == truncated or 20 moves, truncated ==
    score >= goal; the env's legal bitset == the stateless legal kernel on a sample; then 4,096
    sampled boards plus every board that shuffled or needed more than the one-level chain's draws
    (the k_env_fix recompute) replayed through the oracle from their first episode."""
    import sys

    from conftest import ROOT

    sys.path.insert(0, ROOT)
    import bench

    n, goal = 1 << 18, 500
    env = BatchedMatch3Env(n, 16, 16, 8, num_moves=20, env_goal=goal, seed_base=1, autoreset=True, shards=2)
    allowed = np.array(list(range(1, 9)) + [16, 32], np.int8)
    ep_total = np.zeros(n, np.int64)
    moves = np.zeros(n, np.int64)
    special = np.zeros(n, bool)
    resets = 0
    for t in range(20):
        env.step()
        r, dn, tr = env.rewards(), env.dones(), env.truncateds()
        assert (r >= 0).all()
        ep_total += r
        moves += 1
        assert (dn == (tr | (moves == 20))).all(), t
        assert (tr == (ep_total >= goal)).all(), t
        sc, mv = env.scores(), env.moves()
        assert (sc[~dn] == ep_total[~dn]).all() and (mv[~dn] == moves[~dn]).all(), t
        assert (sc[dn] == 0).all() and (mv[dn] == 0).all(), t
        ep_total[dn] = 0
        moves[dn] = 0
        resets += int(dn.sum())
        special |= ((env.flags() & _native.FLAG_SHUFFLED) != 0) | (env.draws() >= 227)
        if t in (0, 9, 19):
            assert np.isin(env.observations(), allowed).all(), t
    assert resets > n // 4, resets  # truncations restarted episodes mid-run
    obs = env.observations().reshape(n, -1)
    idx = np.random.default_rng(1).choice(n, 4096, replace=False)
    assert (env.ctx.legal_bits(obs[idx]) == env.legal_bits()[idx]).all()
    idx = np.union1d(idx, np.flatnonzero(special))
    chk = bench.oracle_sample_check(env, (16, 16, 8), 20, goal, 1, n, 20, idx=idx)
    assert chk["boards"] == len(idx) and chk["mismatches"] == 0, chk
    env.close()


def test_abi_rejects_bad_cells_on_device(ctxs):
    """A cell byte outside [0, 127] (int8 < 0) handed straight to the C ABI is caught while the
    boards are staged on the device (no host pass over the bytes): M3_ERR_INVALID."""
    c = ctxs["9x9x6"]
    n = 300
    seeds = np.arange(1, n + 1, dtype=np.uint32)
    b, _, fa = c.init_boards(seeds)
    b = np.ascontiguousarray(b.reshape(n, -1))
    b[257, 40] = -3  # fifth wave
    na = np.full(n, 20, np.int32)
    fa = np.ascontiguousarray(fa, dtype=np.int32)
    outs = [np.empty(n * 81, np.int8)] + [np.empty(n, np.int32) for _ in range(3)]
    routs = [np.empty(n, np.int32) for _ in range(4)]  # every buffer outlives the calls
    P = _native.ptr
    L = _native.lib()
    rc = L.m3_apply_actions(c.handle, n, P(b), P(seeds), P(na), P(fa), *[P(o) for o in outs], None, None)
    assert rc == -1 and b"outside [0, 127]" in L.m3_last_error()
    rc = L.m3_rollouts(c.handle, n, P(b), P(seeds), P(na), P(seeds), *[P(o) for o in routs], None)
    assert rc == -1
    b[257, 40] = 3  # a valid value: both calls succeed again on the same context
    _native.check(L.m3_apply_actions(c.handle, n, P(b), P(seeds), P(na), P(fa), *[P(o) for o in outs], None, None))
    _native.check(L.m3_rollouts(c.handle, n, P(b), P(seeds), P(na), P(seeds), *[P(o) for o in routs], None))
