#!/usr/bin/env python3
"""Generate golden vectors by running the REAL reference (read-only, this container only).

    PYTHONPATH=/root/reference python3 -B tests/golden/gen_golden.py

The reference (ThorLL/Element-Crush-Gym) ships no tests or fixtures of its own
(SURVEY.md §4), so these vectors are the parity anchor: every array in
``tests/golden/*.npz`` is produced by calling the reference's own functions
(``match3tile.boardv2.BoardV2``, ``match3tile.boardFunctions``, numpy's legacy
``RandomState``). Only data is committed -- no reference source.

Files written:
  prng.npz        MT19937 raw streams, randint/random_interval/shuffle/choice chains
  matches.npz     get_matches mask + get_match_spawn_mask on crafted + random token boards
  legal.npz       legal_actions bitmasks on play boards, boards with specials, dead boards
  init.npz        BoardV2.__init__ boards + raw draws consumed (9x9x6, 16x16x8)
  steps.npz       apply_action transitions (board, seed, n_actions, action) -> (board', reward, draws)
                  incl. specials, all combo pairs, typed specials, illegal swaps, terminal boards
  episodes.npz    samplerTasks.random_task-style seeded episodes (actions, rewards, draws, final board)
  shuffle.npz     dead-board transitions that terminate (shuffle path) + seeds that cycle forever
  env.npz         Match3Env runs of the README.md:18-31 loop (env.board.random_action(), step,
                  reset at done with and without a seed), bookkeeping restated over the reference
                  BoardV2 (env.py cannot run at the snapshot): obs/reward/done/truncated per step
  shapes.npz      init / legal / steps / episodes for BoardConfigs other than 9x9x6 and 16x16x8
  big.npz         init / legal / steps / episodes past the 16 x 16 frame (20x20 .. 32x32) and
                  for types 20 and 31
  types2.npz      BoardConfig(types=2): steps / episodes on 4x4, 5x5, 6x6 (where the reference's
                  cascade returns), resets and legal sets on 9x9, 12x7
                  (square, rows > columns, columns = 3 -- the decode quirk -- and few types), and
                  for rows < columns, where the reference's legal_actions / apply_action raise
                  IndexError, the init boards plus that error
"""
from __future__ import annotations

import os
import signal
import sys
from multiprocessing import Pool

sys.dont_write_bytecode = True
REF = os.environ.get("M3_REFERENCE", "/root/reference")
if REF not in sys.path:
    sys.path.insert(0, REF)

import numpy as np  # noqa: E402

from match3tile.boardConfig import BoardConfig  # noqa: E402
from match3tile.boardFunctions import get_matches, get_match_spawn_mask, legal_actions  # noqa: E402
from match3tile.boardv2 import BoardV2  # noqa: E402

OUT = os.path.dirname(os.path.abspath(__file__))
SHAPES = [(9, 9, 6), (16, 16, 8)]


class _Timeout(Exception):
    pass


def _alarm(signum, frame):
    raise _Timeout()


def raw(n):
    return np.random.mtrand._rand._bit_generator.random_raw(n).astype(np.uint32)


def draws_since_seed(seed: int) -> int:
    """Raw MT outputs consumed since np.random.seed(seed), read off numpy's global state."""
    st = np.random.get_state()
    key, pos = st[1], st[2]
    fresh = np.random.RandomState(seed).get_state()
    if pos == 624 and np.array_equal(fresh[1], key):
        return 0
    rs = np.random.RandomState(seed)
    rs._bit_generator.random_raw(pos)  # d = (t - 1) * 624 + pos for t = 1, 2, ...
    for t in range(1, 4096):
        s2 = rs.get_state()
        if s2[2] == pos and np.array_equal(s2[1], key):
            return (t - 1) * 624 + pos
        rs._bit_generator.random_raw(624)
    raise RuntimeError("could not determine draw count")


def legal_bits(cfg, arr):
    bits = np.zeros(cfg.action_space, dtype=np.uint8)
    for a in legal_actions(cfg, arr):
        bits[a] = 1
    return bits


# ------------------------------------------------------------------------- PRNG
def gen_prng():
    seeds = np.array([1, 100, 12345, 2**31 - 2, 2**32 - 1, 0, 7, 424242], dtype=np.uint64)
    raw_streams = []
    for s in seeds:
        np.random.seed(int(s))
        raw_streams.append(raw(1500))
    # randint chains with size (the reference's tile refill / init calls)
    chains = {}
    for hi in (7, 9):
        out = []
        for s in seeds:
            np.random.seed(int(s))
            out.append(np.random.randint(1, hi, size=300))
        chains[f"randint_1_{hi}"] = np.array(out, dtype=np.int64)
    # choice over lists of every length 1..200 (random_action contract, samplerTasks.py:13)
    ch = []
    for n in range(1, 201):
        np.random.seed(n * 7919)
        lst = list(range(1000, 1000 + n))
        ch.append([np.random.choice(lst) for _ in range(8)])
    # legacy shuffle of rows (boardFunctions.py:22)
    perms = []
    for R in (9, 16):
        for s in seeds:
            np.random.seed(int(s))
            a = np.arange(R * 3).reshape(R, 3)
            np.random.shuffle(a)
            perms.append(np.concatenate([a[:, 0] // 3, np.full(16 - R, -1)]))
    np.savez_compressed(os.path.join(OUT, "prng.npz"), seeds=seeds, raw=np.array(raw_streams),
                        choice=np.array(ch, dtype=np.int64), shuffle_rows=np.array(perms, dtype=np.int64),
                        **chains)


# ---------------------------------------------------------------------- matches
def crafted_token_boards(R, C, T, rng):
    boards = []
    z = lambda: rng.integers(1, T + 1, size=(R, C))  # noqa: E731
    # random boards have some runs; add a bunch of crafted shapes on top
    for _ in range(300):
        boards.append(z())
    shapes = []
    # L corner (horizontal arm starting at the corner), T, corner-both, line 4/5 h and v, cross, long lines
    shapes.append([(0, 0), (1, 0), (2, 0), (2, 1), (2, 2)])
    shapes.append([(0, 0), (0, 1), (0, 2), (1, 0), (2, 0)])
    shapes.append([(0, 1), (1, 1), (2, 1), (2, 0), (2, 2)])
    shapes.append([(1, 0), (1, 1), (1, 2), (0, 1), (2, 1)])
    shapes.append([(0, 0), (0, 1), (0, 2), (0, 3)])
    shapes.append([(0, 0), (0, 1), (0, 2), (0, 3), (0, 4)])
    shapes.append([(0, 0), (1, 0), (2, 0), (3, 0)])
    shapes.append([(0, 0), (1, 0), (2, 0), (3, 0), (4, 0)])
    shapes.append([(0, 2), (1, 2), (2, 2), (2, 0), (2, 1), (2, 3), (2, 4), (3, 2), (4, 2)])
    shapes.append([(0, 3), (1, 3), (2, 3), (2, 1), (2, 2), (3, 1), (4, 1), (2, 4)])
    shapes.append([(0, 0), (0, 1), (0, 2), (1, 2), (2, 2), (2, 3), (2, 4), (3, 4), (4, 4)])
    shapes.append([(r, 4) for r in range(7)])
    shapes.append([(4, c) for c in range(8)])
    for shp in shapes:
        for _ in range(12):
            b = z()
            orr, oc = rng.integers(0, 4), rng.integers(0, 4)
            v = rng.integers(1, T + 1)
            for (r, c) in shp:
                rr, cc = min(r + orr, R - 1), min(c + oc, C - 1)
                b[rr, cc] = v
            # sprinkle zeros (removed cells) sometimes
            if rng.random() < 0.3:
                b[rng.integers(0, R), rng.integers(0, C)] = 0
            boards.append(b)
    # few-type boards produce many/large merged groups
    for _ in range(150):
        boards.append(rng.integers(1, min(T, 3) + 1, size=(R, C)))
    for _ in range(60):
        b = rng.integers(1, 3, size=(R, C))
        b[rng.random((R, C)) < 0.15] = 0
        boards.append(b)
    return boards


def gen_matches():
    rng = np.random.default_rng(1234)
    out = {}
    for (R, C, T) in SHAPES:
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        tbs, masks, spawns, ngroups = [], [], [], []
        for b in crafted_token_boards(R, C, T, rng):
            b = np.asarray(b, dtype=np.int64)
            mask, matches = get_matches(b.copy())
            spawn = get_match_spawn_mask(cfg, [list(m) for m in matches])
            tbs.append(b)
            masks.append(mask)
            spawns.append(spawn)
            ngroups.append(len(matches))
        tag = f"{R}x{C}x{T}"
        out[f"tb_{tag}"] = np.array(tbs, dtype=np.int8)
        out[f"mask_{tag}"] = np.array(masks, dtype=np.uint8)
        out[f"spawn_{tag}"] = np.array(spawns, dtype=np.int32)
        out[f"ngroups_{tag}"] = np.array(ngroups, dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "matches.npz"), **out)


# ------------------------------------------------------------------------ init
def _init_one(args):
    R, C, T, seed = args
    cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
    b = BoardV2(20, cfg)
    return b.array.astype(np.int8), draws_since_seed(int(seed))


def gen_init(pool):
    out = {}
    for (R, C, T), n in zip(SHAPES, (1024, 256)):
        seeds = np.concatenate([np.arange(1, n - 3), [2**31 - 2, 2**32 - 1, 123456789, 987654321]]).astype(np.uint64)
        res = pool.map(_init_one, [(R, C, T, s) for s in seeds])
        tag = f"{R}x{C}x{T}"
        out[f"seeds_{tag}"] = seeds
        out[f"boards_{tag}"] = np.array([r[0] for r in res])
        out[f"draws_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "init.npz"), **out)


# ---------------------------------------------------------------------- episodes
def _episode(args):
    """samplerTasks.random_task (samplerTasks.py:9-14) with a fixed seed (None if the reference
    hangs in a cycling dead-board shuffle, boardv2.py:188-194, or raises in np.random.choice([])
    on a board without a legal action -- both possible on tiny boards)."""
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(5)
    try:
        return _episode_body(args)
    except (_Timeout, ValueError):  # ValueError: np.random.choice([]) -- a board with no legal action
        return None
    finally:
        signal.alarm(0)


def _episode_body(args):
    R, C, T, seed, moves = args
    cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
    state = BoardV2(moves, cfg)
    init_board = state.array.astype(np.int8)
    np.random.seed(cfg.seed)
    acts, rews, drws, boards = [], [], [], []
    prev = 0
    while not state.is_terminal:
        a = int(np.random.choice(state.legal_actions))
        state = state.apply_action(a)
        acts.append(a)
        rews.append(int(state.reward - prev))
        prev = state.reward
        drws.append(draws_since_seed(int(seed)))
        boards.append(state.array.astype(np.int8))
    return init_board, acts, rews, drws, boards


def gen_episodes(pool):
    out = {}
    for (R, C, T), n in zip(SHAPES, (1024, 192)):
        seeds = np.arange(1, n + 1, dtype=np.uint64)
        res = pool.map(_episode, [(R, C, T, s, 20) for s in seeds], chunksize=4)
        tag = f"{R}x{C}x{T}"
        out[f"seeds_{tag}"] = seeds
        out[f"init_{tag}"] = np.array([r[0] for r in res])
        out[f"actions_{tag}"] = np.array([r[1] for r in res], dtype=np.int16)
        out[f"rewards_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        out[f"draws_{tag}"] = np.array([r[3] for r in res], dtype=np.int16)
        # every board of the first 128 episodes, final board for all
        bs = np.array([r[4] for r in res])
        out[f"boards_{tag}"] = bs[:128]
        out[f"final_{tag}"] = bs[:, -1]
    np.savez_compressed(os.path.join(OUT, "episodes.npz"), **out)


# --------------------------------------------------------------------------- env
class _RefEnv:
    """Match3Env (env.py:8-65) restated over the REAL reference BoardV2.

    The reference class itself cannot run (env.py:38,64 pass a `seed` keyword
    BoardV2 does not take; env.py:50 unpacks a BoardV2), so only its
    bookkeeping is restated here: everything a step computes -- the board, its
    reward, the global RNG the next random action draws from -- comes from the
    reference's own BoardV2 / BoardConfig / numpy."""

    def __init__(self, width, height, num_types, num_moves, env_goal, seed):
        self.width, self.height, self.num_types = width, height, num_types
        self.num_moves, self.env_goal = num_moves, env_goal
        self.seed = seed
        self.score, self.moves_taken = 0, 0
        self.action_space = height * (width - 1) + width * (height - 1)          # env.py:36
        self.board = self._board()

    def _board(self):
        return BoardV2(self.num_moves, BoardConfig(seed=self.seed, rows=self.height, columns=self.width,
                                                   types=self.num_types))

    def step(self, action):                                                       # env.py:48-56
        before = self.board.reward
        self.board = self.board.apply_action(action)
        reward = int(self.board.reward - before)
        self.score += reward
        self.moves_taken += 1
        truncated = self.score >= self.env_goal
        done = truncated or self.num_moves == self.moves_taken
        return self.board.array, reward, done, truncated, {}

    def reset(self, seed=None):                                                   # env.py:58-65
        self.seed = seed if seed is not None else (1 + self.seed) % 2 ** 32 - 1
        self.score, self.moves_taken = 0, 0
        self.board = self._board()
        return self.board.array, {}


def _env_run(args):
    """None where the reference crashes (no legal action: np.random.choice([])) or hangs (a cycling
    dead-board shuffle) -- tiny boards only; gen_env keeps the runs that complete."""
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(20)
    try:
        return _env_run_body(args)
    except (_Timeout, ValueError):
        return None
    finally:
        signal.alarm(0)


def _env_run_body(args):
    """The README.md:18-31 loop: action = env.board.random_action() (= np.random.choice(
    board.legal_actions) from numpy's global stream, samplerTasks.py:13), step, reset at done
    with the next entry of `resets` (-1: reset() without a seed, the env.py:62 quirk)."""
    R, C, T, seed, moves, goal, n_steps, resets = args
    env = _RefEnv(C, R, T, moves, goal, int(seed))
    out = dict(init=env.board.array.astype(np.int8), action=[], obs=[], reward=[], done=[], trunc=[],
               reset_arg=[], reset_obs=[], seed_after=[])
    resets = list(resets)
    for _ in range(n_steps):
        a = int(np.random.choice(env.board.legal_actions))
        obs, r, done, tr, _ = env.step(a)
        out["action"].append(a)
        out["obs"].append(obs.astype(np.int8))
        out["reward"].append(r)
        out["done"].append(done)
        out["trunc"].append(tr)
        if done:
            arg = resets.pop(0) if resets else -1
            o2, _ = env.reset(None if arg < 0 else int(arg))
            out["reset_arg"].append(arg)
            out["reset_obs"].append(o2.astype(np.int8))
        else:
            out["reset_arg"].append(-2)
            out["reset_obs"].append(np.zeros((R, C), np.int8))
        out["seed_after"].append(env.seed)
    return out


# shapes beyond the two headline ones (rows, columns, types): square, rows > columns,
# columns = 3 (boardConfig.py:50's literal 3 sends the vertical ids of row r to row r - 1),
# three types, fifteen types
EXTRA_SHAPES = [(7, 7, 4), (8, 8, 5), (10, 8, 5), (5, 3, 3), (12, 12, 7), (16, 3, 4), (6, 5, 15), (3, 3, 3)]
# rows < columns: BoardV2.__init__ works, legal_actions / apply_action raise IndexError
WIDE_SHAPES = [(8, 10, 5), (3, 5, 3)]


def gen_env(pool, shapes=None):
    rng = np.random.default_rng(2024)
    out = {}
    plan = [(20, 500), (20, 150), (7, 10**9), (12, 300)]
    # (tiny or many-type boards where most README runs hit a board without a legal move are left out)
    extra = [((R, C, T), 6, 30) for (R, C, T) in EXTRA_SHAPES if (R, C, T) not in ((3, 3, 3), (6, 5, 15))]
    for (R, C, T), n_runs, n_steps in shapes or [((9, 9, 6), 48, 60), ((16, 16, 8), 16, 45)] + extra:
        args = []
        for i in range(2 * n_runs):
            moves, goal = plan[i % len(plan)]
            resets = [int(rng.integers(1, 2**32 - 1)) if rng.random() < 0.5 else -1 for _ in range(8)]
            args.append((R, C, T, int(rng.integers(1, 2**32 - 1)), moves, goal, n_steps, resets))
        res = pool.map(_env_run, args, chunksize=2)
        keep = [i for i, r in enumerate(res) if r is not None][:n_runs]
        assert len(keep) == n_runs, (R, C, T, len(keep))
        args, res = [args[i] for i in keep], [res[i] for i in keep]
        tag = f"{R}x{C}x{T}"
        out[f"seed_{tag}"] = np.array([a[3] for a in args], dtype=np.uint32)
        out[f"moves_{tag}"] = np.array([a[4] for a in args], dtype=np.int32)
        out[f"goal_{tag}"] = np.array([a[5] for a in args], dtype=np.int64)
        out[f"init_{tag}"] = np.array([r["init"] for r in res])
        for k, dt in (("action", np.int32), ("obs", np.int8), ("reward", np.int32), ("done", np.uint8),
                      ("trunc", np.uint8), ("reset_arg", np.int64), ("reset_obs", np.int8),
                      ("seed_after", np.int64)):
            out[f"{k}_{tag}"] = np.array([r[k] for r in res], dtype=dt)
        out[f"action_space_{tag}"] = np.int64(R * (C - 1) + C * (R - 1))
    np.savez_compressed(os.path.join(OUT, "env.npz"), **out)


# ------------------------------------------------------------------------- steps
def _step_case(args):
    """(next board, reward, draws, n_actions) of one apply_action; draws -2 if the reference hangs
    (a cycling dead-board shuffle, boardv2.py:188-194)."""
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(3)
    try:
        return _step_case_body(args)
    except _Timeout:
        R, C = args[0], args[1]
        return np.zeros((R, C), np.int8), 0, -2, 0
    finally:
        signal.alarm(0)


def _step_case_body(args):
    R, C, T, board, seed, n_actions, action = args
    cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
    st = BoardV2(int(n_actions), cfg, np.array(board, dtype=np.int64))
    np.random.seed(999)  # apply_action must reseed; a terminal board must not touch the RNG
    before = np.random.get_state()
    nxt = st.apply_action(int(action))
    if st.is_terminal:
        after = np.random.get_state()
        assert after[2] == before[2] and np.array_equal(after[1], before[1])
        d = -1
    else:
        d = draws_since_seed(int(seed))
    return nxt.array.astype(np.int8), int(nxt.reward), d, int(nxt.n_actions)


def step_cases(R, C, T, rng, n_play=1500):
    cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
    H, V, B, M, TM = cfg.h_line, cfg.v_line, cfg.bomb, cfg.mega_token, cfg.type_mask
    specials = [H, V, B, M]
    cases = []
    # boards from seeded play
    play = []
    signal.signal(signal.SIGALRM, _alarm)
    for s in range(1, 120):
        c2 = BoardConfig(seed=s, rows=R, columns=C, types=T)
        b = BoardV2(20, c2)
        np.random.seed(s)
        signal.alarm(3)  # tiny boards: the reference can cycle forever in the dead-board shuffle
        try:
            for _ in range(6):
                play.append((b.array.copy(), s))
                la = b.legal_actions
                if not la:
                    break
                b = b.apply_action(int(np.random.choice(la)))
        except _Timeout:
            pass
        finally:
            signal.alarm(0)
    for i in range(n_play):
        board, s = play[rng.integers(0, len(play))]
        board = board.copy()
        kind = rng.random()
        if kind < 0.35:
            for _ in range(rng.integers(1, 4)):       # sprinkle pure specials
                board[rng.integers(0, R), rng.integers(0, C)] = specials[rng.integers(0, 4)]
        elif kind < 0.45:                              # typed specials (dataset.type_switch style)
            for _ in range(rng.integers(1, 3)):
                r, c = rng.integers(0, R), rng.integers(0, C)
                board[r, c] = min(127, int(board[r, c] & TM) + specials[rng.integers(0, 3)])
        if rng.random() < 0.6:
            la = legal_actions(cfg, board)
            a = int(la[rng.integers(0, len(la))]) if la else int(rng.integers(0, cfg.action_space))
        else:
            a = int(rng.integers(0, cfg.action_space))
        seed = int(rng.integers(1, 2**32))
        cases.append((board, seed, 20, a))
    # every combo pair at interior and edge positions
    for sa in specials + [1]:
        for sb in specials + [1]:
            for _ in range(14):
                board, _ = play[rng.integers(0, len(play))]
                board = board.copy()
                a = int(rng.integers(0, cfg.action_space))
                (r1, c1), (r2, c2) = cfg.decode(a)
                board[r1, c1], board[r2, c2] = sa, sb
                cases.append((board, int(rng.integers(1, 2**32)), 20, a))
    # bombs / lines at every edge cell (transposed-window quirk)
    for r in range(R):
        for c in (0, 1, C - 1):
            board, _ = play[rng.integers(0, len(play))]
            board = board.copy()
            board[r, c] = specials[rng.integers(0, 4)]
            cases.append((board, int(rng.integers(1, 2**32)), 20, int(rng.integers(0, cfg.action_space))))
    # large typed values (dataset type_switch produces up to M + STM)
    for _ in range(40):
        board, _ = play[rng.integers(0, len(play))]
        board = board.copy()
        for _ in range(3):
            board[rng.integers(0, R), rng.integers(0, C)] = int(rng.integers(TM + 1, 128))
        cases.append((board, int(rng.integers(1, 2**32)), 20, int(rng.integers(0, cfg.action_space))))
    # terminal boards (n_actions < 1) and n_actions == 1
    for na in (0, -3, 1):
        board, s = play[rng.integers(0, len(play))]
        cases.append((board.copy(), s, na, int(rng.integers(0, cfg.action_space))))
    return cases


def gen_steps(pool):
    rng = np.random.default_rng(4321)
    out = {}
    for (R, C, T), n in zip(SHAPES, (3000, 800)):
        cases = step_cases(R, C, T, rng, n)
        res = pool.map(_step_case, [(R, C, T, b, s, na, a) for (b, s, na, a) in cases], chunksize=16)
        tag = f"{R}x{C}x{T}"
        out[f"board_{tag}"] = np.array([c[0] for c in cases], dtype=np.int8)
        out[f"seed_{tag}"] = np.array([c[1] for c in cases], dtype=np.uint32)
        out[f"n_actions_{tag}"] = np.array([c[2] for c in cases], dtype=np.int32)
        out[f"action_{tag}"] = np.array([c[3] for c in cases], dtype=np.int32)
        out[f"next_{tag}"] = np.array([r[0] for r in res])
        out[f"reward_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"draws_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
    np.savez_compressed(os.path.join(OUT, "steps.npz"), **out)


# ------------------------------------------------------------------------- legal
def gen_legal():
    rng = np.random.default_rng(99)
    out = {}
    for (R, C, T) in SHAPES:
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        boards = []
        for s in range(1, 200):
            c2 = BoardConfig(seed=s, rows=R, columns=C, types=T)
            boards.append(BoardV2(20, c2).array.copy())
        for _ in range(300):
            b = rng.integers(1, T + 1, size=(R, C))
            if rng.random() < 0.5:
                for _ in range(rng.integers(1, 5)):
                    b[rng.integers(0, R), rng.integers(0, C)] = [cfg.h_line, cfg.v_line, cfg.bomb,
                                                                  cfg.mega_token, 0][rng.integers(0, 5)]
            boards.append(b)
        for m in range(2, T + 1):   # dead-ish patterned boards
            for a in range(1, 4):
                for bb in range(1, 4):
                    boards.append(np.fromfunction(lambda r, c: (a * r + bb * c) % m + 1, (R, C), dtype=np.int64))
        tag = f"{R}x{C}x{T}"
        out[f"boards_{tag}"] = np.array(boards, dtype=np.int8)
        out[f"legal_{tag}"] = np.array([legal_bits(cfg, b) for b in boards], dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "legal.npz"), **out)


# ----------------------------------------------------------------------- shuffle
def _shuffle_case(args):
    R, C, T, board, seed, action = args
    cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(3)
    try:
        nxt = BoardV2(20, cfg, np.array(board, dtype=np.int64)).apply_action(int(action))
        signal.alarm(0)
        return nxt.array.astype(np.int8), int(nxt.reward), draws_since_seed(int(seed)), 1
    except _Timeout:
        return np.zeros((R, C), np.int8), 0, 0, 0


def gen_shuffle(pool):
    """Boards whose post-swap cascade ends dead: exercise the shuffle loop (boardv2.py:188-194)."""
    out = {}
    for (R, C, T) in SHAPES:
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        cases = []
        for m in range(2, T + 1):
            for a in range(1, 5):
                for bb in range(1, 5):
                    board = np.fromfunction(lambda r, c: (a * r + bb * c) % m + 1, (R, C), dtype=np.int64)
                    # a swap of two cells inside one row keeps most of the pattern dead
                    for seed in (1, 2, 3, 17, 12345):
                        for act in (0, C - 1, 2 * C):
                            cases.append((board, seed, act))
        res = pool.map(_shuffle_case, [(R, C, T, b, s, a) for (b, s, a) in cases], chunksize=8)
        tag = f"{R}x{C}x{T}"
        out[f"board_{tag}"] = np.array([c[0] for c in cases], dtype=np.int8)
        out[f"seed_{tag}"] = np.array([c[1] for c in cases], dtype=np.uint32)
        out[f"action_{tag}"] = np.array([c[2] for c in cases], dtype=np.int32)
        out[f"next_{tag}"] = np.array([r[0] for r in res])
        out[f"reward_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"draws_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        out[f"terminates_{tag}"] = np.array([r[3] for r in res], dtype=np.uint8)
    np.savez_compressed(os.path.join(OUT, "shuffle.npz"), **out)


def _wide_case(args):
    R, C, T, seed = args
    cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
    b = BoardV2(20, cfg)
    d = draws_since_seed(int(seed))  # (before the calls below reseed and raise)
    errs = []
    for call in (lambda: b.legal_actions, lambda: b.apply_action(0)):
        try:
            call()
            errs.append("")
        except Exception as e:  # noqa: BLE001 -- the reference's own exception is the datum
            errs.append(type(e).__name__)
    return b.array.astype(np.int8), d, errs


def gen_shapes(pool):
    rng = np.random.default_rng(777)
    out = {}
    for (R, C, T) in EXTRA_SHAPES:
        tag = f"{R}x{C}x{T}"
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        seeds = np.concatenate([np.arange(1, 253), [2**31 - 2, 2**32 - 1, 123456789, 987654321]]).astype(np.uint64)
        res = pool.map(_init_one, [(R, C, T, s) for s in seeds])
        out[f"init_seeds_{tag}"] = seeds
        out[f"init_boards_{tag}"] = np.array([r[0] for r in res])
        out[f"init_draws_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        # legal sets: init boards, boards with specials / zeros, patterned (near-dead) boards
        boards = [r[0].astype(np.int64) for r in res[:120]]
        for _ in range(120):
            b = rng.integers(1, T + 1, size=(R, C))
            for _ in range(rng.integers(0, 4)):
                b[rng.integers(0, R), rng.integers(0, C)] = [cfg.h_line, cfg.v_line, cfg.bomb, cfg.mega_token,
                                                             0][rng.integers(0, 5)]
            boards.append(b)
        for m in range(2, T + 1):
            for a in range(1, 3):
                for bb in range(1, 3):
                    boards.append(np.fromfunction(lambda r, c: (a * r + bb * c) % m + 1, (R, C), dtype=np.int64))
        out[f"legal_boards_{tag}"] = np.array(boards, dtype=np.int8)
        out[f"legal_{tag}"] = np.array([legal_bits(cfg, b) for b in boards], dtype=np.uint8)
        # apply_action transitions (play, specials, typed values, combos, edges, illegal swaps, terminal)
        cases = step_cases(R, C, T, rng, 400)
        res = pool.map(_step_case, [(R, C, T, b, s, na, a) for (b, s, na, a) in cases], chunksize=16)
        out[f"step_board_{tag}"] = np.array([c[0] for c in cases], dtype=np.int8)
        out[f"step_seed_{tag}"] = np.array([c[1] for c in cases], dtype=np.uint32)
        out[f"step_n_actions_{tag}"] = np.array([c[2] for c in cases], dtype=np.int32)
        out[f"step_action_{tag}"] = np.array([c[3] for c in cases], dtype=np.int32)
        out[f"step_next_{tag}"] = np.array([r[0] for r in res])
        out[f"step_reward_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"step_draws_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        # seeded random_task episodes
        eseeds = np.arange(1, 81, dtype=np.uint64)
        res = pool.map(_episode, [(R, C, T, s, 20) for s in eseeds], chunksize=2)
        keep = [i for i, r in enumerate(res) if r is not None][:64]  # (drop seeds where the reference hangs)
        eseeds, res = eseeds[keep], [res[i] for i in keep]
        out[f"ep_seeds_{tag}"] = eseeds
        out[f"ep_init_{tag}"] = np.array([r[0] for r in res])
        out[f"ep_actions_{tag}"] = np.array([r[1] for r in res], dtype=np.int16)
        out[f"ep_rewards_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        out[f"ep_draws_{tag}"] = np.array([r[3] for r in res], dtype=np.int16)
        out[f"ep_final_{tag}"] = np.array([r[4][-1] for r in res])
    for (R, C, T) in WIDE_SHAPES:
        tag = f"{R}x{C}x{T}"
        seeds = np.arange(1, 129, dtype=np.uint64)
        res = pool.map(_wide_case, [(R, C, T, s) for s in seeds])
        out[f"wide_seeds_{tag}"] = seeds
        out[f"wide_boards_{tag}"] = np.array([r[0] for r in res])
        out[f"wide_draws_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"wide_errors_{tag}"] = np.array(sorted({e for r in res for e in r[2]}))
    np.savez_compressed(os.path.join(OUT, "shapes.npz"), **out)


# types = 2 (BoardConfig(types=2): TM 3, H 4, V 8, B 12, M 16). The reference resets every size,
# but on boards from about 7x7 up a refill of two colours almost always leaves a new match, so
# its cascade (boardv2.py:138-202) does not return (and a 16x16x2 reset can take millions of draws):
# steps and episodes are recorded for the small
# boards where it does, resets and legal sets for the large ones, plus how many first moves of
# seeded play return within 3 s there.
TYPES2_PLAY = [(5, 5, 2), (4, 4, 2), (6, 6, 2)]
TYPES2_RESET = [(9, 9, 2), (12, 7, 2)]


def _first_move_returns(args):
    R, C, T, seed = args
    signal.signal(signal.SIGALRM, _alarm)
    signal.alarm(3)
    try:
        cfg = BoardConfig(seed=int(seed), rows=R, columns=C, types=T)
        b = BoardV2(20, cfg)
        np.random.seed(cfg.seed)
        b.apply_action(int(np.random.choice(b.legal_actions)))
        return 1
    except _Timeout:
        return 0
    finally:
        signal.alarm(0)


def gen_types2(pool):
    rng = np.random.default_rng(2222)
    out = {}
    for (R, C, T) in TYPES2_PLAY + TYPES2_RESET:
        tag = f"{R}x{C}x{T}"
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        seeds = np.concatenate([np.arange(1, 125), [2**31 - 2, 2**32 - 1, 123456789, 987654321]]).astype(np.uint64)
        res = pool.map(_init_one, [(R, C, T, s) for s in seeds])
        out[f"init_seeds_{tag}"] = seeds
        out[f"init_boards_{tag}"] = np.array([r[0] for r in res])
        out[f"init_draws_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        boards = [r[0].astype(np.int64) for r in res[:60]]
        for _ in range(60):
            b = rng.integers(1, T + 1, size=(R, C))
            for _ in range(rng.integers(0, 4)):
                b[rng.integers(0, R), rng.integers(0, C)] = [cfg.h_line, cfg.v_line, cfg.bomb, cfg.mega_token,
                                                             0][rng.integers(0, 5)]
            boards.append(b)
        out[f"legal_boards_{tag}"] = np.array(boards, dtype=np.int8)
        out[f"legal_{tag}"] = np.array([legal_bits(cfg, b) for b in boards], dtype=np.uint8)
        if (R, C, T) in TYPES2_RESET:
            ret = pool.map(_first_move_returns, [(R, C, T, s) for s in range(1, 17)])
            out[f"first_move_returns_{tag}"] = np.array(ret, dtype=np.uint8)
            continue
        cases = step_cases(R, C, T, rng, 300)
        res = pool.map(_step_case, [(R, C, T, b, s, na, a) for (b, s, na, a) in cases], chunksize=8)
        out[f"step_board_{tag}"] = np.array([c[0] for c in cases], dtype=np.int8)
        out[f"step_seed_{tag}"] = np.array([c[1] for c in cases], dtype=np.uint32)
        out[f"step_n_actions_{tag}"] = np.array([c[2] for c in cases], dtype=np.int32)
        out[f"step_action_{tag}"] = np.array([c[3] for c in cases], dtype=np.int32)
        out[f"step_next_{tag}"] = np.array([r[0] for r in res])
        out[f"step_reward_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"step_draws_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        eseeds = np.arange(1, 81, dtype=np.uint64)
        res = pool.map(_episode, [(R, C, T, s, 20) for s in eseeds], chunksize=2)
        keep = [i for i, r in enumerate(res) if r is not None][:48]
        eseeds, res = eseeds[keep], [res[i] for i in keep]
        out[f"ep_seeds_{tag}"] = eseeds
        out[f"ep_init_{tag}"] = np.array([r[0] for r in res])
        out[f"ep_actions_{tag}"] = np.array([r[1] for r in res], dtype=np.int16)
        out[f"ep_rewards_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        out[f"ep_draws_{tag}"] = np.array([r[3] for r in res], dtype=np.int16)
        out[f"ep_final_{tag}"] = np.array([r[4][-1] for r in res])
    np.savez_compressed(os.path.join(OUT, "types2.npz"), **out)


# Boards past the 16 x 16 frame and tile alphabets past 15 types (BoardConfig accepts any rows /
# columns / types, boardConfig.py:26-43; main.py:100-102 takes them from the command line). With
# types >= 16 (5 token bits) every special token is >= 32 and the clip of boardv2.py:163 turns it
# into 32.
BIG_SHAPES = [(20, 20, 6), (24, 17, 5), (32, 32, 8), (17, 17, 3), (9, 9, 20), (12, 12, 31)]


def gen_big(pool):
    rng = np.random.default_rng(4242)
    out = {}
    for (R, C, T) in BIG_SHAPES:
        tag = f"{R}x{C}x{T}"
        cfg = BoardConfig(seed=1, rows=R, columns=C, types=T)
        seeds = np.concatenate([np.arange(1, 61), [2**31 - 2, 2**32 - 1, 123456789, 987654321]]).astype(np.uint64)
        res = pool.map(_init_one, [(R, C, T, s) for s in seeds])
        out[f"init_seeds_{tag}"] = seeds
        out[f"init_boards_{tag}"] = np.array([r[0] for r in res])
        out[f"init_draws_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        boards = [r[0].astype(np.int64) for r in res[:40]]
        for _ in range(40):
            b = rng.integers(1, T + 1, size=(R, C))
            for _ in range(rng.integers(0, 6)):
                b[rng.integers(0, R), rng.integers(0, C)] = [cfg.h_line, cfg.v_line, cfg.bomb, cfg.mega_token,
                                                             0][rng.integers(0, 5)]
            boards.append(np.clip(b, 0, 127))
        for m in range(2, min(T, 6) + 1):
            boards.append(np.fromfunction(lambda r, c: (r + 2 * c) % m + 1, (R, C), dtype=np.int64))
        out[f"legal_boards_{tag}"] = np.array(boards, dtype=np.int8)
        out[f"legal_{tag}"] = np.array([legal_bits(cfg, b) for b in boards], dtype=np.uint8)
        cases = [c for c in step_cases(R, C, T, rng, 200) if np.asarray(c[0]).max() <= 127]
        res = pool.map(_step_case, [(R, C, T, b, s, na, a) for (b, s, na, a) in cases], chunksize=8)
        out[f"step_board_{tag}"] = np.array([c[0] for c in cases], dtype=np.int8)
        out[f"step_seed_{tag}"] = np.array([c[1] for c in cases], dtype=np.uint32)
        out[f"step_n_actions_{tag}"] = np.array([c[2] for c in cases], dtype=np.int32)
        out[f"step_action_{tag}"] = np.array([c[3] for c in cases], dtype=np.int32)
        out[f"step_next_{tag}"] = np.array([r[0] for r in res])
        out[f"step_reward_{tag}"] = np.array([r[1] for r in res], dtype=np.int32)
        out[f"step_draws_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        eseeds = np.arange(1, 41, dtype=np.uint64)
        res = pool.map(_episode, [(R, C, T, s, 20) for s in eseeds], chunksize=2)
        keep = [i for i, r in enumerate(res) if r is not None][:32]
        eseeds, res = eseeds[keep], [res[i] for i in keep]
        out[f"ep_seeds_{tag}"] = eseeds
        out[f"ep_init_{tag}"] = np.array([r[0] for r in res])
        out[f"ep_actions_{tag}"] = np.array([r[1] for r in res], dtype=np.int16)
        out[f"ep_rewards_{tag}"] = np.array([r[2] for r in res], dtype=np.int32)
        out[f"ep_draws_{tag}"] = np.array([r[3] for r in res], dtype=np.int16)
        out[f"ep_final_{tag}"] = np.array([r[4][-1] for r in res])
        print("  ", tag, len(cases), "steps", len(keep), "episodes", flush=True)
    np.savez_compressed(os.path.join(OUT, "big.npz"), **out)


def main():
    which = sys.argv[1:] or ["prng", "matches", "legal", "init", "steps", "episodes", "shuffle", "env", "shapes",
                             "types2", "big"]
    with Pool(8) as pool:
        for w in which:
            print("generating", w, flush=True)
            if w == "prng":
                gen_prng()
            elif w == "matches":
                gen_matches()
            elif w == "legal":
                gen_legal()
            elif w == "init":
                gen_init(pool)
            elif w == "steps":
                gen_steps(pool)
            elif w == "episodes":
                gen_episodes(pool)
            elif w == "shuffle":
                gen_shuffle(pool)
            elif w == "env":
                gen_env(pool)
            elif w == "shapes":
                gen_shapes(pool)
            elif w == "types2":
                gen_types2(pool)
            elif w == "big":
                gen_big(pool)


if __name__ == "__main__":
    main()
