"""ctypes wrapper around the C oracle (TEST INFRASTRUCTURE ONLY).

Only tests/, ``__graft_entry__.smoke()`` and ``bench.py``'s ``cpu_baseline``
leg may import this module. It is the checker for the HIP path, never the
thing measured or shipped: the product package (``element-crush-gym_amd``)
does not import it.

Parity of the oracle itself is pinned by ``tests/golden/*.npz``, generated
from the real reference (``tests/golden/gen_golden.py``).
"""
from __future__ import annotations

import ctypes
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_LIB_PATH = os.path.join(_HERE, "build", "liboracle.so")
_lib = None

FLAG_TERMINAL = 0x01
FLAG_BAD_ACTION = 0x02
FLAG_SHUFFLE_CAP = 0x04
FLAG_NO_LEGAL = 0x08
FLAG_SHUFFLED = 0x10


class MT(ctypes.Structure):
    _fields_ = [("key", ctypes.c_uint32 * 624), ("pos", ctypes.c_int), ("draws", ctypes.c_int64)]


class Cfg(ctypes.Structure):
    _fields_ = [(n, ctypes.c_int) for n in ("R", "C", "T", "TM", "STM", "H", "V", "B", "M", "A")]


def build() -> str:
    subprocess.run(["make", "-s", "-C", _HERE], check=True)
    return _LIB_PATH


def lib():
    global _lib
    if _lib is None:
        srcs = [os.path.join(_HERE, f) for f in ("m3_oracle.c", "m3_oracle.h")]
        if not os.path.exists(_LIB_PATH) or (
                all(os.path.exists(s) for s in srcs)
                and os.path.getmtime(_LIB_PATH) < max(os.path.getmtime(s) for s in srcs)):
            build()
        L = ctypes.CDLL(_LIB_PATH)
        P = ctypes.POINTER
        i32p, u8p, u32p, i64p = P(ctypes.c_int32), P(ctypes.c_uint8), P(ctypes.c_uint32), P(ctypes.c_int64)
        L.m3o_mt_seed.argtypes = [P(MT), ctypes.c_uint32]
        L.m3o_mt_next32.argtypes = [P(MT)]
        L.m3o_mt_next32.restype = ctypes.c_uint32
        L.m3o_randint.argtypes = [P(MT), ctypes.c_int64, ctypes.c_int64]
        L.m3o_randint.restype = ctypes.c_int64
        L.m3o_random_interval.argtypes = [P(MT), ctypes.c_uint64]
        L.m3o_random_interval.restype = ctypes.c_uint64
        L.m3o_cfg_init.argtypes = [P(Cfg), ctypes.c_int, ctypes.c_int, ctypes.c_int]
        L.m3o_decode.argtypes = [P(Cfg), ctypes.c_int] + [P(ctypes.c_int)] * 4
        L.m3o_encode.argtypes = [P(Cfg)] + [ctypes.c_int] * 4
        L.m3o_encode.restype = ctypes.c_int
        L.m3o_get_matches.argtypes = [P(Cfg), i32p, u8p]
        L.m3o_get_matches.restype = ctypes.c_int
        L.m3o_matches_and_spawn.argtypes = [P(Cfg), i32p, u8p, i32p]
        L.m3o_matches_and_spawn.restype = ctypes.c_int
        L.m3o_legal_actions.argtypes = [P(Cfg), i32p, i32p]
        L.m3o_legal_actions.restype = ctypes.c_int
        L.m3o_init_board.argtypes = [P(Cfg), ctypes.c_uint32, i32p, P(MT)]
        L.m3o_init_board.restype = ctypes.c_int64
        L.m3o_apply_action.argtypes = [P(Cfg), ctypes.c_uint32, ctypes.c_int, i32p, ctypes.c_int,
                                       i32p, P(MT), P(ctypes.c_int), ctypes.c_int]
        L.m3o_apply_action.restype = ctypes.c_int64
        L.m3o_set_episode_shuffle_cap.argtypes = [ctypes.c_int]
        L.m3o_random_episode.argtypes = [P(Cfg), ctypes.c_uint32, ctypes.c_int, ctypes.c_int,
                                         i32p, i32p, i32p, u8p, i32p, P(ctypes.c_int)]
        L.m3o_random_episode.restype = ctypes.c_int
        L.m3o_run_episodes.argtypes = [P(Cfg), ctypes.c_int64, u32p, ctypes.c_int, ctypes.c_int,
                                       ctypes.c_int, i64p]
        L.m3o_run_episodes.restype = ctypes.c_int64
        L.m3o_batch_episodes.argtypes = [P(Cfg), ctypes.c_int64, u32p, ctypes.c_int, ctypes.c_int, ctypes.c_int,
                                         i32p, i32p, i32p, u8p, i32p, i32p, i32p]
        L.m3o_batch_episodes.restype = None
        L.m3o_batch_rollouts.argtypes = [P(Cfg), ctypes.c_int64, i32p, u32p, i32p, u32p, ctypes.c_int,
                                         i32p, i32p, i64p, i32p, i32p]
        L.m3o_batch_rollouts.restype = None
        _lib = L
    return _lib


def _p(a, ct):
    return a.ctypes.data_as(ctypes.POINTER(ct))


class Oracle:
    """Python face of the C oracle for one board shape."""

    def __init__(self, rows=9, columns=9, types=6, shuffle_cap=1024, episode_shuffle_cap=1 << 20):
        """shuffle_cap: apply_action's (the GPU's 1024); episode_shuffle_cap: the episode / rollout
        drivers' (default: effectively none, like the reference)."""
        self.episode_shuffle_cap = episode_shuffle_cap
        self.cfg = Cfg()
        lib().m3o_cfg_init(ctypes.byref(self.cfg), rows, columns, types)
        self.R, self.C, self.T = rows, columns, types
        self.A = self.cfg.A
        self.shuffle_cap = shuffle_cap

    # --- PRNG -------------------------------------------------------------------
    def mt_raw(self, seed: int, n: int) -> np.ndarray:
        mt = MT()
        lib().m3o_mt_seed(ctypes.byref(mt), seed & 0xFFFFFFFF)
        return np.array([lib().m3o_mt_next32(ctypes.byref(mt)) for _ in range(n)], dtype=np.uint32)

    # --- rule kernels -------------------------------------------------------------
    def decode(self, action):
        v = [ctypes.c_int() for _ in range(4)]
        lib().m3o_decode(ctypes.byref(self.cfg), int(action), *[ctypes.byref(x) for x in v])
        return (v[0].value, v[1].value), (v[2].value, v[3].value)

    def get_matches(self, tb):
        tb = np.ascontiguousarray(tb, dtype=np.int32)
        mask = np.zeros(tb.shape, dtype=np.uint8)
        spawn = np.zeros(tb.shape, dtype=np.int32)
        n = lib().m3o_matches_and_spawn(ctypes.byref(self.cfg), _p(tb, ctypes.c_int32),
                                        _p(mask, ctypes.c_uint8), _p(spawn, ctypes.c_int32))
        return mask.astype(bool), spawn, n

    def legal_actions(self, board):
        board = np.ascontiguousarray(board, dtype=np.int32)
        out = np.zeros(self.A, dtype=np.int32)
        n = lib().m3o_legal_actions(ctypes.byref(self.cfg), _p(board, ctypes.c_int32), _p(out, ctypes.c_int32))
        return [int(x) for x in out[:n]]

    def init_board(self, seed):
        board = np.zeros((self.R, self.C), dtype=np.int32)
        mt = MT()
        d = lib().m3o_init_board(ctypes.byref(self.cfg), seed & 0xFFFFFFFF, _p(board, ctypes.c_int32),
                                 ctypes.byref(mt))
        return board, int(d)

    def apply_action(self, board, seed, action, n_actions=20):
        """Returns (next_board, reward, draws_since_last_reseed, flags)."""
        board = np.ascontiguousarray(board, dtype=np.int32)
        out = np.zeros_like(board)
        mt = MT()
        flags = ctypes.c_int()
        r = lib().m3o_apply_action(ctypes.byref(self.cfg), seed & 0xFFFFFFFF, int(n_actions),
                                   _p(board, ctypes.c_int32), int(action), _p(out, ctypes.c_int32),
                                   ctypes.byref(mt), ctypes.byref(flags), self.shuffle_cap)
        return out, int(r), int(mt.draws), int(flags.value)

    def random_episode(self, seed, num_moves=20, env_goal=2**31 - 1):
        acts = np.zeros(num_moves, np.int32)
        rews = np.zeros(num_moves, np.int32)
        drw = np.zeros(num_moves, np.int32)
        done = np.zeros(num_moves, np.uint8)
        fb = np.zeros((self.R, self.C), np.int32)
        flags = ctypes.c_int()
        lib().m3o_set_episode_shuffle_cap(self.episode_shuffle_cap)
        n = lib().m3o_random_episode(ctypes.byref(self.cfg), seed & 0xFFFFFFFF, num_moves, env_goal,
                                     _p(acts, ctypes.c_int32), _p(rews, ctypes.c_int32), _p(drw, ctypes.c_int32),
                                     _p(done, ctypes.c_uint8), _p(fb, ctypes.c_int32), ctypes.byref(flags))
        return dict(n=n, actions=acts[:n], rewards=rews[:n], draws=drw[:n], done=done[:n],
                    final=fb, flags=int(flags.value))

    def batch_episodes(self, seeds, num_moves=20, env_goal=2**31 - 1, threads=None):
        """Seeded random episodes for many boards at once (OpenMP over boards)."""
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        n = len(seeds)
        threads = threads or min(16, os.cpu_count() or 1)
        acts = np.zeros((n, num_moves), np.int32)
        rews = np.zeros((n, num_moves), np.int32)
        drw = np.zeros((n, num_moves), np.int32)
        done = np.zeros((n, num_moves), np.uint8)
        final = np.zeros((n, self.R * self.C), np.int32)
        moves = np.zeros(n, np.int32)
        flags = np.zeros(n, np.int32)
        lib().m3o_set_episode_shuffle_cap(self.episode_shuffle_cap)
        lib().m3o_batch_episodes(ctypes.byref(self.cfg), n, _p(seeds, ctypes.c_uint32), num_moves, env_goal, threads,
                                 _p(acts, ctypes.c_int32), _p(rews, ctypes.c_int32), _p(drw, ctypes.c_int32),
                                 _p(done, ctypes.c_uint8), _p(final, ctypes.c_int32), _p(moves, ctypes.c_int32),
                                 _p(flags, ctypes.c_int32))
        return dict(actions=acts, rewards=rews, draws=drw, done=done, final=final, moves=moves, flags=flags)

    def rollouts(self, boards, seeds, n_actions, rollout_seeds, threads=None):
        """MCTS.rollout (mctslib/standard/mcts.py:14-19) for many states at once (OpenMP)."""
        boards = np.ascontiguousarray(boards, dtype=np.int32).reshape(-1, self.R * self.C)
        n = boards.shape[0]
        seeds = np.ascontiguousarray(np.broadcast_to(seeds, (n,)), dtype=np.uint32)
        n_actions = np.ascontiguousarray(np.broadcast_to(n_actions, (n,)), dtype=np.int32)
        rollout_seeds = np.ascontiguousarray(np.broadcast_to(rollout_seeds, (n,)), dtype=np.uint32)
        threads = threads or min(16, os.cpu_count() or 1)
        gain = np.zeros(n, np.int32)
        steps = np.zeros(n, np.int32)
        draws = np.zeros(n, np.int64)
        flags = np.zeros(n, np.int32)
        final = np.zeros((n, self.R * self.C), np.int32)
        lib().m3o_set_episode_shuffle_cap(self.episode_shuffle_cap)
        lib().m3o_batch_rollouts(ctypes.byref(self.cfg), n, _p(boards, ctypes.c_int32), _p(seeds, ctypes.c_uint32),
                                 _p(n_actions, ctypes.c_int32), _p(rollout_seeds, ctypes.c_uint32), threads,
                                 _p(gain, ctypes.c_int32), _p(steps, ctypes.c_int32), _p(draws, ctypes.c_int64),
                                 _p(flags, ctypes.c_int32), _p(final, ctypes.c_int32))
        return dict(gain=gain, steps=steps, draws=draws, flags=flags, final=final)

    def run_episodes(self, seeds, num_moves=20, env_goal=2**31 - 1, threads=1):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        tot = np.zeros(len(seeds), dtype=np.int64)
        lib().m3o_set_episode_shuffle_cap(self.episode_shuffle_cap)
        steps = lib().m3o_run_episodes(ctypes.byref(self.cfg), len(seeds), _p(seeds, ctypes.c_uint32),
                                       num_moves, env_goal, threads, _p(tot, ctypes.c_int64))
        return int(steps), tot
