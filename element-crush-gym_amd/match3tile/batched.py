"""BatchedMatch3Env: n independent Match3Env boards resident on one MI355X.

The state of every board (int8 grid, seed, cached MT19937 word, score, moves,
pre-drawn seeded random action) lives in HBM; one ``step()`` is one launch of
the fused step kernel over all boards (plus a tiny overflow-fixup launch and,
with autoreset, the reset launch for finished boards). Nothing is copied to
the host unless asked for.

Semantics per board are exactly Match3Env.step (env.py:48-56, restated in
env.py here) over BoardV2.apply_action; with ``actions=None`` every board
plays its seeded ``random_action()``: legal[randint(0, len(legal))] drawn from
the board's MT19937 stream where the previous apply_action left it, i.e. the
reference's samplerTasks.random_task episode (samplerTasks.py:9-14).

Autoreset (gymnasium vector-env style, same-step): a board that finishes is
re-initialised in the same step with seed += seed_stride; ``done`` and
``reward`` still report the finished step, the observation is the new board.

Multi-GPU: one process per GPU, each owning its own boards (no data exchange
during a step). ``init_comm()`` + ``gather()`` do one RCCL all-gather of the
packed (reward << 2 | truncated << 1 | done) words over xGMI.

Checkpoint / resume: ``save(path)`` writes every board's state (the
reference's BoardV2 state (array, cfg.seed, n_actions, _reward) plus
Match3Env's score / moves_taken and the pre-drawn next action) to one .npz;
``BatchedMatch3Env.load(path)`` builds an env that steps on exactly as the
saved one would have (m3_env_set, include/m3.h).
"""
from __future__ import annotations

import ctypes

import numpy as np

from . import _native
from ._native import check, lib, ptr


class BatchedMatch3Env:
    def __init__(self, n: int, rows: int = 9, columns: int = 9, types: int = 6, num_moves: int = 20,
                 env_goal: int = 500, device: int = 0, seeds=None, seed_base: int = 1,
                 autoreset: bool = True, seed_stride: int = None, shards: int = None):
        self.n = int(n)
        self.rows, self.columns, self.types = rows, columns, types
        self.num_moves, self.env_goal = num_moves, env_goal
        self.ctx = _native.Context(rows, columns, types, device)
        self.N, self.A, self.words = self.ctx.N, self.ctx.A, self.ctx.words
        h = ctypes.c_void_p()
        check(lib().m3_env_create(self.ctx.handle, self.n, num_moves, env_goal, ctypes.byref(h)))
        self.handle = h
        stride = self.n if seed_stride is None else int(seed_stride)
        self.set_autoreset(autoreset, stride)
        if shards is not None:
            self.set_shards(shards)
        self.nranks = 1
        if seeds is not False:  # (load() fills the state instead)
            self.reset(seeds=seeds, seed_base=seed_base)

    # ---- lifecycle -------------------------------------------------------------------
    def close(self):
        if getattr(self, "handle", None):
            lib().m3_env_destroy(self.handle)
            self.handle = None
        if getattr(self, "ctx", None):
            self.ctx.close()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def set_autoreset(self, enabled: bool, seed_stride: int):
        check(lib().m3_env_set_autoreset(self.handle, int(bool(enabled)), int(seed_stride) & 0xFFFFFFFF))
        self.autoreset, self.seed_stride = bool(enabled), int(seed_stride) & 0xFFFFFFFF

    def reset(self, seeds=None, seed_base: int = 1):
        """Match3Env.reset for every board; seeds default to seed_base + i."""
        s = None if seeds is None else np.ascontiguousarray(seeds, dtype=np.uint32)
        if s is not None and len(s) != self.n:
            raise ValueError("need one seed per board")
        check(lib().m3_env_reset(self.handle, ptr(s), int(seed_base) & 0xFFFFFFFF))
        return self

    # ---- stepping --------------------------------------------------------------------
    def step(self, actions=None, copy: bool = False):
        """One env step on every board. actions: int array [n] or None (seeded random)."""
        a = None
        if actions is not None:
            a = np.ascontiguousarray(actions, dtype=np.int32)
            if a.shape != (self.n,):
                raise ValueError("need one action per board")
        check(lib().m3_env_step(self.handle, ptr(a)))
        if copy:
            return self.observations(), self.rewards(), self.dones(), self.truncateds(), {"flags": self.flags()}
        return None

    def step_device(self, device_actions_ptr=None):
        check(lib().m3_env_step_device(self.handle, device_actions_ptr))

    def synchronize(self):
        check(lib().m3_env_synchronize(self.handle))

    def set_shards(self, nshards: int):
        """Number of independent board shards / HIP streams (1..8); results do not depend on it."""
        check(lib().m3_env_set_shards(self.handle, int(nshards)))

    def enable_timing(self, capacity: int):
        """Record HIP events around the next `capacity` step-kernel launches."""
        check(lib().m3_env_timing(self.handle, int(capacity)))

    def kernel_ms(self, step_kernel_only: bool = False) -> np.ndarray:
        """Per-launch durations (ms) of each shard's step pipeline (k_env_step .. k_env_fix) since
        enable_timing(); step_kernel_only: of k_env_step alone."""
        cap = 1 << 16
        out = np.empty(cap, np.float32)
        n = ctypes.c_int(0)
        fn = lib().m3_env_step_kernel_ms if step_kernel_only else lib().m3_env_kernel_ms
        check(fn(self.handle, ptr(out), cap, ctypes.byref(n)))
        return out[: n.value].copy()

    def stats(self) -> dict:
        """Cumulative counters since reset (exact-fallback recomputes, autoresets, shards)."""
        out = np.zeros(4, np.uint64)
        check(lib().m3_env_stats(self.handle, ptr(out)))
        return dict(step_recomputes=int(out[0]), reset_recomputes=int(out[1]), autoresets=int(out[2]),
                    shards=int(out[3]))

    # ---- copy-outs ------------------------------------------------------------------
    def _get(self, what, dtype, shape):
        out = np.empty(shape, dtype=dtype)
        check(lib().m3_env_get(self.handle, what, ptr(out)))
        return out

    def observations(self):
        return self._get(_native.ENV_BOARDS, np.int8, (self.n, self.rows, self.columns))

    def rewards(self):
        return self._get(_native.ENV_REWARD, np.int32, (self.n,))

    def dones(self):
        return self._get(_native.ENV_DONE, np.uint8, (self.n,)).astype(bool)

    def truncateds(self):
        return self._get(_native.ENV_TRUNCATED, np.uint8, (self.n,)).astype(bool)

    def scores(self):
        return self._get(_native.ENV_SCORE, np.int32, (self.n,))

    def moves(self):
        return self._get(_native.ENV_MOVES, np.int32, (self.n,))

    def flags(self):
        return self._get(_native.ENV_FLAGS, np.uint32, (self.n,))

    def next_actions(self):
        return self._get(_native.ENV_NEXT_ACTION, np.int32, (self.n,))

    def legal_bits(self):
        return self._get(_native.ENV_LEGAL, np.uint32, (self.n, self.words))

    def seeds(self):
        return self._get(_native.ENV_SEEDS, np.uint32, (self.n,))

    def draws(self):
        return self._get(_native.ENV_DRAWS, np.uint32, (self.n,))

    # ---- checkpoint / resume ------------------------------------------------------------
    _STATE = (("boards", _native.ENV_BOARDS, np.int8), ("seeds", _native.ENV_SEEDS, np.uint32),
              ("score", _native.ENV_SCORE, np.int32), ("moves", _native.ENV_MOVES, np.int32),
              ("next_action", _native.ENV_NEXT_ACTION, np.int32), ("reward", _native.ENV_REWARD, np.int32),
              ("done", _native.ENV_DONE, np.uint8), ("truncated", _native.ENV_TRUNCATED, np.uint8),
              ("flags", _native.ENV_FLAGS, np.uint32), ("draws", _native.ENV_DRAWS, np.uint32))

    def state_dict(self) -> dict:
        """Every board's resumable state (host copies) + the env's configuration."""
        shapes = {"boards": (self.n, self.rows, self.columns)}
        st = {k: self._get(w, dt, shapes.get(k, (self.n,))) for k, w, dt in self._STATE}
        st["config"] = np.array([self.n, self.rows, self.columns, self.types, self.num_moves, self.env_goal,
                                 int(self.autoreset), self.seed_stride], dtype=np.int64)
        return st

    def load_state_dict(self, st: dict):
        cfg = [int(x) for x in st["config"]]
        if cfg[:6] != [self.n, self.rows, self.columns, self.types, self.num_moves, self.env_goal]:
            raise ValueError(f"checkpoint is for env {cfg[:6]}, not "
                             f"{[self.n, self.rows, self.columns, self.types, self.num_moves, self.env_goal]}")
        self.set_autoreset(bool(cfg[6]), cfg[7])
        for k, w, dt in self._STATE:
            a = np.ascontiguousarray(st[k], dtype=dt)
            check(lib().m3_env_set(self.handle, w, ptr(a)))
        return self

    def save(self, path):
        np.savez(path, **self.state_dict())

    @classmethod
    def load(cls, path, device: int = 0, shards: int = None) -> "BatchedMatch3Env":
        with np.load(path, allow_pickle=False) as f:
            st = {k: f[k] for k in f.files}
        n, rows, columns, types, num_moves, env_goal, autoreset, stride = (int(x) for x in st["config"])
        env = cls(n, rows, columns, types, num_moves=num_moves, env_goal=env_goal, device=device, seeds=False,
                  autoreset=bool(autoreset), seed_stride=stride, shards=shards)
        return env.load_state_dict(st)

    def device_ptr(self, what) -> int:
        p = ctypes.c_void_p()
        check(lib().m3_env_device_ptr(self.handle, what, ctypes.byref(p)))
        return p.value

    # ---- multi-GPU ----------------------------------------------------------------------
    @staticmethod
    def comm_unique_id() -> bytes:
        buf = (ctypes.c_uint8 * 128)()
        check(lib().m3_comm_unique_id(buf))
        return bytes(buf)

    def init_comm(self, unique_id: bytes, nranks: int, rank: int):
        buf = (ctypes.c_uint8 * 128).from_buffer_copy(unique_id)
        check(lib().m3_env_comm_init(self.handle, buf, int(nranks), int(rank)))
        self.nranks = nranks

    def comm_size(self) -> int:
        """Ranks of the env's RCCL communicator as RCCL reports them (1 before init_comm)."""
        n = ctypes.c_int(0)
        check(lib().m3_env_comm_size(self.handle, ctypes.byref(n)))
        return n.value

    def gather(self, to_host: bool = False):
        """RCCL all-gather of packed reward/truncated/done of every board of every rank."""
        out = np.empty(self.nranks * self.n, np.int32) if to_host else None
        check(lib().m3_env_gather(self.handle, ptr(out)))
        return out

    def gather_device(self, device_out_ptr=None):
        """Enqueue the all-gather into a caller-owned device buffer int32[nranks][n] (None: the env's own,
        ENV_GATHERED); valid once the env's context stream gets there (synchronize() or any copy-out)."""
        check(lib().m3_env_gather_device(self.handle, device_out_ptr))

    def gathered(self):
        """Host copy of the env's gather buffer [nranks * n] (ordered after every enqueued gather)."""
        return self._get(_native.ENV_GATHERED, np.int32, (self.nranks * self.n,))

    def debug_stall(self, usec: int):
        """Test hook: idle the context stream (where gathers run) for ~usec."""
        check(lib().m3_env_debug_stall(self.handle, int(usec)))
