"""ctypes binding of libm3.so (include/m3.h) -- the only way this package computes.

There is no CPU fallback: if the library is missing, or no gfx950 device is
visible, every compute entry point raises ``M3Error``. (The CPU restatement in
``oracle/`` is test infrastructure and is never imported here.)
"""
from __future__ import annotations

import ctypes
import os
import threading

import numpy as np

_PKG_ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LIB_PATH = os.environ.get("M3_LIB", os.path.join(_PKG_ROOT, "build", "libm3.so"))

M3_OK = 0
ERR_NAMES = {-1: "M3_ERR_INVALID", -2: "M3_ERR_UNSUPPORTED", -3: "M3_ERR_HIP", -4: "M3_ERR_RCCL",
             -5: "M3_ERR_NO_DEVICE", -6: "M3_ERR_STATE", -7: "M3_ERR_CAP"}

FLAG_TERMINAL = 0x01
FLAG_BAD_ACTION = 0x02
FLAG_SHUFFLE_CAP = 0x04
FLAG_NO_LEGAL = 0x08
FLAG_SHUFFLED = 0x10
FLAG_CASCADE_CAP = 0x100
FLAG_RESET_CAP = 0x200

ENV_BOARDS, ENV_REWARD, ENV_DONE, ENV_TRUNCATED, ENV_SCORE, ENV_MOVES, ENV_FLAGS, ENV_NEXT_ACTION, \
    ENV_LEGAL, ENV_SEEDS, ENV_DRAWS, ENV_GATHERED = range(12)

# every symbol declared in include/m3.h
EXPORTS = [
    "m3_abi_version", "m3_last_error", "m3_device_count", "m3_supported", "m3_action_space",
    "m3_ctx_create", "m3_ctx_destroy", "m3_ctx_synchronize", "m3_dev_alloc", "m3_dev_free", "m3_dev_copy",
    "m3_init_boards", "m3_init_boards_ex", "m3_apply_actions", "m3_legal_actions", "m3_rollouts", "m3_rollouts_device",
    "m3_env_create", "m3_env_destroy", "m3_env_reset", "m3_env_set_shards", "m3_env_synchronize",
    "m3_env_set_autoreset", "m3_env_step",
    "m3_env_step_device", "m3_env_get", "m3_env_set", "m3_env_device_ptr",
    "m3_comm_unique_id", "m3_env_comm_init", "m3_env_comm_size", "m3_env_gather", "m3_env_gather_device", "m3_env_debug_stall",
    "m3_env_stats", "m3_env_timing",
    "m3_env_kernel_ms", "m3_env_step_kernel_ms",
]


class M3Error(RuntimeError):
    def __init__(self, code, msg):
        super().__init__(f"{ERR_NAMES.get(code, code)}: {msg}")
        self.code = code


_lib = None
_lock = threading.Lock()


def lib():
    """Load libm3.so (raises M3Error if it has not been built)."""
    global _lib
    if _lib is not None:
        return _lib
    with _lock:
        if _lib is not None:
            return _lib
        if not os.path.exists(LIB_PATH):
            raise M3Error(-5, f"{LIB_PATH} not found: build it with `make -C element-crush-gym_amd` "
                              "(there is no CPU fallback)")
        L = ctypes.CDLL(LIB_PATH)
        vp, i32, i64, u32 = ctypes.c_void_p, ctypes.c_int, ctypes.c_int64, ctypes.c_uint32
        sig = {
            "m3_abi_version": ([], i32),
            "m3_last_error": ([], ctypes.c_char_p),
            "m3_device_count": ([vp], i32),
            "m3_supported": ([i32, i32, i32], i32),
            "m3_action_space": ([i32, i32, vp, vp], i32),
            "m3_ctx_create": ([i32, i32, i32, i32, vp], i32),
            "m3_ctx_destroy": ([vp], i32),
            "m3_ctx_synchronize": ([vp], i32),
            "m3_dev_alloc": ([vp, i64, vp], i32),
            "m3_dev_free": ([vp, vp], i32),
            "m3_dev_copy": ([vp, vp, vp, i64, i32], i32),
            "m3_init_boards": ([vp, i64, vp, vp, vp, vp], i32),
            "m3_init_boards_ex": ([vp, i64, vp, vp, vp, vp, vp], i32),
            "m3_apply_actions": ([vp, i64, vp, vp, vp, vp, vp, vp, vp, vp, vp, vp], i32),
            "m3_legal_actions": ([vp, i64, vp, vp], i32),
            "m3_rollouts": ([vp, i64] + [vp] * 9, i32),
            "m3_rollouts_device": ([vp, i64] + [vp] * 9, i32),
            "m3_env_create": ([vp, i64, i32, i32, vp], i32),
            "m3_env_destroy": ([vp], i32),
            "m3_env_reset": ([vp, vp, u32], i32),
            "m3_env_set_shards": ([vp, i32], i32),
            "m3_env_synchronize": ([vp], i32),
            "m3_env_set_autoreset": ([vp, i32, u32], i32),
            "m3_env_step": ([vp, vp], i32),
            "m3_env_step_device": ([vp, vp], i32),
            "m3_env_get": ([vp, i32, vp], i32),
            "m3_env_set": ([vp, i32, vp], i32),
            "m3_env_device_ptr": ([vp, i32, vp], i32),
            "m3_env_comm_size": ([vp, vp], i32),
            "m3_comm_unique_id": ([vp], i32),
            "m3_env_comm_init": ([vp, vp, i32, i32], i32),
            "m3_env_gather": ([vp, vp], i32),
            "m3_env_gather_device": ([vp, vp], i32),
            "m3_env_debug_stall": ([vp, u32], i32),
            "m3_env_stats": ([vp, vp], i32),
            "m3_env_timing": ([vp, i32], i32),
            "m3_env_kernel_ms": ([vp, vp, i32, vp], i32),
            "m3_env_step_kernel_ms": ([vp, vp, i32, vp], i32),
        }
        for name, (args, res) in sig.items():
            fn = getattr(L, name, None)  # (an older A/B build may lack newer entry points;
            if fn is None:               #  tests/test_abi_cpu.py holds the real library to the header)
                continue
            fn.argtypes = args
            fn.restype = res
        _lib = L
    return _lib


def check(rc):
    if rc != M3_OK:
        raise M3Error(rc, lib().m3_last_error().decode(errors="replace"))


def ptr(a):
    return None if a is None else ctypes.c_void_p(a.ctypes.data)


def device_count() -> int:
    n = ctypes.c_int(0)
    check(lib().m3_device_count(ctypes.byref(n)))
    return n.value


def supported(rows, columns, types) -> bool:
    return bool(lib().m3_supported(rows, columns, types))


class DeviceArray:
    """Device memory on a context's device (m3_dev_alloc): for benches and tests that feed the
    *_device entry points without a second HIP runtime (torch) in the process."""

    def __init__(self, ctx, nbytes: int):
        self.ctx, self.nbytes = ctx, int(nbytes)
        p = ctypes.c_void_p()
        check(lib().m3_dev_alloc(ctx.handle, self.nbytes, ctypes.byref(p)))
        self.ptr = p

    def upload(self, a):
        a = np.ascontiguousarray(a)
        if a.nbytes != self.nbytes:
            raise ValueError(f"{a.nbytes} bytes into a {self.nbytes}-byte device array")
        check(lib().m3_dev_copy(self.ctx.handle, self.ptr, ptr(a), self.nbytes, 1))
        return self

    def to_host(self, dtype, shape):
        out = np.empty(shape, dtype)
        if out.nbytes != self.nbytes:
            raise ValueError(f"{self.nbytes}-byte device array as {out.nbytes} bytes")
        check(lib().m3_dev_copy(self.ctx.handle, ptr(out), self.ptr, self.nbytes, 2))
        return out

    def at(self, offset: int):
        return ctypes.c_void_p(self.ptr.value + int(offset))

    def free(self):
        if self.ptr:
            check(lib().m3_dev_free(self.ctx.handle, self.ptr))
            self.ptr = None


class Context:
    """One HIP stream + scratch on one device for one board shape (m3_ctx)."""

    def __init__(self, rows=9, columns=9, types=6, device=0):
        self.rows, self.columns, self.types, self.device = rows, columns, types, device
        self.N = rows * columns
        self.A = rows * (columns - 1) * 2
        self.words = (self.A + 31) // 32
        h = ctypes.c_void_p()
        check(lib().m3_ctx_create(device, rows, columns, types, ctypes.byref(h)))
        self.handle = h
        self._lock = threading.Lock()

    def close(self):
        if getattr(self, "handle", None):
            lib().m3_ctx_destroy(self.handle)
            self.handle = None

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass

    def device_empty(self, nbytes: int) -> DeviceArray:
        return DeviceArray(self, nbytes)

    def device_array(self, a) -> DeviceArray:
        a = np.ascontiguousarray(a)
        return DeviceArray(self, a.nbytes).upload(a)

    # ---- stateless batch calls --------------------------------------------------
    def _boards(self, boards):
        b = np.asarray(boards)
        if b.size and (b.min() < 0 or b.max() > 127):
            raise ValueError("cell values must lie in [0, 127]")
        return np.ascontiguousarray(b.reshape(-1, self.N), dtype=np.int8)

    def init_boards(self, seeds, flags=False):
        """BoardV2.__init__ of each seed: (boards, draws, first_action[, flags]). Without flags, a reset
        that stopped at the redraw-round cap raises (M3_ERR_CAP: the reference would keep drawing)."""
        seeds = np.ascontiguousarray(np.atleast_1d(seeds), dtype=np.uint32)
        n = len(seeds)
        out = np.empty((n, self.N), np.int8)
        draws = np.empty(n, np.uint32)
        first = np.empty(n, np.int32)
        fl = np.empty(n, np.uint32) if flags else None
        with self._lock:
            if flags:
                check(lib().m3_init_boards_ex(self.handle, n, ptr(seeds), ptr(out), ptr(draws), ptr(first), ptr(fl)))
            else:
                check(lib().m3_init_boards(self.handle, n, ptr(seeds), ptr(out), ptr(draws), ptr(first)))
        res = (out.reshape(n, self.rows, self.columns), draws, first)
        return res + (fl,) if flags else res

    def apply_actions(self, boards, seeds, n_actions, actions, legal=False, next_action=False):
        b = self._boards(boards)
        n = len(b)
        seeds = np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, dtype=np.uint32), (n,)))
        na = np.ascontiguousarray(np.broadcast_to(np.asarray(n_actions, dtype=np.int32), (n,)))
        act = np.ascontiguousarray(np.broadcast_to(np.asarray(actions, dtype=np.int32), (n,)))
        out = np.empty_like(b)
        rew = np.empty(n, np.int32)
        draws = np.empty(n, np.uint32)
        flags = np.empty(n, np.uint32)
        lg = np.empty((n, self.words), np.uint32) if legal else None
        nx = np.empty(n, np.int32) if next_action else None
        with self._lock:
            check(lib().m3_apply_actions(self.handle, n, ptr(b), ptr(seeds), ptr(na), ptr(act), ptr(out), ptr(rew),
                                         ptr(draws), ptr(flags), ptr(lg), ptr(nx)))
        res = dict(boards=out.reshape(n, self.rows, self.columns), reward=rew, draws=draws, flags=flags)
        if legal:
            res["legal"] = lg
        if next_action:
            res["next_action"] = nx
        return res

    def legal_bits(self, boards):
        b = self._boards(boards)
        out = np.empty((len(b), self.words), np.uint32)
        with self._lock:
            check(lib().m3_legal_actions(self.handle, len(b), ptr(b), ptr(out)))
        return out

    def rollouts(self, boards, seeds, n_actions, rollout_seeds, final_boards=False):
        """MCTS.rollout (mctslib/standard/mcts.py:14-19) of n states in one launch.

        Returns gain (summed step rewards), steps, draws (global stream position
        since its last seed) and flags per rollout, and optionally the terminal boards."""
        b = self._boards(boards)
        n = len(b)
        seeds = np.ascontiguousarray(np.broadcast_to(np.asarray(seeds, dtype=np.uint32), (n,)))
        na = np.ascontiguousarray(np.broadcast_to(np.asarray(n_actions, dtype=np.int32), (n,)))
        rs = np.ascontiguousarray(np.broadcast_to(np.asarray(rollout_seeds, dtype=np.uint32), (n,)))
        gain = np.empty(n, np.int32)
        steps = np.empty(n, np.int32)
        draws = np.empty(n, np.uint32)
        flags = np.empty(n, np.uint32)
        fin = np.empty_like(b) if final_boards else None
        with self._lock:
            check(lib().m3_rollouts(self.handle, n, ptr(b), ptr(seeds), ptr(na), ptr(rs), ptr(gain), ptr(steps),
                                    ptr(draws), ptr(flags), ptr(fin)))
        res = dict(gain=gain, steps=steps, draws=draws, flags=flags)
        if final_boards:
            res["final"] = fin.reshape(n, self.rows, self.columns)
        return res

    def legal_actions(self, board):
        """Ascending legal action ids of one board (boardFunctions.legal_actions)."""
        return bits_to_actions(self.legal_bits(board)[0], self.A)


def bits_to_actions(words, A):
    bits = np.unpackbits(np.ascontiguousarray(words, dtype="<u4").view(np.uint8), bitorder="little")[:A]
    return [int(i) for i in np.flatnonzero(bits)]


_contexts = {}
_ctx_lock = threading.Lock()


def context(rows=9, columns=9, types=6, device=0) -> Context:
    """Process-wide cached context for a shape (used by the BoardV2 facade)."""
    key = (rows, columns, types, device, threading.get_ident())
    c = _contexts.get(key)
    if c is None:
        with _ctx_lock:
            c = _contexts.get(key)
            if c is None:
                c = Context(rows, columns, types, device)
                _contexts[key] = c
    return c
