"""ctypes face of the TEST-ONLY host build of the device rule code (hostcore.hip)."""
import ctypes
import os
import subprocess

import numpy as np

HERE = os.path.dirname(os.path.abspath(__file__))
LIB = os.path.join(HERE, "libhostcore.so")
SRC = [os.path.join(HERE, "hostcore.hip")] + [
    os.path.join(HERE, "..", "..", "element-crush-gym_amd", "csrc", f) for f in
    ("m3_rules.hpp", "m3_bitboard.hpp", "m3_rng.hpp")]
_lib = None
CFG_ID = {(9, 9, 6): 0, (16, 16, 8): 1}
FRAME = 2  # any other shape, in its frame (16 x 16, or 32 x 32 for a side > 16; hc_set_frame)


def build():
    newest = max(os.path.getmtime(s) for s in SRC)
    if os.path.exists(LIB) and os.path.getmtime(LIB) >= newest:
        return
    # -O0: the 32 x 32-frame instantiations take ~30 min to optimise on the host (1024-bit planes,
    # fully unrolled); unoptimised, the whole harness builds in ~2 min and the tests still run in seconds
    subprocess.run(["hipcc", "--offload-arch=gfx950", "-O0", "-std=c++17", "-fPIC", "-shared",
                    "-o", LIB + ".tmp", SRC[0]], check=True)
    os.replace(LIB + ".tmp", LIB)


def lib():
    global _lib
    if _lib is None:
        build()
        _lib = ctypes.CDLL(LIB)
        _lib.hc_chain_draw.restype = ctypes.c_uint32
        _lib.hc_chain_draw.argtypes = [ctypes.c_uint32, ctypes.c_int]
        _lib.hc_mask_mismatches.restype = ctypes.c_long
        _lib.hc_mask_mismatches.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p]
        _lib.hc_fast_match_mismatches.restype = ctypes.c_long
        _lib.hc_fast_match_mismatches.argtypes = [ctypes.c_int, ctypes.c_long, ctypes.c_void_p, ctypes.c_void_p]
    return _lib


def _p(a):
    return ctypes.c_void_p(a.ctypes.data)


class HostCore:
    """frame=None: the specialised config for 9x9x6 / 16x16x8, the frame for any other shape;
    frame=True forces the frame form (e.g. to run 9x9x6 through it)."""

    def __init__(self, R=9, C=9, T=6, frame=None):
        self.shape = (R, C, T)
        self.frame = (R, C, T) not in CFG_ID if frame is None else bool(frame)
        self.cfg = FRAME if self.frame else CFG_ID[(R, C, T)]
        self.N = R * C
        self.A = R * (C - 1) * 2
        self.aw = (self.A + 31) // 32

    def _sel(self):
        if self.frame:
            assert lib().hc_set_frame(*self.shape) == 0, self.shape

    def apply(self, boards, seeds, n_actions, actions, small=False):
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        n = len(boards)
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        na = np.ascontiguousarray(np.broadcast_to(n_actions, (n,)), dtype=np.int32)
        acts = np.ascontiguousarray(actions, dtype=np.int32)
        out = np.zeros_like(boards)
        rew = np.zeros(n, np.int32); drw = np.zeros(n, np.int32); flg = np.zeros(n, np.int32)
        legal = np.zeros((n, self.aw), np.uint32); nxt = np.zeros(n, np.int32)
        self._sel()
        self.recomputed = lib().hc_apply(self.cfg, ctypes.c_long(n), _p(boards), _p(seeds), _p(na), _p(acts),
                                         _p(out), _p(rew), _p(drw), _p(flg), _p(legal), _p(nxt), int(small))
        return out, rew, drw, flg, legal, nxt

    def mask_mismatches(self, boards):
        """boards whose fast match mask (union of runs when no run start is covered by an earlier
        run of the other direction) differs from the sequential scan's"""
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        self._sel()
        return lib().hc_mask_mismatches(self.cfg, ctypes.c_long(len(boards)), _p(boards))

    def fast_match_mismatches(self, boards):
        """(boards where get_matches differs from the sequential scan, boards its loop-free path took)"""
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        fast = ctypes.c_long(0)
        self._sel()
        bad = lib().hc_fast_match_mismatches(self.cfg, ctypes.c_long(len(boards)), _p(boards), ctypes.byref(fast))
        return bad, fast.value

    def init(self, seeds):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        n = len(seeds)
        out = np.zeros((n, self.N), np.int8); drw = np.zeros(n, np.int32)
        m397 = np.zeros(n, np.uint32); fa = np.zeros(n, np.int32)
        self._sel()
        self.recomputed = lib().hc_init(self.cfg, ctypes.c_long(n), _p(seeds), _p(out), _p(drw), _p(m397), _p(fa))
        return out, drw, m397, fa

    def legal(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        out = np.zeros((len(boards), self.aw), np.uint32)
        self._sel()
        lib().hc_legal(self.cfg, ctypes.c_long(len(boards)), _p(boards), _p(out))
        return out

    def matches(self, tbs):
        tbs = np.ascontiguousarray(tbs, dtype=np.int8).reshape(-1, self.N)
        n = len(tbs)
        mask = np.zeros((n, self.N), np.uint8); sp = np.zeros((n, self.N), np.int32); fd = np.zeros(n, np.int32)
        self._sel()
        lib().hc_matches(self.cfg, ctypes.c_long(n), _p(tbs), _p(mask), _p(sp), _p(fd))
        return mask, sp, fd

    def roundtrip(self, boards):
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        out = np.zeros_like(boards)
        self._sel()
        lib().hc_roundtrip(self.cfg, ctypes.c_long(len(boards)), _p(boards), _p(out))
        return out


    def rollouts(self, boards, seeds, n_actions, rseeds):
        """rollout_one of k_rollout on the CPU (gain -1: the chain ran out, the kernel's replay case)"""
        boards = np.ascontiguousarray(boards, dtype=np.int8).reshape(-1, self.N)
        n = len(boards)
        seeds = np.ascontiguousarray(np.broadcast_to(seeds, (n,)), dtype=np.uint32)
        na = np.ascontiguousarray(np.broadcast_to(n_actions, (n,)), dtype=np.int32)
        rs = np.ascontiguousarray(np.broadcast_to(rseeds, (n,)), dtype=np.uint32)
        gain = np.zeros(n, np.int32); steps = np.zeros(n, np.int32)
        draws = np.zeros(n, np.uint32); flags = np.zeros(n, np.uint32)
        self._sel()
        lib().hc_rollout(self.cfg, ctypes.c_long(n), _p(boards), _p(seeds), _p(na), _p(rs), _p(gain), _p(steps),
                         _p(draws), _p(flags))
        return dict(gain=gain, steps=steps, draws=draws, flags=flags)

    def init_scalar(self, seeds):
        seeds = np.ascontiguousarray(seeds, dtype=np.uint32)
        n = len(seeds)
        out = np.zeros((n, self.N), np.int8); drw = np.zeros(n, np.int32)
        self._sel()
        lib().hc_init_scalar(self.cfg, ctypes.c_long(n), _p(seeds), _p(out), _p(drw))
        return out, drw


def bits_to_list(words, A):
    bits = np.unpackbits(np.asarray(words, dtype="<u4").view(np.uint8), bitorder="little")[:A]
    return [int(i) for i in np.nonzero(bits)[0]]
