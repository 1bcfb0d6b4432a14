#!/usr/bin/env python3
"""Per-phase wave-cycle breakdown of k_env_step / k_init (profiling build).

    make -C element-crush-gym_amd prof && python3 tools/phase_prof.py [--boards N --shards S --steps K]

Loads build/libm3_prof.so (compiled with -DM3_PHASE_PROF: s_memtime marks at
phase boundaries, charged to the wave by its first active lane), steps the
batched env and prints cycles per wave per phase. The marks cost a few
instructions each, so absolute totals are slightly above the normal build's.
"""
import argparse
import ctypes
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
PKG = os.path.join(ROOT, "element-crush-gym_amd")
_lib = "libm3_prof.so"
for i, a in enumerate(sys.argv):
    if a == "--lib" and i + 1 < len(sys.argv):
        _lib = sys.argv[i + 1]
os.environ["M3_LIB"] = os.path.join(PKG, "build", _lib)
sys.path.insert(0, PKG)

import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402
from match3tile.batched import BatchedMatch3Env  # noqa: E402

PHASES = ["load", "swap", "match", "clear", "drop", "refill", "legal", "next", "reset", "queue", "store",
          "tbytes", "tload", "tatom"]


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--boards", type=int, default=1 << 20)
    ap.add_argument("--shards", type=int, default=1)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--shape", default="9x9x6")
    ap.add_argument("--lib", default="libm3_prof.so", help="profiling build under element-crush-gym_amd/build")
    a = ap.parse_args()
    R, C, T = (int(x) for x in a.shape.split("x"))
    L = _native.lib()
    L.m3_prof_read.argtypes = [ctypes.c_void_p, ctypes.c_int]
    L.m3_prof_read.restype = ctypes.c_int
    env = BatchedMatch3Env(a.boards, R, C, T, shards=a.shards)
    for _ in range(5):
        env.step()
    env.synchronize()
    nph = len(PHASES)
    buf = np.zeros((2, nph + 2), np.uint64)
    L.m3_prof_read(buf.ctypes.data, 1)
    env.enable_timing(a.steps)
    for _ in range(a.steps):
        env.step()
    env.synchronize()
    L.m3_prof_read(buf.ctypes.data, 0)
    kms = env.kernel_ms()
    out = {"boards": a.boards, "shards": a.shards, "steps": a.steps, "shape": a.shape,
           "k_env_step_ms_mean": float(kms.mean()) if len(kms) else None, "stats": env.stats()}
    for which, name in ((0, "k_env_step"), (1, "k_init")):
        waves = int(buf[which, nph + 1])
        if not waves:
            continue
        tot = float(buf[which, nph]) / waves
        ph = {p: float(buf[which, i]) / waves for i, p in enumerate(PHASES)}
        out[name] = {"waves": waves, "cycles_per_wave": tot,
                     "phase_cycles_per_wave": ph,
                     "phase_frac": {p: v / tot for p, v in ph.items()}}
        print(f"{name}: {waves} waves, {tot:,.0f} cycles/wave", flush=True)
        for p in PHASES:
            print(f"   {p:7s} {ph[p]:12,.0f}  {ph[p] / tot * 100:5.1f}%", flush=True)
    print(json.dumps(out))
    env.close()


if __name__ == "__main__":
    main()
