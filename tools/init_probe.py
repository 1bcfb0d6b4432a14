"""Time the stateless reset kernels for several batch sizes (run under rocprofv3 --kernel-trace)."""
import os
import sys
import time

sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "element-crush-gym_amd"))
import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402

ctx = _native.Context(9, 9, 6)
for n in (64, 1024, 16384, 65536, 262144, 1048576):
    seeds = np.arange(1, n + 1, dtype=np.uint32)
    ctx.init_boards(seeds)  # warm
    t = time.perf_counter()
    for _ in range(3):
        ctx.init_boards(seeds)
    print(f"init n={n:8d}  {(time.perf_counter() - t) / 3 * 1e3:8.3f} ms/call (host, incl. copies)", flush=True)
