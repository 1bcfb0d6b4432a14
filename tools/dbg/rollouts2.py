"""debug: which configurations / batch sizes / paths mismatch"""
import os, sys
ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd")); sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np
from match3tile import _native
from oracle import Oracle
def run(ctx, boards, seeds, rs, chunk):
    out = {k: [] for k in ("gain", "steps", "draws", "flags")}
    for i in range(0, len(boards), chunk):
        r = ctx.rollouts(boards[i:i + chunk], seeds[i:i + chunk], 20, rs[i:i + chunk])
        for k in out: out[k].append(r[k])
    return {k: np.concatenate(v) for k, v in out.items()}
for (R, C, T) in [(12, 12, 7), (10, 10, 6), (10, 8, 9), (10, 8, 5), (16, 16, 15), (11, 9, 4)]:
    ctx = _native.Context(R, C, T)
    seeds = np.arange(1, 4097, dtype=np.uint32)
    boards, _, _ = ctx.init_boards(seeds)
    rs = (np.arange(4096, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    want = Oracle(R, C, T).rollouts(boards.astype(np.int32), seeds, 20, rs, threads=8)
    res = []
    for chunk in (4096, 2):
        if chunk == 1 and R * C > 90: continue
        ro = run(ctx, boards, seeds, rs, chunk)
        bad = np.flatnonzero((ro["gain"] != want["gain"]) | (ro["draws"] != want["draws"]))
        res.append((chunk, len(bad), bad[:6].tolist()))
    # device path
    d = [ctx.device_array(x) for x in (boards.reshape(4096, -1), seeds, np.full(4096, 20, np.int32), rs)]
    og = [ctx.device_empty(4096 * 4) for _ in range(4)]
    _native.check(_native.lib().m3_rollouts_device(ctx.handle, 4096, d[0].ptr, d[1].ptr, d[2].ptr, d[3].ptr,
                  og[0].ptr, og[1].ptr, og[2].ptr, og[3].ptr, None))
    g = og[0].to_host(np.int32, 4096); dr = og[2].to_host(np.uint32, 4096)
    bad = np.flatnonzero((g != want["gain"]) | (dr != want["draws"]))
    res.append(("device", len(bad), bad[:6].tolist()))
    print((R, C, T), res, flush=True)
    ctx.close()
