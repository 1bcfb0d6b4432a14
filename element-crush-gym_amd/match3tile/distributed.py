"""Host side of the multi-GPU batched env: one process per GPU, boards sharded by seed range.

Boards are independent (no cross-board dependency in Match3Env.step, env.py:48-56),
so the N-GPU job is N independent shards plus one exchange step: the RCCL
all-gather of each step's packed outcome words over xGMI (m3_env_gather, include/m3.h).

* ``seed_plan`` fixes which seeds a rank owns: rank r steps boards with
  seeds ``seed0 + r*n .. seed0 + (r+1)*n - 1`` and, with autoreset, replaces a
  finished board's seed by ``seed + world*n``, so every (rank, board, episode)
  plays a distinct seed and the union over ranks is exactly the single-GPU job
  on ``world*n`` boards (weak scaling: per-GPU work fixed as N grows).
* ``pack_outcomes`` / ``unpack_outcomes`` are the wire format of the gather
  (``reward << 2 | truncated << 1 | done`` as int32, rank-major ``[world][n]``),
  the same packing k_env_step writes on the device.
* ``timed_steps`` is the bench contract's timed region: W untimed steps, a
  barrier + device sync on both sides of exactly K steps, the max over ranks.

``dist`` arguments are a ``match3tile.rendezvous.Rendezvous`` (what bench.py
uses: plain TCP, no torch), ``torch.distributed`` (the CPU tests' gloo
groups), or None for one process; RCCL carries the data on GPUs.
"""
from __future__ import annotations

import time

import numpy as np


def seed_plan(rank: int, world: int, boards_per_rank: int, seed0: int = 1):
    """(seed_base, seed_stride) of a rank's BatchedMatch3Env."""
    if not (0 <= rank < world) or boards_per_rank <= 0:
        raise ValueError("need 0 <= rank < world and boards_per_rank > 0")
    return (seed0 + rank * boards_per_rank) & 0xFFFFFFFF, (world * boards_per_rank) & 0xFFFFFFFF


def episode_seeds(rank: int, world: int, boards_per_rank: int, episode: int, seed0: int = 1) -> np.ndarray:
    """Seeds of a rank's boards in their `episode`-th episode (0 = after reset)."""
    base, stride = seed_plan(rank, world, boards_per_rank, seed0)
    s = np.arange(boards_per_rank, dtype=np.uint64) + base + np.uint64(episode) * stride
    return (s & 0xFFFFFFFF).astype(np.uint32)


def pack_outcomes(reward, truncated, done) -> np.ndarray:
    r = np.asarray(reward, dtype=np.int32)
    return (r << 2) | (np.asarray(truncated, dtype=np.int32) << 1) | np.asarray(done, dtype=np.int32)


def unpack_outcomes(packed):
    p = np.asarray(packed, dtype=np.int32)
    return p >> 2, ((p >> 1) & 1).astype(bool), (p & 1).astype(bool)


def _active(dist) -> bool:
    if dist is None:
        return False
    if hasattr(dist, "allmax"):  # Rendezvous
        return dist.get_world_size() > 1
    return dist.is_initialized() and dist.get_world_size() > 1


def max_over_ranks(value: float, dist=None) -> float:
    if not _active(dist):
        return float(value)
    if hasattr(dist, "allmax"):
        return dist.allmax(value)
    import torch

    t = torch.tensor([float(value)], dtype=torch.float64)
    dist.all_reduce(t, op=dist.ReduceOp.MAX)
    return float(t.item())


def timed_steps(step, sync, steps: int, warmup: int, dist=None, on_start=None, on_end=None,
                return_local: bool = False):
    """Run `warmup` untimed then exactly `steps` timed calls of step(); seconds, max over ranks.

    on_start() runs after the opening barrier, just before the clock starts
    (bench.py arms the per-launch HIP event timing there); on_end() runs after
    the last timed step and before the closing device sync, so whatever it
    enqueues is timed (bench.py --gather final: the one RCCL all-gather of the
    last step's outcome words). With return_local, returns (max over ranks,
    this rank's own seconds)."""
    for _ in range(warmup):
        step()
    sync()
    if _active(dist):
        dist.barrier()
    if on_start is not None:
        on_start()
    t0 = time.perf_counter()
    for _ in range(steps):
        step()
    if on_end is not None:
        on_end()
    sync()
    elapsed = time.perf_counter() - t0
    if _active(dist):
        dist.barrier()
    mx = max_over_ranks(elapsed, dist)
    return (mx, elapsed) if return_local else mx
