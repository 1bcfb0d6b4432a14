"""GPU side of the N>1 path on one MI355X: each rank's shard (seed plan + autoreset stride) and the RCCL gather.

A world-2 job is two BatchedMatch3Env shards with seed_plan(r, 2, n); here both
shards run on the one GPU of the box (one process), and every step's outcomes
must equal the CPU oracle's same-step-autoreset timeline of that rank
(tests/test_dist_cpu.py, which also proves the shards union to the single-GPU
job). The RCCL all-gather itself is exercised with a 1-rank communicator: its
packed words must be exactly reward << 2 | truncated << 1 | done of the step.
"""
import ctypes

import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


class DeviceBuffer:
    """Test-side device memory through the HIP runtime libm3.so itself runs on (no torch: a second
    HIP runtime in the process is not reliable)."""

    @staticmethod
    def _hip_runtime():
        """The libamdhip64 that libm3.so itself loaded (read from /proc/self/maps), so the test
        allocates through the same runtime whatever its soname."""
        from match3tile import _native

        _native.lib()
        with open("/proc/self/maps") as f:
            paths = {line.split()[-1] for line in f if "libamdhip64.so" in line}
        assert len(paths) == 1, paths
        return ctypes.CDLL(paths.pop())

    def __init__(self, nbytes):
        self.hip = self._hip_runtime()
        self.nbytes = nbytes
        self.ptr = ctypes.c_void_p()
        assert self.hip.hipMalloc(ctypes.byref(self.ptr), ctypes.c_size_t(nbytes)) == 0
        assert self.hip.hipMemset(self.ptr, 0xFF, ctypes.c_size_t(nbytes)) == 0
        assert self.hip.hipDeviceSynchronize() == 0

    def at(self, offset):
        return ctypes.c_void_p(self.ptr.value + offset)

    def to_host(self, dtype, shape):
        out = np.empty(shape, dtype)
        assert out.nbytes == self.nbytes
        assert self.hip.hipMemcpy(ctypes.c_void_p(out.ctypes.data), self.ptr, ctypes.c_size_t(self.nbytes), 2) == 0
        return out

    def free(self):
        self.hip.hipFree(self.ptr)


def test_rank_shards_match_oracle_autoreset_timeline():
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import pack_outcomes, seed_plan
    from test_dist_cpu import GOAL, MOVES, STEPS, autoreset_outcomes

    world, n = 2, 1000
    for rank in range(world):
        base, stride = seed_plan(rank, world, n)
        env = BatchedMatch3Env(n, 9, 9, 6, num_moves=MOVES, env_goal=GOAL, seed_base=base, seed_stride=stride)
        got = np.zeros((STEPS, n), np.int32)
        for t in range(STEPS):
            _, r, d, tr, _ = env.step(copy=True)
            got[t] = pack_outcomes(r, tr, d)
        env.close()
        want = autoreset_outcomes(rank, world, n)
        assert (got == want).all(), f"rank {rank}: {(got != want).sum()} outcome words differ"


def test_rccl_gather_packs_step_outcomes():
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import pack_outcomes, unpack_outcomes

    n = 4096
    env = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=200)
    env.init_comm(BatchedMatch3Env.comm_unique_id(), 1, 0)
    seen_done = 0
    for _ in range(25):
        env.step()
        g = env.gather(to_host=True)
        r, tr, d = env.rewards(), env.truncateds(), env.dones()
        assert g.shape == (n,) and (g == pack_outcomes(r, tr, d)).all()
        r2, _, d2 = unpack_outcomes(g)
        assert (r2 == r).all() and (d2 == d).all()
        seen_done += int(d.sum())
    env.close()
    assert seen_done >= n  # every board finished at least once (autoreset ran)


def test_rccl_gather_async_double_buffer():
    """Gathers held in flight while later steps run (packed words double-buffered by step parity).

    Each step's gather lands in a device buffer of its own and is delayed on the context stream
    (m3_env_debug_stall) long enough that steps t+1 and t+2 are enqueued and would have finished
    before it reads; what every gather actually read is compared with that step's outcomes from a
    second env stepped synchronously on the same seeds. Without the step t+2 -> gather t wait,
    gather t reads step t+2's words."""
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import pack_outcomes

    n, steps = 70_000, 10
    want = np.zeros((steps, n), np.int32)
    ref = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=300, shards=2)
    for t in range(steps):
        _, r, d, tr, _ = ref.step(copy=True)
        want[t] = pack_outcomes(r, tr, d)
    ref.close()

    env = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=300, shards=2)
    env.init_comm(BatchedMatch3Env.comm_unique_id(), 1, 0)
    outs = DeviceBuffer(steps * n * 4)
    for t in range(steps):
        env.step()
        env.debug_stall(3000)  # the gather of step t starts >= 3 ms after it is enqueued
        env.gather_device(outs.at(t * n * 4))
    env.synchronize()
    got = outs.to_host(np.int32, (steps, n))
    outs.free()
    last = env.gathered()  # the env's own buffer: untouched by gathers into caller buffers
    env.close()
    for t in range(steps):
        assert (got[t] == want[t]).all(), f"gather of step {t}: {(got[t] != want[t]).sum()} words differ"
    assert last.shape == (n,)


def test_comm_init_twice_is_rejected():
    from match3tile._native import M3Error
    from match3tile.batched import BatchedMatch3Env

    env = BatchedMatch3Env(256, 9, 9, 6)
    uid = BatchedMatch3Env.comm_unique_id()
    env.init_comm(uid, 1, 0)
    with pytest.raises(M3Error, match="M3_ERR_STATE"):
        env.init_comm(uid, 1, 0)
    env.step()
    env.gather()
    assert env.gathered().shape == (256,)
    env.close()


def test_host_actions_double_buffered_upload():
    """Host-action steps interleaved with in-flight gathers and random-action steps: every step's
    outcome equals a synchronously stepped twin's, and the caller's buffer is reusable at once."""
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import pack_outcomes

    n, steps = 20_000, 12
    rng = np.random.default_rng(5)
    plan = [None if t % 4 == 3 else rng.integers(0, 144, n).astype(np.int32) for t in range(steps)]
    want = np.zeros((steps, n), np.int32)
    ref = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=300, shards=2)
    for t in range(steps):
        _, r, d, tr, _ = ref.step(None if plan[t] is None else plan[t].copy(), copy=True)
        want[t] = pack_outcomes(r, tr, d)
    ref_boards = ref.observations()
    ref.close()

    env = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=300, shards=2)
    env.init_comm(BatchedMatch3Env.comm_unique_id(), 1, 0)
    buf = np.empty(n, np.int32)
    got = []
    for t in range(steps):
        if plan[t] is None:
            env.step()
        else:
            buf[:] = plan[t]
            env.step(buf)
            buf[:] = -7  # reused at once: the step must have taken its own copy
        env.debug_stall(500)
        got.append(env.gather(to_host=(t % 3 == 2)))
        if got[-1] is not None:
            assert (got[-1] == want[t]).all(), t
    assert (env.observations() == ref_boards).all()
    env.close()
