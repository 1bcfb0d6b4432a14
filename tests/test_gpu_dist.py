"""GPU side of the N>1 path on one MI355X: each rank's shard (seed plan + autoreset stride) and the RCCL gather.

A world-2 job is two BatchedMatch3Env shards with seed_plan(r, 2, n); here both
shards run on the one GPU of the box (one process), and every step's outcomes
must equal the CPU oracle's same-step-autoreset timeline of that rank
(tests/test_dist_cpu.py, which also proves the shards union to the single-GPU
job). The RCCL all-gather itself is exercised with a 1-rank communicator: its
packed words must be exactly reward << 2 | truncated << 1 | done of the step.
"""
import numpy as np
import pytest

from conftest import gpu_available

pytestmark = [pytest.mark.gpu, pytest.mark.skipif(not gpu_available(), reason="needs an MI355X")]


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
    """Gathers left in flight while later steps run (packed words double-buffered by step parity):
    every gathered snapshot must be the outcome of the step it followed."""
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import pack_outcomes

    n = 70_000
    env = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=300, shards=2)
    env.init_comm(BatchedMatch3Env.comm_unique_id(), 1, 0)
    for t in range(12):
        env.step()
        if t % 3 == 2:  # synchronous check every third step
            g = env.gather(to_host=True)
            assert (g == pack_outcomes(env.rewards(), env.truncateds(), env.dones())).all(), t
        else:
            env.gather()  # async: the next step runs while this gather reads its buffer
    env.close()
