"""Checkpoint / resume of the batched env (SURVEY.md §5 checkpoint row; m3_env_set).

The reference's per-board state is (array, cfg.seed, n_actions, _reward)
(boardv2.py:12-16) plus Match3Env's score / moves_taken (env.py:34). An env
saved after step 7 and loaded into a fresh process-side env must step on
exactly like the uninterrupted env: same observations, rewards, done /
truncated flags, scores, moves, seeds (autoreset), pre-drawn seeded actions
and legal sets, for 23 more steps (through several autoresets).
"""
import numpy as np
import pytest

from conftest import SHAPES

pytestmark = pytest.mark.gpu

from match3tile import _native  # noqa: E402
from match3tile.batched import BatchedMatch3Env  # noqa: E402


@pytest.fixture(scope="module", autouse=True)
def _need_gpu():
    if _native.device_count() == 0:
        pytest.fail("no GPU visible: -m gpu tests must run on the MI355X box")


def _state(env):
    return (env.observations(), env.rewards(), env.dones(), env.truncateds(), env.scores(), env.moves(),
            env.seeds(), env.next_actions(), env.legal_bits(), env.flags(), env.draws())


@pytest.mark.parametrize("tag", list(SHAPES))
def test_save_at_step_7_resume_equals_uninterrupted(tmp_path, tag):
    n = 8192 if tag == "9x9x6" else 2048
    a = BatchedMatch3Env(n, *SHAPES[tag], num_moves=20, env_goal=400, seed_base=3, autoreset=True, shards=2)
    for _ in range(7):
        a.step()
    path = str(tmp_path / "ck.npz")
    a.save(path)
    b = BatchedMatch3Env.load(path, shards=1)
    for x, y in zip(_state(a), _state(b)):
        assert (x == y).all()
    resets = 0
    for t in range(23):
        if t % 5 == 4:  # host actions too
            acts = np.random.default_rng(t).integers(0, a.A, size=n).astype(np.int32)
            a.step(acts)
            b.step(acts)
        else:
            a.step()
            b.step()
        for x, y in zip(_state(a), _state(b)):
            assert (x == y).all(), t
        resets += int(a.dones().sum())
    assert resets > n  # every board went through at least one autoreset after the resume
    a.close()
    b.close()


def test_load_rejects_wrong_shape_and_derived_fields(tmp_path):
    a = BatchedMatch3Env(256, seed_base=1, autoreset=False)
    a.step()
    path = str(tmp_path / "ck.npz")
    a.save(path)
    other = BatchedMatch3Env(128, seed_base=1, autoreset=False)
    with pytest.raises(ValueError):
        other.load_state_dict(dict(np.load(path)))
    with pytest.raises(_native.M3Error) as e:
        _native.check(_native.lib().m3_env_set(a.handle, _native.ENV_LEGAL, _native.ptr(np.zeros((256, 5), np.uint32))))
    assert e.value.code == -1
    with pytest.raises(_native.M3Error):
        bad = np.full((256, 9, 9), -1, np.int8)
        _native.check(_native.lib().m3_env_set(a.handle, _native.ENV_BOARDS, _native.ptr(bad)))
    a.close()
    other.close()


def test_loaded_boards_step_like_the_stateless_kernel():
    """Arbitrary boards / seeds loaded into an env step like BoardV2.apply_action on them."""
    n = 1024
    ctx = _native.Context(9, 9, 6)
    seeds = np.arange(5000, 5000 + n, dtype=np.uint32)
    boards, _, first = ctx.init_boards(seeds)
    env = BatchedMatch3Env(n, seeds=False, autoreset=False)
    st = {k: v for k, v in env.state_dict().items()}
    st.update(boards=boards, seeds=seeds, score=np.zeros(n, np.int32), moves=np.zeros(n, np.int32),
              next_action=first)
    env.load_state_dict(st)
    assert (env.legal_bits() == ctx.legal_bits(boards)).all()
    env.step()
    ref = ctx.apply_actions(boards, seeds, 20, first, next_action=True)
    assert (env.observations() == ref["boards"]).all()
    assert (env.rewards() == ref["reward"]).all()
    assert (env.next_actions() == ref["next_action"]).all()
    env.close()
    ctx.close()


def test_reload_after_odd_step_count_then_host_actions():
    """A stepped env (odd step count) reloaded and then stepped twice with host actions equals
    the uninterrupted env: the reload restarts the step counter before the upload buffer of the
    next host-action step is chosen."""
    n = 4096
    a = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=400, seed_base=11, autoreset=True, shards=2)
    for _ in range(3):
        a.step()
    st = a.state_dict()
    b = BatchedMatch3Env(n, 9, 9, 6, num_moves=20, env_goal=400, seed_base=99, autoreset=True, shards=2)
    for _ in range(7):  # odd: the next host-action upload would pick buffer 1 without the restart
        b.step()
    b.load_state_dict(st)  # no read of b before it steps again
    rng = np.random.default_rng(5)
    for t in range(4):
        acts = rng.integers(0, a.A, size=n).astype(np.int32)
        a.step(acts)
        b.step(acts)
    for x, y in zip(_state(a), _state(b)):
        assert (x == y).all()
    a.close()
    b.close()


def test_partial_load_is_not_ready_and_fresh_env_reads_zeros():
    n = 512
    env = BatchedMatch3Env(n, seeds=False, autoreset=False)
    st = env.state_dict()  # never reset: zero-initialised fields, not stale device memory
    for k in ("boards", "seeds", "score", "moves", "next_action", "reward", "flags"):
        assert not st[k].any(), k
    ctx = _native.Context(9, 9, 6)
    boards, _, first = ctx.init_boards(np.arange(1, n + 1, dtype=np.uint32))
    _native.check(_native.lib().m3_env_set(env.handle, _native.ENV_BOARDS, _native.ptr(boards)))
    with pytest.raises(_native.M3Error) as e:  # seeds / score / moves / next_action never loaded
        env.step()
    assert e.value.code == -6
    for what, arr in ((_native.ENV_SEEDS, np.arange(1, n + 1, dtype=np.uint32)),
                      (_native.ENV_SCORE, np.zeros(n, np.int32)), (_native.ENV_MOVES, np.zeros(n, np.int32)),
                      (_native.ENV_NEXT_ACTION, first)):
        _native.check(_native.lib().m3_env_set(env.handle, what, _native.ptr(arr)))
    env.step()  # now complete
    ref = ctx.apply_actions(boards, np.arange(1, n + 1, dtype=np.uint32), 20, first)
    assert (env.observations() == ref["boards"]).all()
    env.close()
    ctx.close()
