"""debug (round 5): frame-kernel lane interference through the env (k_env_step) and the stateless
k_apply kernel, on the library in M3_LIB. Usage: lanes_env.py RxCxT"""
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
sys.path.insert(0, os.path.join(ROOT, "element-crush-gym_amd"))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
import numpy as np  # noqa: E402

from match3tile import _native  # noqa: E402
from match3tile.batched import BatchedMatch3Env  # noqa: E402
from oracle import Oracle  # noqa: E402

shape = sys.argv[1] if len(sys.argv) > 1 else "10x8x9"
R, C, T = (int(x) for x in shape.split("x"))
N, M, GOAL = 4096, 20, 1 << 30
o = Oracle(R, C, T)
env = BatchedMatch3Env(N, R, C, T, num_moves=M, env_goal=GOAL, seed_base=1, autoreset=False, shards=1)
obs, acts, rews, drws = [env.observations().copy()], [], [], []
for t in range(M):
    acts.append(env.next_actions().copy())
    env.step()
    obs.append(env.observations().copy())
    rews.append(env.rewards().copy())
    drws.append(env.draws().copy() if hasattr(env, "draws") else None)
ref = o.batch_episodes(np.arange(1, N + 1, dtype=np.uint32), M, GOAL)
A = np.stack(acts, 1)
Rw = np.stack(rews, 1)
bad_step = np.full(N, -1)
for b in range(N):
    d = np.nonzero((A[b] != ref["actions"][b]) | (Rw[b] != ref["rewards"][b]))[0]
    if len(d):
        bad_step[b] = d[0]
bad = np.nonzero(bad_step >= 0)[0]
print(shape, "env: boards with a wrong step", len(bad), "of", N, flush=True)
print("   first:", [(int(b), int(bad_step[b])) for b in bad[:16]], flush=True)
ctx = _native.Context(R, C, T)
# stateless k_apply on the pre-step boards of the first bad step (the step t where board b went wrong:
# its pre-step board obs[t][b] is still right), whole waves vs alone
for b in bad[:6]:
    t = int(bad_step[b])
    if t > 0 and (A[b][t - 1] != ref["actions"][b][t - 1]):
        continue
    w0 = b - b % 64
    idx = np.arange(w0, min(w0 + 64, N))
    pre = obs[t][idx]
    act = A[idx, t]
    na = np.full(len(idx), M - t, np.int32)
    seeds = (idx + 1).astype(np.uint32)
    g = ctx.apply_actions(pre, seeds, na, act)
    g1 = ctx.apply_actions(obs[t][b:b + 1], seeds[b - w0:b - w0 + 1], na[:1], act[b - w0:b - w0 + 1])
    want = o.apply_action(obs[t][b].reshape(R, C), b + 1, int(act[b - w0]), M - t)
    l = b - w0
    print(f"   board {b} step {t}: oracle reward {want[1]} draws {want[2]} | wave k_apply reward {g['reward'][l]} "
          f"draws {g['draws'][l]} board_ok {(g['boards'][l].reshape(-1) == want[0].reshape(-1)).all()} | alone "
          f"reward {g1['reward'][0]} draws {g1['draws'][0]} board_ok {(g1['boards'][0].reshape(-1) == want[0].reshape(-1)).all()}",
          flush=True)
