#!/usr/bin/env python3
"""Headline benchmark: batched Match3Env.step throughput on MI355X (BASELINE.json metric).

One "step" = one env step of every board on every GPU: the fused HIP step
kernel (swap, combos, cascade fixed point, MT19937 refill, dead-board
shuffle, scoring, legal mask, next seeded random action), the overflow-fixup
launch, and the autoreset launch that re-initialises finished boards
(seed += stride); for N > 1 also the RCCL all-gather of packed
reward/truncated/done over xGMI. Inputs are resident in HBM before timing.

    python bench.py [--gpus N --steps K --warmup W --boards B]
    torchrun --nproc-per-node N bench.py --gpus N ...   (one process per GPU)

`python bench.py --gpus N` without a launcher starts N rank processes itself
(one per GPU, LOCAL_RANK = device) from a parent that never touches the GPU;
under a launcher WORLD_SIZE must equal --gpus. Ranks rendezvous over a plain
TCP socket (match3tile/rendezvous.py): no torch anywhere in the process.

Prints ONE JSON line on rank 0.
"""
import argparse
import json
import os
import subprocess
import sys
import time

ROOT = os.path.dirname(os.path.abspath(__file__))
PKG = os.path.join(ROOT, "element-crush-gym_amd")
for p in (PKG, os.path.join(ROOT, "oracle")):
    if p not in sys.path:
        sys.path.insert(0, p)

METRIC = "env-steps/sec (batched boards) at 1/2/4/8 MI355X, 9×9×6; bit-exact vs CPU"
HBM_PEAK_GBS = 8000.0  # MI355X_MICROARCH.md chip table (spec)


def algorithmic_bytes_per_step(rows, cols):
    """board in+out (2*R*C int8) + action 2 + reward 4 + done 1 + moves 2 + score 8 + seed 4."""
    return 2 * rows * cols + 21


def host_cores():
    """(usable cores, nproc, cgroup CPU quota): every core this process may run on -- its affinity
    set, capped by the cgroup's cpu.max quota when one is set (a GPU box's share of the host)."""
    aff = len(os.sched_getaffinity(0))
    quota = None
    try:
        with open("/sys/fs/cgroup/cpu.max") as f:
            q, per = f.read().split()[:2]
        if q != "max":
            quota = max(1, -(-int(q) // int(per)))
    except (OSError, ValueError):
        pass
    return (aff if quota is None else min(aff, quota)), os.cpu_count(), quota


def cpu_baseline(rows, cols, types, moves, goal, seconds):
    """The C oracle (bit-exact port of the reference step) on ALL usable host cores, bounded sample,
    plus the calibrated reference-Python equivalent (profiles/cpu_calibration.json)."""
    from oracle import Oracle

    threads, nproc, quota = host_cores()
    o = Oracle(rows, cols, types)
    probe = 2048
    t0 = time.perf_counter()
    steps, _ = o.run_episodes(list(range(10**6, 10**6 + probe)), moves, goal, threads)
    dt = time.perf_counter() - t0
    n = max(probe, int(probe * seconds / max(dt, 1e-3)))
    seeds = list(range(2 * 10**6, 2 * 10**6 + n))
    t0 = time.perf_counter()
    steps, _ = o.run_episodes(seeds, moves, goal, threads)
    dt = time.perf_counter() - t0
    res = {"value": steps / dt, "unit": "env-steps/s", "cores": threads, "nproc": nproc, "cgroup_cpus": quota,
           "kind": "port",
           "sample": f"{n} seeded {rows}x{cols}x{types} random-action episodes of {moves} moves "
                     f"(init + legal_actions + choice + apply_action per move; {steps} steps, {dt:.1f} s), "
                     f"oracle/m3_oracle.c, OpenMP over episodes on {threads} threads"}
    # the same port on ONE core (the C restatement timed on all host cores and on 1 core),
    # a quarter of the sample time
    n1 = max(256, int(probe * seconds / 4 / max(dt / n * probe * threads, 1e-3)))
    seeds1 = list(range(3 * 10**6, 3 * 10**6 + n1))
    t0 = time.perf_counter()
    steps1, _ = o.run_episodes(seeds1, moves, goal, 1)
    dt1 = time.perf_counter() - t0
    res["one_core"] = {"value": steps1 / dt1, "unit": "env-steps/s", "cores": 1, "kind": "port",
                       "sample": f"{n1} episodes ({steps1} steps, {dt1:.1f} s), oracle/m3_oracle.c on 1 thread"}
    try:  # C port here / reference Python here, both measured in the build container (tools/calibrate_cpu.py)
        with open(os.path.join(ROOT, "profiles", "cpu_calibration.json")) as f:
            cal = json.load(f)
        if (rows, cols, types) == (9, 9, 6):
            how = ("this host's C-port rate x (reference Python / C port per core, both timed on "
                   f"{cal['cores']} build-container cores: {cal['ref_python_1']['env_steps_per_s']:.0f} / "
                   f"{cal['c_port_1']['env_steps_per_s']:.0f} env-steps/s), profiles/cpu_calibration.json")
            res["reference_python_equiv"] = {"value": res["value"] * cal["ratio_1core"], "unit": "env-steps/s",
                                             "cores": threads, "how": how}
            res["one_core"]["reference_python_equiv"] = {"value": res["one_core"]["value"] * cal["ratio_1core"],
                                                         "unit": "env-steps/s", "cores": 1, "how": how}
    except (OSError, KeyError, ValueError):
        pass
    return res


# VALU issue peak: 256 CUs x 4 SIMDs, one wave64 VALU instruction per 2 cycles per SIMD
# (MI355X_MICROARCH.md: SIMD-32, wave64 over 2 cycles), 2.4 GHz
VALU_PEAK_WAVE_INSTR_S = 256 * 4 * 2.4e9 / 2


def load_profile(shape_tag, boards, boards_per_launch, steps, warmup):
    """The committed rocprofv3 summary of this configuration (profiles/traffic_<shape>.json, or
    profiles/traffic.json for the headline shape; tools/collect_profiles.py), taken from the same
    command line: shape, boards, shards, steps and warmup must all match, else {}."""
    for name in (f"traffic_{shape_tag}.json", "traffic.json"):
        try:
            with open(os.path.join(ROOT, "profiles", name)) as f:
                t = json.load(f)
            if (t.get("shape") == shape_tag and int(t.get("boards")) == boards
                    and int(t.get("boards_per_launch", -1)) == boards_per_launch
                    and int(t.get("steps", -1)) == steps and int(t.get("warmup", -1)) == warmup):
                return t
        except Exception:
            pass
    return {}


def dist_setup(rank, world):
    """Host-side rendezvous of the ranks (barriers, the max over ranks, the ncclUniqueId broadcast)
    over plain TCP (match3tile/rendezvous.py); RCCL carries the data. None for one process."""
    if world <= 1:
        return None
    from match3tile import rendezvous

    return rendezvous.from_env(rank, world)


def dist_close(dist, rank):
    if dist is None:
        return
    dist.barrier()  # every rank done with the server before rank 0 tears it down
    dist.close()
    if rank == 0:
        from match3tile import rendezvous

        rendezvous.cleanup_port_file()


def share_unique_id(dist, rank, make_id):
    """Rank 0 makes the 128-byte ncclUniqueId, every rank receives it."""
    return dist.broadcast(make_id() if rank == 0 else b"", src=0)


def gather_check(env, dist, rank, world):
    """After timing: one RCCL all-gather of the last step's packed outcome words, checked against
    every rank's own words (each rank's slice of the gathered buffer must equal what that rank
    packed locally; compared through a crc exchanged over the rendezvous). True on every rank iff
    all agree."""
    import zlib

    import numpy as np

    from match3tile.distributed import pack_outcomes

    n = env.n
    got = env.gather(to_host=True).reshape(world, n)
    mine = pack_outcomes(env.rewards(), env.truncateds(), env.dones())
    crcs = dist.allgather_obj(zlib.crc32(mine.tobytes()))
    ok = bool((got[rank] == mine).all()) and all(zlib.crc32(np.ascontiguousarray(got[r]).tobytes()) == crcs[r]
                                                 for r in range(world))
    return all(dist.allgather_obj(ok))


def step_fns(env, world, mode):
    """(step, on_end) of the timed region: one env step per call; for N > 1 the RCCL all-gather of the
    packed outcome words after every step (mode "step") or once after the last timed step ("final")."""
    def step():
        env.step()
        if world > 1 and mode == "step":
            env.gather()

    return step, ((lambda: env.gather()) if world > 1 and mode == "final" else None)


class _StubEnv:
    """--dry-rendezvous: counts what the timed region would enqueue (no device)."""

    def __init__(self):
        self.steps = self.gathers = 0

    def step(self):
        self.steps += 1

    def gather(self):
        self.gathers += 1

    def synchronize(self):
        pass


def spawn_ranks(args):
    """`bench.py --gpus N` without a launcher: start N rank processes (RANK = LOCAL_RANK = device),
    host their rendezvous here, and exit with the first failing rank's code (the other ranks are
    then stopped). This process never touches the GPU (no HIP call before the children start)."""
    from match3tile.rendezvous import RendezvousServer

    n = args.gpus
    srv = RendezvousServer(n)
    procs = []
    for r in range(n):
        env = dict(os.environ, RANK=str(r), LOCAL_RANK=str(r), WORLD_SIZE=str(n), LOCAL_WORLD_SIZE=str(n),
                   GROUP_RANK="0", MASTER_ADDR="127.0.0.1", M3_RDV=srv.address, M3_SPAWNED="1")
        env.pop("MASTER_PORT", None)
        procs.append(subprocess.Popen([sys.executable, os.path.abspath(__file__)] + sys.argv[1:], env=env))
    rc = 0
    live = list(procs)
    while live:
        for p in list(live):
            code = p.poll()
            if code is None:
                continue
            live.remove(p)
            if code != 0 and rc == 0:
                rc = code
                print(f"bench.py: rank {procs.index(p)} exited with {code}; stopping the other ranks",
                      file=sys.stderr)
                for q in live:
                    q.terminate()
        time.sleep(0.05)
    srv.close()
    return rc


def state_digest(env):
    """crc32 of every board's final state (observation, score, moves, seed, pre-drawn action)."""
    import zlib

    c = 0
    for a in (env.observations(), env.scores(), env.moves(), env.seeds(), env.next_actions()):
        c = zlib.crc32(a.tobytes(), c)
    return f"{c:08x}"


SHUFFLE_CAP_FLAG = 0x04  # M3_FLAG_SHUFFLE_CAP (include/m3.h), also the oracle's


def oracle_sample_check(env, shape, moves, goal, seed_base, stride, total_steps, k=256, idx=None):
    """After the clock stops: replay k boards spread over the shard (or the boards `idx`) through
    the C oracle (the checker, never the thing timed) from their first episode, through every
    same-step autoreset, to the step the env stopped at; compare board, score, moves, seed and the
    pre-drawn action."""
    import numpy as np

    from oracle import Oracle

    # the device's dead-board shuffle cap (1,024 per step): a board whose replay hits it has no
    # reference result (the reference keeps shuffling) and is counted apart, not compared
    o = Oracle(*shape, episode_shuffle_cap=1024)
    n = env.n
    if idx is None:
        idx = np.unique(np.linspace(0, n - 1, k).astype(np.int64))
    obs = env.observations().reshape(n, -1)
    score, mv, seeds, nxt = env.scores(), env.moves(), env.seeds(), env.next_actions()
    dev_flags = env.flags()
    bad = capped = 0
    for b in idx:
        rem, e = total_steps, 0
        want = None
        while True:
            seed = (seed_base + int(b) + e * stride) & 0xFFFFFFFF
            ep = o.random_episode(seed, moves, goal)
            if ep["n"] <= rem:  # a whole episode inside the replayed steps: its cap matters
                if ep["flags"] & SHUFFLE_CAP_FLAG:
                    break
                rem -= ep["n"]
                e += 1
                if rem == 0:  # autoreset in the step that finished the episode
                    seed = (seed + stride) & 0xFFFFFFFF
                    want = (o.init_board(seed)[0].reshape(-1), 0, 0, seed, o.random_episode(seed, 1, goal)["actions"][0])
                    break
            else:  # the replay ends inside this episode: only its first `rem` steps (and the next action) count
                part = o.random_episode(seed, rem, goal)
                if part["flags"] & SHUFFLE_CAP_FLAG:
                    break
                want = (part["final"].reshape(-1), int(part["rewards"].sum()), rem, seed, ep["actions"][rem])
                break
        if want is None:
            capped += 1
            continue
        got = (obs[b], score[b], mv[b], seeds[b], nxt[b])
        bad += not ((got[0] == want[0]).all() and all(int(x) == int(y) for x, y in zip(got[1:], want[1:])))
    # boards the device itself flagged at the shuffle cap in the last step (their replay is in `shuffle_capped`
    # when the oracle hits the cap within the replayed steps too)
    dev_capped = int(((dev_flags[idx] & SHUFFLE_CAP_FLAG) != 0).sum())
    return {"boards": int(len(idx)) - capped, "mismatches": int(bad), "steps_replayed": total_steps,
            "shuffle_capped": capped, "device_shuffle_capped_last_step": dev_capped}


def bench_rollouts(a):
    """--rollouts: device MCTS rollouts (m3_rollouts_device), one launch per timed step.

    n = --boards states (fresh seeded boards, n_actions = --moves, distinct cfg
    and rollout seeds) resident in HBM before timing (device buffers from
    libm3's own allocator, m3_dev_alloc); prints rollouts/s and the env-steps/s
    inside them, and the C oracle's rate on a bounded host sample (which also
    checks the gains)."""
    import numpy as np

    from match3tile import _native

    R, C, T = (int(x) for x in a.shape.split("x"))
    ctx = _native.Context(R, C, T)
    n = a.boards
    seeds = np.arange(1, n + 1, dtype=np.uint32)
    boards = np.empty((n, R * C), np.int8)
    chunk = 1 << 18
    for i in range(0, n, chunk):
        boards[i:i + chunk] = ctx.init_boards(seeds[i:i + chunk])[0].reshape(-1, R * C)
    rseeds = (np.arange(n, dtype=np.uint64) * 2654435761 % (2**31)).astype(np.uint32)
    ins = [ctx.device_array(x) for x in (boards, seeds, np.full(n, a.moves, np.int32), rseeds)]
    outs = [ctx.device_empty(n * 4) for _ in range(4)]
    L = _native.lib()

    def run():
        _native.check(L.m3_rollouts_device(ctx.handle, n, *[d.ptr for d in ins], *[o.ptr for o in outs], None))

    for _ in range(max(1, a.warmup)):
        run()
    _native.check(L.m3_ctx_synchronize(ctx.handle))
    t0 = time.perf_counter()
    for _ in range(a.steps):
        run()
    _native.check(L.m3_ctx_synchronize(ctx.handle))
    dt = (time.perf_counter() - t0) / a.steps
    gain = outs[0].to_host(np.int32, (n,))
    steps = int(outs[1].to_host(np.int32, (n,)).sum())
    res = {"metric": "MCTS rollouts/s (device, m3_rollouts_device)", "shape": a.shape, "rollouts": n,
           "moves": a.moves, "ms_per_launch": dt * 1e3, "rollouts_per_s": n / dt, "env_steps_per_s": steps / dt,
           "steps_per_rollout": steps / n}
    if not a.no_cpu_baseline:
        from oracle import Oracle

        o = Oracle(R, C, T)
        m = min(n, 20000)
        threads = min(16, os.cpu_count() or 1)
        t0 = time.perf_counter()
        r = o.rollouts(boards[:m].astype(np.int32), seeds[:m], a.moves, rseeds[:m], threads=threads)
        cdt = time.perf_counter() - t0
        assert (r["gain"] == gain[:m]).all(), "device rollouts differ from the oracle"
        res["cpu_baseline"] = {"rollouts_per_s": m / cdt, "env_steps_per_s": float(r["steps"].sum()) / cdt,
                               "cores": threads, "kind": "port", "sample": f"{m} rollouts, oracle/m3_oracle.c"}
    for d in ins + outs:
        d.free()
    ctx.close()
    print(json.dumps(res))


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--gpus", type=int, default=1)
    ap.add_argument("--steps", type=int, default=60)
    ap.add_argument("--warmup", type=int, default=10)
    ap.add_argument("--boards", type=int, default=1 << 20, help="boards per GPU (C3: 1,048,576)")
    ap.add_argument("--shape", default="9x9x6")
    ap.add_argument("--moves", type=int, default=20)
    ap.add_argument("--goal", type=int, default=500)
    ap.add_argument("--cpu-seconds", type=float, default=12.0)
    ap.add_argument("--no-cpu-baseline", action="store_true")
    ap.add_argument("--shards", type=int, default=2,
                    help="board shards per GPU, each on its own step + prefetch HIP stream (fastest: 2 with "
                         "--hw-queues >= 8, DESIGN §4)")
    ap.add_argument("--no-autoreset", action="store_true",
                    help="diagnostic only: boards stop at done (later steps are terminal no-ops); not the headline")
    ap.add_argument("--hw-queues", type=int, default=8,
                    help="GPU_MAX_HW_QUEUES for this process (HIP reads it at init; <= 32): 2 shards use "
                         "5 streams (context + 2 x (step, prefetch)), each on its own hardware queue")
    ap.add_argument("--rollouts", action="store_true",
                    help="secondary bench: device MCTS rollouts (f3) instead of the env step")
    ap.add_argument("--dry-rendezvous", action="store_true",
                    help="test hook: run the N>1 rendezvous and unique-id broadcast with a stand-in id, print "
                         "what each rank received and exit before any GPU work (tests/test_bench_cpu.py)")
    ap.add_argument("--check-boards", type=int, default=256,
                    help="boards per rank replayed through the C oracle after the clock stops (0: none)")
    ap.add_argument("--gather", choices=("final", "step"), default="final",
                    help="N > 1: RCCL all-gather of the packed reward/truncated/done words once, after the last "
                         "timed step (final: BASELINE north_star's 'final reward/done gather', the headline) or "
                         "after every step (step); both inside the timed region")
    ap.add_argument("--allow-stale-lib", action="store_true",
                    help="if `make` fails, time the library already built (recorded as build.stale in the line)")
    args = ap.parse_args()
    if args.hw_queues is not None:
        if not 1 <= args.hw_queues <= 32:
            raise SystemExit("--hw-queues must be in [1, 32]")
        os.environ["GPU_MAX_HW_QUEUES"] = str(args.hw_queues)
    if args.rollouts:
        return bench_rollouts(args)
    if args.gpus < 1:
        raise SystemExit("--gpus must be >= 1")
    if "WORLD_SIZE" not in os.environ and args.gpus > 1:
        return spawn_ranks(args)  # one process per GPU, this one stays off the GPU

    rank = int(os.environ.get("RANK", "0"))
    world = int(os.environ.get("WORLD_SIZE", "1"))
    local = int(os.environ.get("LOCAL_RANK", "0"))
    if world != args.gpus:
        raise SystemExit(f"bench.py: --gpus {args.gpus} but the launcher started {world} rank(s) (WORLD_SIZE); "
                         f"run `python bench.py --gpus {args.gpus}` (it starts the ranks) or a launcher with "
                         f"--nproc-per-node {args.gpus}")
    rows, cols, types = (int(x) for x in args.shape.split("x"))

    dist = dist_setup(rank, world)
    if args.dry_rendezvous:
        import hashlib

        uid = share_unique_id(dist, rank, lambda: os.urandom(128)) if dist else os.urandom(128)
        from match3tile.distributed import timed_steps

        stub = _StubEnv()
        st, end = step_fns(stub, world, args.gather)
        timed_steps(st, stub.synchronize, args.steps, args.warmup, dist, on_end=end)
        line = json.dumps({"rank": rank, "world": world, "local_rank": local, "gather": args.gather,
                           "stub_steps": stub.steps, "stub_gathers": stub.gathers,
                           "dist_world": dist.get_world_size() if dist else 1,
                           "spawned": os.environ.get("M3_SPAWNED") == "1", "torch_loaded": "torch" in sys.modules,
                           "id_bytes": len(uid), "id_sha256": hashlib.sha256(uid).hexdigest()})
        sys.stdout.flush()
        os.write(sys.stdout.fileno(), (line + "\n").encode())  # one write: the ranks share the pipe
        dist_close(dist, rank)
        return

    # no-op when libm3.so is up to date with its sources and compile flags (build/flags.stamp);
    # A/B variants are separate files (make variant), selected with M3_LIB (then nothing is
    # built). The ranks of one node share the tree: they take turns under a file lock, so at
    # most one builds. A failed build stops the bench unless --allow-stale-lib.
    build = {"library": os.environ.get("M3_LIB", os.path.join(PKG, "build", "libm3.so")), "make_rc": None,
             "stale": False}
    if "M3_LIB" not in os.environ:
        import fcntl

        os.makedirs(os.path.join(PKG, "build"), exist_ok=True)
        with open(os.path.join(PKG, "build", ".make.lock"), "w") as lk:
            fcntl.flock(lk, fcntl.LOCK_EX)
            r = subprocess.run(["make", "-s", "-C", PKG])
            fcntl.flock(lk, fcntl.LOCK_UN)
        build["make_rc"] = r.returncode
        if r.returncode != 0:
            if not (args.allow_stale_lib and os.path.exists(build["library"])):
                raise SystemExit("bench.py: building libm3.so failed (pass --allow-stale-lib to time the old one)")
            build["stale"] = True
            print("bench.py: make failed; timing the existing build/libm3.so (build.stale)", file=sys.stderr)
    from match3tile import _native
    from match3tile.batched import BatchedMatch3Env
    from match3tile.distributed import seed_plan, timed_steps

    ndev = _native.device_count()
    if local >= ndev:
        raise SystemExit(f"bench.py: rank {rank} wants GPU {local} but {ndev} GPU(s) are visible "
                         f"(--gpus {args.gpus} needs {args.gpus})")
    uid = share_unique_id(dist, rank, BatchedMatch3Env.comm_unique_id) if dist else None
    B = args.boards
    seed_base, seed_stride = seed_plan(rank, world, B)
    env = BatchedMatch3Env(B, rows, cols, types, num_moves=args.moves, env_goal=args.goal, device=local,
                           seed_base=seed_base, autoreset=not args.no_autoreset, seed_stride=seed_stride,
                           shards=args.shards)
    if dist:
        env.init_comm(uid, world, rank)

    step, final_gather = step_fns(env, world, args.gather)
    elapsed, elapsed_local = timed_steps(step, env.synchronize, args.steps, args.warmup, dist,
                                         on_start=lambda: env.enable_timing(args.steps), on_end=final_gather,
                                         return_local=True)
    rank_ms = dist.allgather_obj(elapsed_local / args.steps * 1e3) if dist else [elapsed_local / args.steps * 1e3]
    kms = env.kernel_ms()
    kms_step = env.kernel_ms(step_kernel_only=True)
    stats = env.stats()
    # ---- after the clock: attest the run (nothing below is timed) ----
    nranks = env.comm_size()
    gather_ok = gather_check(env, dist, rank, world) if dist else None
    parity = {"digest": state_digest(env)}
    if dist:
        parity["digest_all_ranks"] = dist.allgather_obj(parity["digest"])
    if args.check_boards and not args.no_autoreset:
        chk = oracle_sample_check(env, (rows, cols, types), args.moves, args.goal, seed_base, seed_stride,
                                  args.warmup + args.steps, args.check_boards)
        if dist:
            nb, nm, nc = dist.allsum([chk["boards"], chk["mismatches"], chk["shuffle_capped"]])
            chk.update(boards=nb, mismatches=nm, shuffle_capped=nc, ranks=world)
        parity["oracle_sample"] = chk
        parity["oracle_match"] = chk["mismatches"] == 0 and chk["boards"] > 0
    env.close()

    if rank != 0:
        dist_close(dist, rank)
        return

    total_steps = world * B * args.steps
    value = total_steps / elapsed
    step_s = elapsed / args.steps
    avg_kernel_s = float(kms.mean()) / 1e3 if len(kms) else float("nan")
    avg_step_kernel_s = float(kms_step.mean()) / 1e3 if len(kms_step) else float("nan")
    # one launch of the step pipeline processes one shard (B / shards boards, contiguous, the last may be short)
    shard_boards = -(-B // stats["shards"])
    alg = algorithmic_bytes_per_step(rows, cols)
    bytes_per_launch = shard_boards * alg
    prof = load_profile(args.shape, B, shard_boards, args.steps, args.warmup)
    dom = prof.get("dominant")
    # HBM roofline of the dominant kernel (k_env_step) in the contract's form: algorithmic bytes per
    # launch (2RC + 21 per env-step) over its average launch duration, both live (HIP
    # events on the shard's stream around k_env_step); traffic = the committed PMC pass's HBM bytes
    hbm = {
        "kernel": "k_env_step",
        "achieved": bytes_per_launch / avg_step_kernel_s / 1e9, "peak": HBM_PEAK_GBS, "unit": "GB/s",
        "frac": bytes_per_launch / avg_step_kernel_s / 1e9 / HBM_PEAK_GBS,
        "traffic": dom["hbm_bytes_per_launch"] if dom else None,
        "traffic_bytes_per_board": dom["hbm_bytes_per_board"] if dom else None,
        "algorithmic_bytes_per_launch": bytes_per_launch, "boards_per_launch": shard_boards,
        "avg_kernel_ms": avg_step_kernel_s * 1e3,
        "note": f"{alg} B per {rows}x{cols} env-step (2RC + 21); the path is integer VALU-bound, see roofline"}
    pipeline = {
        # one shard's whole step pipeline: k_env_step + k_env_cont_grid (the long cascades) + k_env_fix,
        # bracketed by HIP events on the shard's stream
        "kernels": "k_env_step + k_env_cont_grid + k_env_fix", "avg_ms": avg_kernel_s * 1e3,
        "achieved_gbs": bytes_per_launch / avg_kernel_s / 1e9,
        "traffic": prof.get("pipeline", {}).get("hbm_bytes_per_launch"),
        "aggregate_gbs": value / world * alg / 1e9,
        "aggregate_frac": value / world * alg / 1e9 / HBM_PEAK_GBS}
    if dom:
        # What binds: VALU issue. The dominant kernel's wave64 VALU instructions (committed PMC pass of
        # this same command, profiles/<round>_dispatch.csv) against the chip's VALU issue peak: per step
        # over the step's wall time (the two shards' launches overlap, so the per-launch quotient is
        # about half the chip's rate), per launch over the live launch duration beside it; SIMT = active
        # lanes per VALU instruction (SQ_THREAD_CYCLES_VALU / 64 SQ_ACTIVE_INST_VALU), lane_frac = frac x SIMT.
        vw = dom["valu_insts_per_step"] / step_s
        roofline = {
            "bound": "valu", "kernel": "k_env_step",
            "achieved": vw, "peak": VALU_PEAK_WAVE_INSTR_S, "unit": "wave64 VALU instr/s",
            "frac": vw / VALU_PEAK_WAVE_INSTR_S,
            "frac_per_launch": dom["valu_insts_per_launch"] / avg_step_kernel_s / VALU_PEAK_WAVE_INSTR_S,
            "simt": dom["simt"], "lane_frac": vw / VALU_PEAK_WAVE_INSTR_S * dom["simt"],
            "traffic": dom["hbm_bytes_per_launch"],
            "valu_insts_per_launch": dom["valu_insts_per_launch"], "valu_insts_per_step": dom["valu_insts_per_step"],
            "wait_frac": dom["wait_frac"], "vmem_wr_per_wave": dom["vmem_wr_per_wave"],
            "ms_per_step": step_s * 1e3,
            "how": "frac = valu_insts_per_step / (ms_per_step / 1e3) / peak; frac_per_launch = valu_insts_per_launch "
                   "/ hbm.avg_kernel_ms (live) / peak; peak = 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 "
                   "VALU instruction; counts from " + prof.get("dispatch_csv", "?"),
            "whole_step_frac": prof["valu_insts_per_step"]["total"] / step_s / VALU_PEAK_WAVE_INSTR_S,
            "hbm": hbm, "pipeline": pipeline}
    else:
        roofline = dict(hbm, bound="hbm", valu=None, hbm=hbm, pipeline=pipeline)
    out = {
        "metric": METRIC,
        "value": value,
        "unit": "env-steps/s",
        "n_gpus": world,
        "steps": args.steps,
        "warmup": args.warmup,
        "ms_per_step": elapsed / args.steps * 1e3,
        "higher_is_better": True,
        "scaling": "weak",
        "vs_baseline": None,
        "dtype": "int8",
        "data": "synthetic: seeded initial boards (seed = 1 + board index), seeded random_action per move "
                "(samplerTasks.random_task contract), 20-move episodes, autoreset with seed += n_boards",
        "config": {
            "workload": f"{'C3' if (rows, cols) == (9, 9) else 'C4'}: {B:,} boards per GPU, {rows}x{cols}x{types}, Match3Env.step x {args.steps} "
                        "(step kernel + overflow fixup + autoreset; N>1: RCCL reward/done all-gather "
                        + ("once after the last step" if args.gather == "final" else "after every step") + ")",
            "boards_per_gpu": B,
            "shape": args.shape,
            "num_moves": args.moves,
            "env_goal": args.goal,
            "parallelism": f"dp{world}",
            "shards_per_gpu": stats["shards"],
            "hw_queues": args.hw_queues,
            "autoreset": not args.no_autoreset,
        },
        "nranks": nranks,
        "gather": (args.gather if world > 1 else None),
        "ms_per_step_per_rank": rank_ms,
        "gather_ok": gather_ok,
        "parity": parity,
        "path_stats": {"autoresets": stats["autoresets"], "reset_recomputes": stats["reset_recomputes"],
                       "step_recomputes": stats["step_recomputes"]},
        "roofline": roofline,
        "build": build,
    }
    if world == 1 and not args.no_cpu_baseline:
        out["cpu_baseline"] = cpu_baseline(rows, cols, types, args.moves, args.goal, args.cpu_seconds)
    print(json.dumps(out), flush=True)
    dist_close(dist, rank)


if __name__ == "__main__":
    sys.exit(main())
