#!/usr/bin/env python3
"""Calibrate the C oracle against the reference's own Python step path, on THIS container's cores.

bench.py's cpu_baseline times oracle/m3_oracle.c (a bit-exact scalar port of the
reference step) on the GPU host, because the reference Python cannot travel
there. SURVEY.md §8(d) turns that into a "reference-Python-equivalent on the
GPU host" figure: time both here on the same workload, and scale the GPU host's
C-port rate by (reference Python / C port) measured here. This script measures
that ratio and writes profiles/cpu_calibration.json, which bench.py reads.

Workload (both sides): samplerTasks.random_task episodes (samplerTasks.py:9-14),
9x9x6, 20 moves: BoardV2(20, BoardConfig(seed)) + 20 x (legal_actions,
np.random.choice, apply_action), seeds 1, 2, ...

    PYTHONPATH=/root/reference python3 -B tools/calibrate_cpu.py [--seconds 20]
"""
import argparse
import json
import multiprocessing as mp
import os
import sys
import time

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "oracle"))
sys.path.insert(0, os.path.join(ROOT, "tools"))


def c_port_rate(threads, seconds):
    from oracle import Oracle

    o = Oracle(9, 9, 6)
    probe = 512 * threads
    t0 = time.perf_counter()
    o.run_episodes(list(range(1, probe + 1)), 20, 500, threads)
    n = max(probe, int(probe * seconds / max(time.perf_counter() - t0, 1e-3)))
    t0 = time.perf_counter()
    steps, _ = o.run_episodes(list(range(1, n + 1)), 20, 500, threads)
    dt = time.perf_counter() - t0
    return {"env_steps_per_s": steps / dt, "steps": int(steps), "seconds": dt, "threads": threads}


def py_rate(procs, seconds):
    from time_reference import worker

    with mp.Pool(procs) as pool:
        out = pool.map(worker, [(1 + 1_000_000 * i, seconds) for i in range(procs)])
    steps = sum(o[0] for o in out)
    wall = max(o[2] for o in out)
    return {"env_steps_per_s": steps / wall, "steps": steps, "seconds": wall, "procs": procs}


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--seconds", type=float, default=20.0)
    a = ap.parse_args()
    cores = len(os.sched_getaffinity(0))
    res = {"what": "samplerTasks.random_task episodes, 9x9x6, 20 moves (env_goal 500 on the C side: "
                   "random_task has no goal, 20-move episodes reach 500 in <1% of seeds)",
           "host": "build container", "nproc": os.cpu_count(), "cores": cores,
           "c_port_1": c_port_rate(1, a.seconds), f"c_port_{cores}": c_port_rate(cores, a.seconds),
           "ref_python_1": py_rate(1, a.seconds), f"ref_python_{cores}": py_rate(cores, a.seconds)}
    res["ratio_1core"] = res["ref_python_1"]["env_steps_per_s"] / res["c_port_1"]["env_steps_per_s"]
    res["ratio_allcores"] = (res[f"ref_python_{cores}"]["env_steps_per_s"]
                             / res[f"c_port_{cores}"]["env_steps_per_s"])
    out = os.path.join(ROOT, "profiles", "cpu_calibration.json")
    with open(out, "w") as f:
        json.dump(res, f, indent=1)
    print(json.dumps(res))


if __name__ == "__main__":
    main()
