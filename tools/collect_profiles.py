#!/usr/bin/env python3
"""Copy a gpu_round.sh run's evidence into profiles/ (tracked) and derive profiles/traffic.json.

    python3 tools/collect_profiles.py gpurun_out/<tag> <round-tag>

Writes profiles/<round-tag>_bench.json (the bench line), <round-tag>_kernel_stats.csv
(rocprofv3 --kernel-trace --stats of the same bench command), <round-tag>_pmc.txt
(per-kernel PMC means, one rocprofv3 pass per counter group) and traffic.json
(traffic_<shape>.json for a shape other than 9x9x6):
HBM bytes per launch of one shard's step pipeline (k_env_step + k_env_cont(_grid) + k_env_fix, the
two kernels bench.py's HIP events bracket) = 2 * FETCH_SIZE + WRITE_SIZE (KB ->
bytes), the factor 2 being MI355X_MICROARCH.md's gfx950 correction for wide
coalesced reads (FETCH_SIZE reports half of them; narrower accesses are
uncalibrated).
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import subprocess
import sys

src, tag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")


def last_json(path):  # (rocprofv3 logs its own lines after the bench line)
    return json.loads([ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1])


bench = last_json(os.path.join(src, "bench.log"))
json.dump(bench, open(os.path.join(P, f"{tag}_bench.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(P, f"{tag}_kernel_stats.csv"))
pmc = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src],
                     capture_output=True, text=True, check=True).stdout
open(os.path.join(P, f"{tag}_pmc.txt"), "w").write(pmc)

PIPE = ("k_env_step", "k_env_cont", "k_env_cont_grid", "k_env_fix")
# every kernel that runs inside a timed step: the step pipeline and the autoreset (prefetch) kernels
STEP_KERNELS = PIPE + ("k_init", "k_init_coop", "k_init_fix_lane", "k_init_chain2", "k_reset_stream", "k_reset_tiles")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
# the SQ pass, per dispatch: (dispatch id, kernel, SQ_INSTS_VALU summed over its records)
disp = collections.defaultdict(lambda: [None, 0.0])
sq_dir = None
for f in glob.glob(f"{src}/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = [p for p in PIPE if p + "<" in name]
        if k and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_SALU"):
            agg[r["Counter_Name"]][k[0]].append(float(r["Counter_Value"]))
        if r["Counter_Name"] == "SQ_INSTS_VALU":
            sq_dir = os.path.dirname(os.path.dirname(f))
            k2 = [p for p in STEP_KERNELS if p + "<" in name]
            d = disp[int(r["Dispatch_Id"])]
            d[0] = k2[0] if k2 else re.sub(r"\(.*", "", name).replace("void ", "")
            d[1] += float(r["Counter_Value"])  # (a counter may come per XCD / SE: summed per dispatch)


def per_launch(counter):  # mean per launch of each pipeline kernel, summed over the pipeline
    return sum(sum(v) / len(v) for v in agg[counter].values())


def valu_per_step():
    """wave64 VALU instructions of one timed step over every kernel it runs, SUMMED over the dispatches
    of the timed window of the profiled bench command / its timed steps. The window starts at the first
    dispatch of timed step `warmup` (the (warmup * shards)-th k_env_step) and runs to the last dispatch
    (nothing is launched after the timed steps). The per-dispatch rows go to profiles/<tag>_valu_dispatch.csv."""
    sq_log = glob.glob(os.path.join(src, "sq.log"))
    run = last_json(sq_log[0]) if sq_log else bench  # the bench line of the profiled command itself
    shards = run["config"].get("shards_per_gpu", 1)
    warm, steps = run["warmup"], run["steps"]
    ids = sorted(disp)
    step_ids = [i for i in ids if disp[i][0] == "k_env_step"]
    if len(step_ids) < (warm + steps) * shards:
        raise SystemExit(f"{len(step_ids)} k_env_step dispatches, expected {(warm + steps) * shards}")
    first = step_ids[-steps * shards]  # the timed steps are the last `steps` of the run
    per = collections.defaultdict(float)
    with open(os.path.join(P, f"{tag}_valu_dispatch.csv"), "w") as f:
        f.write("dispatch_id,kernel,sq_insts_valu,timed\n")
        for i in ids:
            k, v = disp[i]
            timed = i >= first
            f.write(f"{i},{k},{v:.0f},{int(timed)}\n")
            if timed and k in STEP_KERNELS:
                per[k] += v / steps
    total = sum(per.values())
    return {"kernels": sorted(per), "per_kernel": dict(per), "share": {k: v / total for k, v in per.items()},
            "total": total, "shards": shards, "timed_steps": steps, "warmup": warm,
            "dispatch_csv": f"profiles/{tag}_valu_dispatch.csv",
            "how": "sum of SQ_INSTS_VALU over every dispatch of the timed window (rocprofv3 --pmc, per-dispatch "
                   "records) / timed steps"}


def duration_share():
    """each step kernel's share of the kernel-trace duration (rocprofv3 --stats of the same command;
    the kernels overlap across streams, so these are shares of summed durations, not of wall time)"""
    rows = list(csv.DictReader(open(os.path.join(src, "kt", "kt_kernel_stats.csv"))))
    dur = collections.defaultdict(float)
    for r in rows:
        k = [p for p in STEP_KERNELS if p + "<" in r["Name"]]
        if k:
            dur[k[0]] += float(r["TotalDurationNs"])
    t = sum(dur.values())
    return {k: v / t for k, v in dur.items()}


fetch = per_launch("FETCH_SIZE") * 1024
write = per_launch("WRITE_SIZE") * 1024
cfg = bench["config"]
rl = bench["roofline"].get("hbm", bench["roofline"])  # (the HBM block sits inside a VALU-bound roofline)
traffic = {"shape": cfg["shape"], "boards": cfg["boards_per_gpu"],
           "kernel": "k_env_step + k_env_cont(_grid) + k_env_fix (the kernels of one shard's step pipeline)",
           "boards_per_launch": rl.get("boards_per_launch"),
           "fetch_size_bytes": fetch, "write_size_bytes": write,
           "hbm_bytes_per_launch": 2 * fetch + write,
           "bytes_per_board": (2 * fetch + write) / rl.get("boards_per_launch", cfg["boards_per_gpu"]),
           "valu_insts_per_launch": per_launch("SQ_INSTS_VALU"),
           "valu_insts_per_step": valu_per_step(),
           "duration_share": duration_share(),
           "salu_insts_per_launch": per_launch("SQ_INSTS_SALU"),
           "source": f"profiles/{tag}_pmc.txt (rocprofv3 --pmc passes: FETCH_SIZE and WRITE_SIZE for the bytes, "
                     "the SQ_INSTS_VALU / SQ_INSTS_SALU group for the instruction counts)",
           "correction": "2 x FETCH_SIZE (gfx950 wide-read calibration) + WRITE_SIZE"}
# one summary per board shape: traffic.json (the headline 9x9x6) / traffic_<shape>.json
tname = "traffic.json" if cfg["shape"] == "9x9x6" else f"traffic_{cfg['shape']}.json"
json.dump(traffic, open(os.path.join(P, tname), "w"), indent=1)
print(json.dumps(traffic, indent=1))
