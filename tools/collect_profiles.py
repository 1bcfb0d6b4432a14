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


def last_json(path):
    return json.loads(open(path).read().strip().splitlines()[-1])


bench = last_json(os.path.join(src, "bench.log"))
json.dump(bench, open(os.path.join(P, f"{tag}_bench.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(P, f"{tag}_kernel_stats.csv"))
pmc = subprocess.run([sys.executable, os.path.join(ROOT, "tools", "pmc_summary.py"), src],
                     capture_output=True, text=True, check=True).stdout
open(os.path.join(P, f"{tag}_pmc.txt"), "w").write(pmc)

PIPE = ("k_env_step", "k_env_cont", "k_env_cont_grid", "k_env_fix")
# every kernel that runs inside a timed step: the step pipeline and the autoreset (prefetch) kernels
STEP_KERNELS = PIPE + ("k_init", "k_init_coop", "k_init_fix_lane", "k_init_chain2")
agg = collections.defaultdict(lambda: collections.defaultdict(list))
allk = collections.defaultdict(lambda: collections.defaultdict(list))
for f in glob.glob(f"{src}/**/*_counter_collection.csv", recursive=True):
    for r in csv.DictReader(open(f)):
        name = r["Kernel_Name"]
        k = [p for p in PIPE if p + "<" in name]
        if k and r["Counter_Name"] in ("FETCH_SIZE", "WRITE_SIZE", "SQ_INSTS_VALU", "SQ_INSTS_SALU"):
            agg[r["Counter_Name"]][k[0]].append(float(r["Counter_Value"]))
        k2 = [p for p in STEP_KERNELS if p + "<" in name]
        if k2 and r["Counter_Name"] == "SQ_INSTS_VALU":
            allk[k2[0]][r.get("Dispatch_Id", len(allk[k2[0]]))].append(float(r["Counter_Value"]))


def per_launch(counter):  # mean per launch of each pipeline kernel, summed over the pipeline
    return sum(sum(v) / len(v) for v in agg[counter].values())


def valu_per_step():
    """wave64 VALU instructions of one timed step over every kernel it runs: per kernel the median
    per launch (the per-step launches outnumber the env's initial reset launches ~25:1) times its
    launches per step (one per board shard)."""
    shards = bench["config"].get("shards_per_gpu", 1)
    per = {}
    for k, d in allk.items():
        vals = sorted(sum(v) for v in d.values())  # (a counter may come per XCD / SE: summed per dispatch)
        if vals:
            per[k] = vals[len(vals) // 2] * shards
    return {"kernels": sorted(per), "per_kernel": per, "total": sum(per.values()), "shards": shards,
            "how": "median SQ_INSTS_VALU per launch x launches per step (shards), rocprofv3 --pmc pass"}


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
           "salu_insts_per_launch": per_launch("SQ_INSTS_SALU"),
           "source": f"profiles/{tag}_pmc.txt (rocprofv3 --pmc passes: FETCH_SIZE and WRITE_SIZE for the bytes, "
                     "the SQ_INSTS_VALU / SQ_INSTS_SALU group for the instruction counts)",
           "correction": "2 x FETCH_SIZE (gfx950 wide-read calibration) + WRITE_SIZE"}
# one summary per board shape: traffic.json (the headline 9x9x6) / traffic_<shape>.json
tname = "traffic.json" if cfg["shape"] == "9x9x6" else f"traffic_{cfg['shape']}.json"
json.dump(traffic, open(os.path.join(P, tname), "w"), indent=1)
print(json.dumps(traffic, indent=1))
