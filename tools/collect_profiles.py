#!/usr/bin/env python3
"""Copy a tools/gpu_profile.sh run into profiles/ (tracked) and derive the roofline inputs bench.py reads.

    python3 tools/collect_profiles.py gpurun_out/<tag>/s9 <round-tag>      (9x9x6 -> profiles/traffic.json)
    python3 tools/collect_profiles.py gpurun_out/<tag>/s16 <round-tag>     (16x16x8 -> traffic_16x16x8.json)

Every run is the driver's own command (bench.py --gpus 1 --steps 20 --warmup 5 [16x16x8 shape]); the
kernel trace and each --pmc pass are separate runs of it. Writes:
  profiles/<rt>[_16x16x8]_bench.json         the bench line of the un-profiled run
  profiles/<rt>[_16x16x8]_kernel_stats.csv   rocprofv3 --kernel-trace --stats
  profiles/<rt>[_16x16x8]_dispatch.csv       one row per dispatch of the TIMED window: kernel, every counter
                                            of every pass (dispatches of one kernel matched across passes
                                            by their order), and the kernel-trace duration
  profiles/traffic[_16x16x8].json           per-kernel sums over that window / timed steps, and the
                                            dominant kernel's (k_env_step) per-launch figures
Every number in traffic*.json is a sum or ratio of columns of the dispatch CSV (see "how" fields).
HBM bytes = 2 x FETCH_SIZE + WRITE_SIZE (KB -> bytes; the factor 2 is MI355X_MICROARCH.md's gfx950
correction for wide coalesced reads, which FETCH_SIZE reports at half).
"""
import collections
import csv
import glob
import json
import os
import re
import shutil
import sys

src, rtag = sys.argv[1], sys.argv[2]
ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
P = os.path.join(ROOT, "profiles")
KERNELS = ("k_env_step", "k_env_cont_grid", "k_env_fix", "k_init", "k_init_coop", "k_init_fix_lane",
           "k_reset_stream", "k_reset_tiles")
VALU_PEAK = 256 * 4 * 2.4e9 / 2  # wave64 VALU instructions/s: 256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles
HBM_PEAK = 8000e9  # B/s


def last_json(path):  # (rocprofv3 logs its own lines after the bench line)
    return json.loads([ln for ln in open(path).read().splitlines() if ln.startswith("{")][-1])


def kname(name):
    k = [p for p in KERNELS if re.search(r"\b" + p + "<", name)]
    return k[0] if k else re.sub(r"\(.*", "", name).replace("void ", "")


bench = last_json(os.path.join(src, "bench.log"))
shape = bench["config"]["shape"]
sfx = "" if shape == "9x9x6" else f"_{shape}"
json.dump(bench, open(os.path.join(P, f"{rtag}{sfx}_bench.json"), "w"), indent=1)
shutil.copy(os.path.join(src, "kt", "kt_kernel_stats.csv"), os.path.join(P, f"{rtag}{sfx}_kernel_stats.csv"))


def dispatches(rows, id_key, name_key):
    """[(dispatch id, kernel)] in dispatch order"""
    seen = {}
    for r in rows:
        seen.setdefault(int(r[id_key]), kname(r[name_key]))
    return sorted(seen.items())


def timed_ids(order, shards, steps):
    """dispatch ids of the timed window: from the first dispatch of the last `steps` timed steps
    (the (steps * shards)-th k_env_step from the end) to the last dispatch"""
    step_ids = [i for i, k in order if k == "k_env_step"]
    first = step_ids[-steps * shards]
    return {i for i, _ in order if i >= first}


shards, steps, warm = bench["config"]["shards_per_gpu"], bench["steps"], bench["warmup"]
# per pass: counter values per dispatch, then matched across passes by (kernel, occurrence index)
table = collections.defaultdict(dict)  # (kernel, occurrence) -> {column: value}
for f in sorted(glob.glob(os.path.join(src, "p_*", "**", "*_counter_collection.csv"), recursive=True)):
    rows = list(csv.DictReader(open(f)))
    order = dispatches(rows, "Dispatch_Id", "Kernel_Name")
    tids = timed_ids(order, shards, steps)
    occ, key = collections.Counter(), {}
    for i, k in order:
        key[i] = (k, occ[k])
        occ[k] += 1
    vals = collections.defaultdict(float)
    for r in rows:
        vals[(int(r["Dispatch_Id"]), r["Counter_Name"])] += float(r["Counter_Value"])  # (summed per dispatch)
    for (i, c), v in vals.items():
        if i in tids:
            table[key[i]][c] = v
            table[key[i]]["timed"] = 1
# kernel-trace durations, matched the same way
kt = list(csv.DictReader(open(glob.glob(os.path.join(src, "kt", "*kernel_trace.csv"))[0])))
order = sorted({int(r["Dispatch_Id"]): (kname(r["Kernel_Name"]), int(r["End_Timestamp"]) - int(r["Start_Timestamp"]))
                for r in kt}.items())
tids = timed_ids([(i, k) for i, (k, _) in order], shards, steps)
occ = collections.Counter()
for i, (k, d) in order:
    if i in tids and (k, occ[k]) in table:
        table[(k, occ[k])]["duration_ns"] = d
    occ[k] += 1

cols = sorted({c for v in table.values() for c in v if c != "timed"})
csv_path = f"profiles/{rtag}{sfx}_dispatch.csv"
with open(os.path.join(ROOT, csv_path), "w") as f:
    f.write("kernel,occurrence," + ",".join(cols) + "\n")
    for (k, n), v in sorted(table.items(), key=lambda kv: (kv[0][0], kv[0][1])):
        f.write(f"{k},{n}," + ",".join(f"{v.get(c, 0):.0f}" for c in cols) + "\n")

per = collections.defaultdict(lambda: collections.defaultdict(float))
cnt = collections.Counter()
for (k, _), v in table.items():
    cnt[k] += 1
    for c in cols:
        per[k][c] += v.get(c, 0.0)
per_step = {k: {c: x / steps for c, x in d.items()} for k, d in per.items()}
per_launch = {k: {c: x / cnt[k] for c, x in d.items()} for k, d in per.items()}

d = per_launch["k_env_step"]
boards_per_launch = -(-bench["config"]["boards_per_gpu"] // shards)
R, C = (int(x) for x in shape.split("x")[:2])
alg = 2 * R * C + 21
hbm = 2 * d.get("FETCH_SIZE", 0) * 1024 + d.get("WRITE_SIZE", 0) * 1024
simt = d["SQ_THREAD_CYCLES_VALU"] / (64.0 * d["SQ_ACTIVE_INST_VALU"])
ms_step = bench["ms_per_step"]
valu_step = per_step["k_env_step"]["SQ_INSTS_VALU"]
dominant = {
    "kernel": "k_env_step",
    "launches": cnt["k_env_step"],
    "boards_per_launch": boards_per_launch,
    "valu_insts_per_launch": d["SQ_INSTS_VALU"],
    "valu_insts_per_step": valu_step,
    "trace_avg_ms": d.get("duration_ns", 0) / 1e6,
    "valu_frac_trace": d["SQ_INSTS_VALU"] / (d["duration_ns"] / 1e9) / VALU_PEAK,
    "valu_frac_wall": valu_step / (ms_step / 1e3) / VALU_PEAK,
    "simt": simt,
    "lane_frac_wall": valu_step / (ms_step / 1e3) / VALU_PEAK * simt,
    "hbm_bytes_per_launch": hbm,
    "hbm_bytes_per_board": hbm / boards_per_launch,
    "algorithmic_bytes_per_board": alg,
    "hbm_frac_trace": hbm / (d["duration_ns"] / 1e9) / HBM_PEAK,
    "wait_frac": d["SQ_WAIT_ANY"] / d["SQ_WAVE_CYCLES"],
    "vmem_wr_per_wave": d["SQ_INSTS_VMEM_WR"] / d["SQ_WAVES"],
    "vmem_rd_per_wave": d["SQ_INSTS_VMEM_RD"] / d["SQ_WAVES"],
    "lds_bank_conflict_per_lds_inst": d["SQ_LDS_BANK_CONFLICT"] / max(1.0, d["SQ_INSTS_LDS"]),
    "bench_ms_per_step": ms_step,
    "how": {
        "valu_frac_wall": "valu_insts_per_step (sum of SQ_INSTS_VALU over the timed k_env_step dispatches / steps) "
                          "/ bench_ms_per_step / VALU peak (256 CUs x 4 SIMDs x 2.4 GHz / 2 cycles per wave64 instruction)",
        "valu_frac_trace": "valu_insts_per_launch / trace_avg_ms (the kernel trace's mean duration; the two shards' "
                           "launches overlap, so this is a per-launch figure, about half the chip's rate)",
        "simt": "sum SQ_THREAD_CYCLES_VALU / (64 x sum SQ_ACTIVE_INST_VALU) over the timed k_env_step dispatches",
        "lane_frac_wall": "valu_frac_wall x simt (active lanes' share of the VALU issue peak)",
        "hbm": "2 x FETCH_SIZE + WRITE_SIZE per launch (KB -> B), gfx950 wide-read correction"},
}
pipe = [k for k in ("k_env_step", "k_env_cont_grid", "k_env_fix") if k in per_launch]
pipe_hbm = sum(2 * per_launch[k].get("FETCH_SIZE", 0) * 1024 + per_launch[k].get("WRITE_SIZE", 0) * 1024 for k in pipe)
valu_all = {k: v["SQ_INSTS_VALU"] for k, v in per_step.items() if k in KERNELS and "SQ_INSTS_VALU" in v}
tot = sum(valu_all.values())
dur = {k: v.get("duration_ns", 0) for k, v in per.items() if k in KERNELS}
traffic = {
    "shape": shape, "boards": bench["config"]["boards_per_gpu"], "steps": steps, "warmup": warm,
    "shards": shards, "boards_per_launch": boards_per_launch,
    "dominant": dominant,
    "pipeline": {"kernels": pipe, "hbm_bytes_per_launch": pipe_hbm, "hbm_bytes_per_board": pipe_hbm / boards_per_launch},
    "valu_insts_per_step": {"per_kernel": valu_all, "total": tot, "share": {k: v / tot for k, v in valu_all.items()},
                            "how": "sum of SQ_INSTS_VALU over every timed dispatch / steps"},
    "duration_share": {k: v / sum(dur.values()) for k, v in dur.items()},
    "dispatch_csv": csv_path,
    "source": f"gpurun_out pass of tools/gpu_profile.sh -> {csv_path}",
}
tname = "traffic.json" if shape == "9x9x6" else f"traffic_{shape}.json"
json.dump(traffic, open(os.path.join(P, tname), "w"), indent=1)
print(json.dumps(traffic, indent=1))
