#!/usr/bin/env python3
"""Collect the bench lines of A/B runs (gpurun_out/<tag>/*.log written by tools/gpu_ab.sh or
gpu_ab_raw.sh) into one text table: run, library, shape, env-steps/s, ms/step, oracle_match.

    python3 tools/ab_table.py r05c r05d ... > profiles/r05_ab.txt
"""
import glob
import json
import os
import sys

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
for tag in sys.argv[1:]:
    rows = []
    for f in sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "*.log")),
                    key=lambda p: (len(os.path.basename(p)), p)):
        try:
            d = json.loads(open(f).read().strip().splitlines()[-1])
        except (ValueError, IndexError):
            continue
        if "value" not in d:
            continue
        lib = os.path.basename(d.get("build", {}).get("library", "?"))
        rows.append(f"{tag:6s} {os.path.basename(f):24s} {lib:22s} {d['config'].get('shape', '?'):8s} "
                    f"{d['value'] / 1e9:7.4f} G  {d['ms_per_step']:.3f} ms  "
                    f"oracle_match={d.get('parity', {}).get('oracle_match')}")
    gates = sorted(glob.glob(os.path.join(ROOT, "gpurun_out", tag, "parity_*.log")))
    for g in gates:
        last = [ln for ln in open(g).read().splitlines() if "passed" in ln or "failed" in ln]
        rows.append(f"{tag:6s} gate {os.path.basename(g)[7:-4]:22s} " + (" | ".join(x.strip(" =") for x in last) or "?"))
    print("\n".join(rows))
