#!/usr/bin/env python3
"""Per-kernel VGPR/SGPR/scratch/occupancy/LDS table for libm3 (hipcc -Rpass-analysis)."""
import re
import subprocess
import sys

ROOT = __file__.rsplit("/tools/", 1)[0]
src = sys.argv[1] if len(sys.argv) > 1 else f"{ROOT}/element-crush-gym_amd/csrc/m3_api.hip"
out = subprocess.run(["/opt/rocm/bin/hipcc", "-O3", "-std=c++17", "-fPIC", "--offload-arch=gfx950", "-c",
                      "-o", "/tmp/_ru.o", src, "-Rpass-analysis=kernel-resource-usage"],
                     capture_output=True, text=True).stderr
rows, cur = [], None
for line in out.splitlines():
    m = re.search(r"remark:\s+(.*?): (.*) \[-Rpass", line)
    if not m:
        continue
    k, v = m.group(1).strip(), m.group(2).strip()
    if k == "Function Name":
        name = subprocess.run(["c++filt", v], capture_output=True, text=True).stdout.strip()
        name = name.replace("(anonymous namespace)::", "")
        name = re.sub(r"m3::Cfg<(\d+), (\d+), (\d+)>", r"\1x\2x\3", name).split("(")[0]
        cur = {"name": name}
        rows.append(cur)
    elif cur is not None:
        cur[k] = v
for r in rows:
    print("%-32s VGPR %-4s SGPR %-4s scratch %-5s occ %-2s lds %-6s spill(s/v) %s/%s" % (
        r["name"].replace("void ", ""), r.get("VGPRs"), r.get("TotalSGPRs"), r.get("ScratchSize [bytes/lane]"),
        r.get("Occupancy [waves/SIMD]"), r.get("LDS Size [bytes/block]"), r.get("SGPRs Spill"), r.get("VGPRs Spill")))
