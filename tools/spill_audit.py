#!/usr/bin/env python3
"""Register / spill census of the gfx950 kernels in libm3's objects (round 5).

    python3 tools/spill_audit.py [objects...]   (default: element-crush-gym_amd/build/m3_inst_*.o)
    python3 tools/spill_audit.py --json profiles/r05_spill_audit.json

Reads each kernel's AMDGPU metadata (the code object's note: .vgpr_count, .agpr_count,
.vgpr_spill_count, .sgpr_spill_count, .private_segment_fixed_size) from the device code bundled in
the objects. Why it matters: the round-4 frame-kernel lane interference needs VGPR spills -- a
value live out of a divergent loop came back stale for the lanes that left the loop early when the
kernel spilled VGPRs; tests/test_spill_audit_cpu.py keeps every kernel that runs
several boards per wave in the frame configurations spill-free.
"""
import glob
import json
import os
import re
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
LLVM = "/opt/rocm/lib/llvm/bin"
TARGET = "hipv4-amdgcn-amd-amdhsa--gfx950"
FIELDS = ("vgpr_count", "agpr_count", "vgpr_spill_count", "sgpr_spill_count", "sgpr_count",
          "private_segment_fixed_size")


def notes(obj, tmp):
    fat, co = os.path.join(tmp, "fat.bin"), os.path.join(tmp, "dev.hsaco")
    subprocess.run([f"{LLVM}/llvm-objcopy", f"--dump-section=.hip_fatbin={fat}", obj, os.path.join(tmp, "x.o")],
                   check=True, capture_output=True)
    subprocess.run([f"{LLVM}/clang-offload-bundler", "--type=o", f"--targets={TARGET}", f"--input={fat}",
                    f"--output={co}", "--unbundle"], check=True, capture_output=True)
    return subprocess.run([f"{LLVM}/llvm-readelf", "--notes", co], check=True, capture_output=True,
                          text=True).stdout


def demangle(name):
    n = subprocess.run(["c++filt", name], capture_output=True, text=True).stdout.strip()
    n = n.replace("(anonymous namespace)::", "").replace("void ", "")
    n = re.sub(r"m3::Cfg<(\d+), (\d+), (\d+)>", r"\1x\2x\3", n)
    n = re.sub(r"m3::FCfg<(\d+), (\d+)>", r"frame\2/bits\1", n)
    return n.split("(")[0]


def census(objs):
    out = {}
    with tempfile.TemporaryDirectory() as tmp:
        for obj in objs:
            cur = None
            for line in notes(obj, tmp).splitlines():
                m = re.match(r"\s*-?\s*\.(\w+):\s+(\S+)", line)
                if not m:
                    continue
                k, v = m.groups()
                if k == "name" and "_GLOBAL__N_" in v:
                    cur = demangle(v)
                    out[cur] = {"object": os.path.basename(obj)}
                elif cur and k in FIELDS:
                    out[cur][k] = int(v)
    return out


SAFETY_FLAG = "-amdgpu-opt-vgpr-liverange=false"


def command_lines(path):
    """The compile command lines recorded in a library or object (-frecord-command-line, one per
    code object): (device lines, host lines). Device code objects are the ones built with
    -mcpu=gfx950; their strings sit uncompressed in the .hip_fatbin bundles."""
    data = open(path, "rb").read()
    lines = [m.group(0).decode(errors="replace") for m in re.finditer(rb"/[^\0\n]*/clang-\d+ [^\0\n]*", data)]
    dev = [x for x in lines if "-mcpu=gfx950" in x]
    return dev, [x for x in lines if "-mcpu=gfx950" not in x]


def main():
    args = [a for a in sys.argv[1:] if not a.startswith("--") and not a.endswith(".json")]
    objs = args or sorted(glob.glob(os.path.join(ROOT, "element-crush-gym_amd", "build", "m3_inst_*.o")))
    c = census(objs)
    if "--json" in sys.argv:
        with open(sys.argv[sys.argv.index("--json") + 1], "w") as f:
            json.dump(c, f, indent=1, sort_keys=True)
    for k, v in sorted(c.items()):
        print(f"{k:32s} vgpr {v.get('vgpr_count', 0):3d} agpr {v.get('agpr_count', 0):3d} "
              f"vgpr-spill {v.get('vgpr_spill_count', 0):4d} sgpr-spill {v.get('sgpr_spill_count', 0):5d} "
              f"scratch {v.get('private_segment_fixed_size', 0):5d}")
    return c


if __name__ == "__main__":
    main()
