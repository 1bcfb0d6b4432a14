#!/usr/bin/env python3
"""Static instruction mix per kernel from a hipcc -S gfx950 assembly file."""
import collections
import re
import sys

path = sys.argv[1]
pat = sys.argv[2] if len(sys.argv) > 2 else ""
lines = open(path).read().split("\n")
starts = [i for i, l in enumerate(lines) if re.match(r"^_Z\S+:", l)]
for si, st in enumerate(starts):
    name = lines[st].split(":")[0]
    if pat not in name:
        continue
    end = starts[si + 1] if si + 1 < len(starts) else len(lines)
    body = lines[st:end]
    ins = [l.strip().split()[0] for l in body if l.startswith("\t") and l.strip() and not l.strip().startswith((".", ";"))]
    c = collections.Counter()
    for i in ins:
        k = ("valu" if i.startswith("v_") else "salu" if i.startswith("s_") else "lds" if i.startswith("ds_")
             else "scratch" if i.startswith("scratch_") else "vmem" if i.startswith(("global_", "buffer_", "flat_"))
             else "other")
        c[k] += 1
    top = collections.Counter(i for i in ins if i.startswith("v_")).most_common(12)
    print(name[:70], "total", len(ins), dict(c))
    print("   top valu:", top)
