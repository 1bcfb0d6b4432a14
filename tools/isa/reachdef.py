"""Wave-level reaching definitions of one VGPR at one instruction of an AMDGPU .s kernel
(round-6 debug of the lane-interference pin: which writes of the register that a store reads
can reach that store along the wave's control flow graph).
usage: reachdef.py kernel.s <line-of-use> <vN>"""
import re
import sys

path, use_line, reg = sys.argv[1], int(sys.argv[2]), sys.argv[3]
lines = open(path).read().split("\n")
rn = int(reg[1:])
lab = re.compile(r"^(\.LBB\d+_\d+):")
bbc = re.compile(r"^; %bb\.(\d+):")


def writes(ins):
    """does instruction text write VGPR rn (first operand)?"""
    m = re.match(r"\s+([a-z0-9_]+)\s+(\S+)", ins)
    if not m:
        return False
    op, d = m.group(1), m.group(2).rstrip(",")
    if op.startswith(("s_", "global_store", "scratch_store", "buffer_store", "flat_store", "ds_write", "ds_store",
                      "v_cmp", "v_readlane", "v_readfirstlane", "global_atomic_add")) and "v_cmpx" not in op:
        if not (op.startswith("global_atomic") and "sc0" in ins):
            return False
    if op.startswith("v_cmpx") or op == "v_cmp":
        return False
    rm = re.match(r"v(\d+)$", d) or re.match(r"v\[(\d+):(\d+)\]$", d)
    if not rm:
        return False
    lo = int(rm.group(1))
    hi = int(rm.group(2)) if rm.lastindex == 2 else lo
    return lo <= rn <= hi


# basic blocks: start at labels / %bb comments, end after branches
blocks, starts = [], {}
cur = None
for i, l in enumerate(lines, 1):
    m = lab.match(l) or bbc.match(l)
    if m:
        cur = {"name": l.split(":")[0], "start": i, "ins": [], "succ": [], "fall": True}
        blocks.append(cur)
        starts[cur["name"]] = len(blocks) - 1
        continue
    if cur is None:
        continue
    s = l.split(";")[0]
    if not s.strip() or s.strip().startswith("."):
        continue
    cur["ins"].append((i, s))
    t = s.split()
    if t[0] == "s_branch":
        cur["succ"].append(t[1]); cur["fall"] = False
    elif t[0].startswith("s_cbranch"):
        cur["succ"].append(t[1])
    elif t[0] == "s_add_u32" and "(.LBB" in s:
        cur["succ"].append(re.search(r"\((\.LBB\d+_\d+)-", s).group(1))
    elif t[0] in ("s_setpc_b64", "s_endpgm"):
        cur["fall"] = False
succ = []
for k, b in enumerate(blocks):
    ss = [starts[x] for x in b["succ"] if x in starts]
    if b["fall"] and k + 1 < len(blocks):
        ss.append(k + 1)
    succ.append(ss)
pred = [[] for _ in blocks]
for k, ss in enumerate(succ):
    for s in ss:
        pred[s].append(k)
# block + index of the use
ub = max(k for k, b in enumerate(blocks) if b["start"] <= use_line)
# backward search: from the use, walk predecessors until a write of the register
found, seen = {}, set()
work = [(ub, [i for i, _ in blocks[ub]["ins"] if i < use_line])]
while work:
    k, lines_before = work.pop()
    hit = None
    for i in reversed(lines_before):
        s = dict(blocks[k]["ins"])[i]
        if writes(s):
            hit = (i, s.strip())
            break
    if hit:
        found[hit[0]] = hit[1]
        continue
    for p in pred[k]:
        if p not in seen:
            seen.add(p)
            work.append((p, [i for i, _ in blocks[p]["ins"]]))
print(f"{len(blocks)} blocks; writes of {reg} reaching line {use_line}:")
for i in sorted(found):
    k = max(j for j, b in enumerate(blocks) if b["start"] <= i)
    print(f"  line {i} [{blocks[k]['name']}]: {found[i]}")
