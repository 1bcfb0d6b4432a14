"""Register census and compile flags of the built gfx950 kernels (DESIGN.md §4 "Lane interference").

Round 6 pinned the mechanism: LLVM's SIOptimizeVGPRLiveRange pass. The pre-fix source rebuilt with
`-mllvm -amdgpu-opt-vgpr-liverange=false` is exact on the frame shapes that failed; the shipped
library is built with the pass off for every kernel (element-crush-gym_amd/Makefile SAFETY), and
test_every_code_object_built_with_the_pass_off checks that on the library's own recorded command
lines (-frecord-command-line), so no kernel reaches the GPU with it on.

The round-4 lane interference needed a kernel that runs several boards per wave AND spills: the
RNG position carried out of the divergent cascade loop came back stale for the lanes that had left
the loop early. The frame kernels now run that loop wave-uniform; this census keeps the 16 x 16
frame's board-per-lane step kernels out of scratch (at most a few values spilled to AGPRs) and holds every kernel to the spill counts
committed in profiles/r06_spill_audit.json (a ratchet: a build that spills more fails here, on the
CPU, before any GPU run). Reads the code-object metadata of build/m3_inst_*.o (tools/spill_audit.py).
"""
import glob
import json
import os
import sys

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, os.path.join(ROOT, "tools"))
import spill_audit  # noqa: E402

OBJS = sorted(glob.glob(os.path.join(ROOT, "element-crush-gym_amd", "build", "m3_inst_*.o")))
LIB = os.path.join(ROOT, "element-crush-gym_amd", "build", "libm3.so")
REF = os.path.join(ROOT, "profiles", "r06_spill_audit.json")
pytestmark = pytest.mark.skipif(len(OBJS) < 10, reason="library objects not built (make -C element-crush-gym_amd)")

# board-per-lane kernels of the 16 x 16 frame that must keep every value in registers (a few spill
# into AGPRs, no scratch): the env step, the stateless apply / legal kernels, the reset
IN_REGS = ("k_env_step<", "k_apply<", "k_legal<", "k_init_fix_lane<")


@pytest.fixture(scope="module")
def census():
    return spill_audit.census(OBJS)


def test_census_covers_every_configuration(census):
    for tag in ("9x9x6", "16x16x8", "frame16/bits2", "frame16/bits5", "frame32/bits2", "frame32/bits5"):
        assert any(tag in k for k in census), tag


def test_frame16_step_kernels_do_not_spill_to_scratch(census):
    checked = 0
    for name, v in census.items():
        if "frame16/" in name and name.startswith(IN_REGS):
            scratch = v.get("private_segment_fixed_size", 0)
            if name.startswith("k_init_fix_lane<"):
                scratch -= 2516  # its FullMT state: a lane-private array by design, not a spill
            assert scratch == 0 and v.get("vgpr_spill_count", 0) <= 5, (name, v)
            checked += 1
    assert checked == 16


def test_no_kernel_spills_more_than_committed(census):
    with open(REF) as f:
        ref = json.load(f)
    worse = {k: (v.get("vgpr_spill_count", 0), ref[k].get("vgpr_spill_count", 0))
             for k, v in census.items()
             if k in ref and v.get("vgpr_spill_count", 0) > ref[k].get("vgpr_spill_count", 0)}
    assert not worse, worse


def test_every_code_object_built_with_the_pass_off():
    """Static check of the shipped artefacts: every gfx950 code object in libm3.so (one per
    translation unit: the C ABI + 10 configurations) and in each object file was compiled with
    SIOptimizeVGPRLiveRange off -- the pass behind the lane interference."""
    dev, host = spill_audit.command_lines(LIB)
    assert len(dev) >= 11, f"{len(dev)} device command lines recorded in libm3.so (built without -frecord-command-line?)"
    missing = [x for x in dev + host if spill_audit.SAFETY_FLAG not in x]
    assert not missing, missing[:2]
    for obj in OBJS + [os.path.join(ROOT, "element-crush-gym_amd", "build", "m3_api.o")]:
        d, _ = spill_audit.command_lines(obj)
        assert d and all(spill_audit.SAFETY_FLAG in x for x in d), obj
