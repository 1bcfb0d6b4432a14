"""bench.py end to end on the MI355X at reduced size: the bench attests its own run.

After the clock stops, bench.py replays boards spread over the env through the C
oracle (from their first episode through every same-step autoreset to the last
timed step) and reports parity.oracle_match; nranks comes from the RCCL
communicator (1 without one)."""
import json
import os
import subprocess
import sys

import pytest

from conftest import ROOT

pytestmark = pytest.mark.gpu


@pytest.mark.parametrize("shape,boards", [("9x9x6", 65536), ("16x16x8", 16384)])
def test_bench_line_attests_parity(shape, boards):
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--shape", shape, "--boards", str(boards),
           "--steps", "6", "--warmup", "3", "--no-cpu-baseline", "--check-boards", "384"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    d = json.loads(out.stdout.strip().splitlines()[-1])
    assert d["value"] > 0 and d["n_gpus"] == 1 and d["nranks"] == 1 and d["gather_ok"] is None
    assert d["parity"]["oracle_match"] is True, d["parity"]
    assert d["parity"]["oracle_sample"]["boards"] == 384 and len(d["parity"]["digest"]) == 8


def test_more_gpus_than_the_box_has_fails_loudly():
    """`python bench.py --gpus N` with N above the visible GPUs: the rank whose GPU index is not
    visible fails before any device work and the whole job exits non-zero -- no 1-GPU line
    printed under an N-GPU command (the driver's scaling run uses this command form)."""
    from match3tile import _native

    n = _native.device_count()
    cmd = [sys.executable, os.path.join(ROOT, "bench.py"), "--gpus", str(n + 1), "--boards", "4096",
           "--steps", "2", "--warmup", "1", "--no-cpu-baseline", "--check-boards", "0"]
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=300, cwd=ROOT)
    assert out.returncode != 0
    assert not [x for x in out.stdout.splitlines() if x.startswith("{")], out.stdout[-2000:]
