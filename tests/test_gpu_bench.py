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
