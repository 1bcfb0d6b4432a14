"""bench.py's N>1 branch on CPU: launched exactly as the driver launches it
(python -m torch.distributed.run --nnodes=1 --nproc-per-node 2 --master-addr 127.0.0.1 ...),
two gloo ranks run the rendezvous and the ncclUniqueId broadcast (a stand-in id: ncclGetUniqueId
needs a GPU) and stop before any device work. Every rank must be in a world of 2 and hold the
bytes rank 0 made."""
import json
import os
import socket
import subprocess
import sys

from conftest import ROOT


def _free_port():
    with socket.socket() as s:
        s.bind(("127.0.0.1", 0))
        return s.getsockname()[1]


def test_bench_two_rank_rendezvous_and_unique_id_broadcast():
    cmd = [sys.executable, "-m", "torch.distributed.run", "--nnodes=1", "--nproc-per-node", "2",
           "--master-addr", "127.0.0.1", "--master-port", str(_free_port()),
           os.path.join(ROOT, "bench.py"), "--gpus", "2", "--steps", "3", "--warmup", "1", "--dry-rendezvous"]
    env = dict(os.environ, OMP_NUM_THREADS="1")
    out = subprocess.run(cmd, capture_output=True, text=True, timeout=240, env=env, cwd=ROOT)
    assert out.returncode == 0, out.stderr[-3000:]
    lines = [json.loads(x) for x in out.stdout.splitlines() if x.startswith("{")]
    assert sorted(x["rank"] for x in lines) == [0, 1]
    assert all(x["world"] == 2 and x["dist_world"] == 2 and x["id_bytes"] == 128 for x in lines)
    assert len({x["id_sha256"] for x in lines}) == 1
    assert sorted(x["local_rank"] for x in lines) == [0, 1]


def test_host_cores_reports_a_usable_count():
    sys.path.insert(0, ROOT)
    import bench

    cores, nproc, quota = bench.host_cores()
    assert 1 <= cores <= nproc
    assert quota is None or cores <= quota
