"""Host-side rendezvous of the ranks of one node over a plain TCP socket (no torch, no gloo).

The bench ranks only exchange a few small host values -- the 128-byte
ncclUniqueId, barriers around the timed region, the max of the elapsed times,
parity digests and counts. RCCL carries the data; this module carries those.

One process hosts a ``RendezvousServer`` (a thread); every rank holds a
``Rendezvous`` client. The only operation is ``allgather(bytes)``: each rank
sends one frame, and once every rank of the world has sent its frame of that
round, each receives all of them in rank order. ``barrier``, ``broadcast``,
``allmax`` and ``allsum`` are built on it.

Where the server lives:
  * ``bench.py --gpus N`` without a launcher: the parent process (which never
    touches the GPU) hosts it and hands the address to its N children in
    ``M3_RDV=host:port``;
  * under ``torch.distributed.run`` (RANK / WORLD_SIZE / MASTER_* set): rank 0
    hosts it on MASTER_ADDR and publishes the port in a file keyed by
    MASTER_PORT and the launcher's pid (every rank's parent), which the other
    ranks poll. One node only, as the bench contract is.
"""
from __future__ import annotations

import json
import os
import socket
import struct
import tempfile
import threading
import time

_HDR = struct.Struct("<I")
_ERR = 0xFFFFFFFF  # round header of an error frame: the server failed, the text follows


def default_timeout():
    """Seconds a socket waits for a peer (M3_RDV_TIMEOUT; 0 = forever). Long by default: the ranks
    may build the library one after another between two rounds."""
    v = float(os.environ.get("M3_RDV_TIMEOUT", "3600"))
    return None if v <= 0 else v


def _send(sock, data: bytes):
    sock.sendall(_HDR.pack(len(data)) + data)


def _recv_exact(sock, n: int) -> bytes:
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("rendezvous peer closed the connection")
        buf += chunk
    return bytes(buf)


def _recv(sock) -> bytes:
    (n,) = _HDR.unpack(_recv_exact(sock, _HDR.size))
    return _recv_exact(sock, n)


class RendezvousServer:
    """Accepts `world` ranks, then serves allgather rounds until every rank has disconnected."""

    def __init__(self, world: int, host: str = "127.0.0.1", port: int = 0, timeout: float = -1.0):
        self.world = world
        self.timeout = default_timeout() if timeout is not None and timeout < 0 else timeout
        self.sock = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
        self.sock.setsockopt(socket.SOL_SOCKET, socket.SO_REUSEADDR, 1)
        self.sock.bind((host, port))
        self.sock.listen(world)
        self.host, self.port = self.sock.getsockname()[:2]
        self.error = None
        self.thread = threading.Thread(target=self._serve, name="m3-rendezvous", daemon=True)
        self.thread.start()

    @property
    def address(self) -> str:
        return f"{self.host}:{self.port}"

    def _serve(self):
        conns = [None] * self.world
        extra = []  # a rejected connection (bad or duplicate rank): it gets the error frame too
        try:
            self.sock.settimeout(self.timeout)
            for _ in range(self.world):
                c, _ = self.sock.accept()
                c.settimeout(self.timeout)
                rank = int(_recv(c).decode())
                if not 0 <= rank < self.world or conns[rank] is not None:
                    extra.append(c)
                    raise ValueError(f"rendezvous: bad or duplicate rank {rank}")
                conns[rank] = c
            while True:
                frames = []
                for c in conns:
                    try:
                        frames.append(_recv(c))
                    except ConnectionError:
                        return  # a rank finished (all ranks leave together after their last round)
                out = _HDR.pack(self.world) + b"".join(_HDR.pack(len(f)) + f for f in frames)
                for c in conns:
                    _send(c, out)
        except Exception as e:  # surfaced to the clients: an error frame, then a closed connection
            self.error = e
            msg = _HDR.pack(_ERR) + f"{type(e).__name__}: {e}".encode()
            for c in conns + extra:
                if c is not None:
                    try:
                        _send(c, msg)
                        c.shutdown(socket.SHUT_WR)  # the frame goes out before the close (no RST over unread data)
                    except OSError:
                        pass
        finally:
            for c in conns + extra:
                if c is not None:
                    c.close()
            self.sock.close()

    def close(self):
        try:
            self.sock.close()
        except OSError:
            pass


class Rendezvous:
    """Client side: one per rank."""

    def __init__(self, rank: int, world: int, address: str, server: RendezvousServer = None,
                 timeout: float = -1.0):
        self.rank, self.world = rank, world
        timeout = default_timeout() if timeout is not None and timeout < 0 else timeout
        self.server = server
        host, port = address.rsplit(":", 1)
        deadline = time.time() + 60.0
        while True:
            try:
                self.sock = socket.create_connection((host, int(port)), timeout=timeout)
                break
            except OSError:
                if time.time() > deadline:
                    raise
                time.sleep(0.05)
        _send(self.sock, str(rank).encode())

    def allgather(self, data: bytes) -> list:
        try:
            _send(self.sock, bytes(data))
            msg = _recv(self.sock)
        except (ConnectionError, OSError) as e:
            err = getattr(self.server, "error", None)
            raise ConnectionError(f"rendezvous round failed on rank {self.rank}: {e}"
                                  + (f" (server: {err!r})" if err is not None else "")) from e
        (n,) = _HDR.unpack_from(msg, 0)
        if n == _ERR:
            raise ConnectionError(f"rendezvous server failed: {msg[_HDR.size:].decode(errors='replace')}")
        out, off = [], _HDR.size
        for _ in range(n):
            (k,) = _HDR.unpack_from(msg, off)
            off += _HDR.size
            out.append(msg[off:off + k])
            off += k
        return out

    def allgather_obj(self, obj) -> list:
        return [json.loads(x.decode()) for x in self.allgather(json.dumps(obj).encode())]

    def barrier(self):
        self.allgather(b"")

    def broadcast(self, data: bytes, src: int = 0) -> bytes:
        return self.allgather(data if self.rank == src else b"")[src]

    def allmax(self, value: float) -> float:
        return max(self.allgather_obj(float(value)))

    def allsum(self, values):
        rows = self.allgather_obj([int(v) for v in values])
        return [sum(col) for col in zip(*rows)]

    def get_world_size(self) -> int:
        return self.world

    def close(self):
        try:
            self.sock.close()
        finally:
            if self.server is not None:
                self.server.thread.join(timeout=10)
                self.server.close()
                self.server = None


def _port_file(master_addr: str, master_port: str) -> str:
    d = os.environ.get("M3_RDV_DIR", tempfile.gettempdir())
    return os.path.join(d, f"m3_rdv_{master_addr}_{master_port}_{os.getppid()}")


def from_env(rank: int, world: int) -> Rendezvous:
    """The rank's client, wherever the server lives (module docstring)."""
    addr = os.environ.get("M3_RDV")
    if addr:
        return Rendezvous(rank, world, addr)
    master_addr = os.environ.get("MASTER_ADDR", "127.0.0.1")
    master_port = os.environ.get("MASTER_PORT")
    if master_port is None:
        raise RuntimeError("world > 1 needs M3_RDV (bench.py --gpus N) or a launcher's MASTER_ADDR/MASTER_PORT")
    path = _port_file(master_addr, master_port)
    if rank == 0:
        srv = RendezvousServer(world, host=master_addr)
        tmp = path + ".tmp"
        with open(tmp, "w") as f:
            f.write(srv.address)
        os.replace(tmp, path)  # removed by cleanup_port_file() after the last round
        return Rendezvous(0, world, srv.address, server=srv)
    deadline = time.time() + 120.0
    while not os.path.exists(path):
        if time.time() > deadline:
            raise TimeoutError(f"rendezvous: rank 0 never published {path}")
        time.sleep(0.05)
    with open(path) as f:
        return Rendezvous(rank, world, f.read().strip())


def cleanup_port_file():
    """Rank 0 removes the published port (after the last rendezvous round)."""
    mp = os.environ.get("MASTER_PORT")
    if mp is None or os.environ.get("M3_RDV"):
        return
    try:
        os.remove(_port_file(os.environ.get("MASTER_ADDR", "127.0.0.1"), mp))
    except OSError:
        pass
