"""A minimal host-side process group for the ranks of one node: barrier, max-reduce of a
float, broadcast of bytes, and bytes from a rank to rank 0.  TCP over 127.0.0.1 in a star
around rank 0.

bench.py's ranks need exactly these three (the barrier and max-over-ranks timing of the
contract, and handing RCCL's 128-byte unique id and a shared-memory name around).  They
take them from here rather than from torch.distributed: importing torch into the
process brings torch's own HIP / HSA runtime next to /opt/rocm's, and RCCL then fails
to initialise ("no ROCm-capable device").  The product path uses no torch.

Rendezvous: rank 0 listens on an ephemeral port and publishes it in a file named by
MASTER_PORT and the launcher's pid (all ranks of one launch share their parent), so
nothing has to agree on a second fixed port.
"""
from __future__ import annotations

import os
import socket
import struct
import tempfile
import time


def _recvn(sock, n):
    buf = bytearray()
    while len(buf) < n:
        chunk = sock.recv(n - len(buf))
        if not chunk:
            raise ConnectionError("hostgroup peer closed")
        buf.extend(chunk)
    return bytes(buf)


def _send_msg(sock, data: bytes):
    sock.sendall(struct.pack("<Q", len(data)) + data)


def _recv_msg(sock):
    (n,) = struct.unpack("<Q", _recvn(sock, 8))
    return _recvn(sock, n)


class HostGroup:
    def __init__(self, rank: int, world: int, key: str | None = None, timeout: float = 300.0):
        self.rank, self.world = int(rank), int(world)
        self.peers = {}
        self.sock = None
        if self.world == 1:
            return
        key = key or "%s_%d" % (os.environ.get("MASTER_PORT", "0"), os.getppid())
        path = os.path.join(tempfile.gettempdir(), "lslam_hostgroup_%s" % key)
        deadline = time.time() + timeout
        if self.rank == 0:
            srv = socket.socket(socket.AF_INET, socket.SOCK_STREAM)
            srv.bind(("127.0.0.1", 0))
            srv.listen(self.world)
            tmp = path + ".tmp%d" % os.getpid()
            with open(tmp, "w") as f:
                f.write(str(srv.getsockname()[1]))
            os.replace(tmp, path)
            srv.settimeout(timeout)
            try:
                while len(self.peers) < self.world - 1:
                    c, _ = srv.accept()
                    c.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
                    (r,) = struct.unpack("<i", _recvn(c, 4))
                    self.peers[r] = c
            finally:
                srv.close()
                try:
                    os.unlink(path)
                except OSError:
                    pass
        else:
            while True:
                try:
                    with open(path) as f:
                        port = int(f.read())
                    s = socket.create_connection(("127.0.0.1", port), timeout=timeout)
                    break
                except (OSError, ValueError):
                    if time.time() > deadline:
                        raise TimeoutError("hostgroup: rank 0 did not publish %s" % path)
                    time.sleep(0.05)
            s.setsockopt(socket.IPPROTO_TCP, socket.TCP_NODELAY, 1)
            s.sendall(struct.pack("<i", self.rank))
            self.sock = s

    @classmethod
    def from_env(cls):
        return cls(int(os.environ.get("RANK", "0")), int(os.environ.get("WORLD_SIZE", "1")))

    def barrier(self):
        self.allreduce_max(0.0)

    def allreduce_max(self, x: float) -> float:
        if self.world == 1:
            return float(x)
        if self.rank == 0:
            m = float(x)
            for c in self.peers.values():
                m = max(m, struct.unpack("<d", _recv_msg(c))[0])
            for c in self.peers.values():
                _send_msg(c, struct.pack("<d", m))
            return m
        _send_msg(self.sock, struct.pack("<d", float(x)))
        return struct.unpack("<d", _recv_msg(self.sock))[0]

    def broadcast(self, data: bytes | None, root: int = 0) -> bytes:
        """root's bytes on every rank (root 0 only)."""
        if root != 0:
            raise ValueError("hostgroup broadcasts from rank 0")
        if self.world == 1:
            return data
        if self.rank == 0:
            for c in self.peers.values():
                _send_msg(c, data)
            return data
        return _recv_msg(self.sock)

    def send_to_root(self, data: bytes):
        """A non-root rank's bytes to rank 0 (paired with ``recv_from``)."""
        if self.rank == 0:
            raise ValueError("send_to_root from rank 0")
        _send_msg(self.sock, data)

    def recv_from(self, rank: int) -> bytes:
        """On rank 0: the next message ``rank`` sent with ``send_to_root``."""
        if self.rank != 0:
            raise ValueError("recv_from on a non-root rank")
        return _recv_msg(self.peers[int(rank)])

    def close(self):
        for c in self.peers.values():
            c.close()
        if self.sock is not None:
            self.sock.close()
        self.peers, self.sock = {}, None
