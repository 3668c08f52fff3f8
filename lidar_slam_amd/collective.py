"""RCCL over xGMI for the sharded path's one data movement: every rank's per-scan
results to the root, plus the bootstrap and a broadcast.

ctypes on ROCm's librccl (rccl.h: ncclGetUniqueId :187, ncclCommInitRank :220,
ncclBroadcast :591, ncclSend :700, ncclRecv :722, ncclGroupStart/End :923-933).
One process per GPU; the 128-byte unique id travels over the host group
(lidar_slam_amd/hostgroup.py).  Every collective is enqueued on the lslam context's main stream
(lslam_ctx_stream), so it runs after the pipeline call that wrote its buffers and
before the context's later calls, with no host sync.

``gatherv`` is the variable-size gather as grouped point-to-point operations: the
root receives rank r's bytes at offset sum(counts[:r]) from each peer (one xGMI
link per peer, all in flight together) and copies its own with a device copy;
every other rank sends once.  Shards of 65,536 720-point scans over 8 ranks are
equal, but the CSR layout allows ragged shards, which plain ncclGather does not.
"""
from __future__ import annotations

import ctypes as C
import os

from .device import DeviceArray

NCCL_UINT8 = 1  # rccl.h ncclDataType_t


class RcclError(RuntimeError):
    pass


class UniqueId(C.Structure):
    _fields_ = [("internal", C.c_ubyte * 128)]  # bytes, not a C string: it holds NULs


_rccl = None


def load():
    global _rccl
    if _rccl is not None:
        return _rccl
    # RCCL's diagnostics default to stdout, where bench.py prints its one JSON line
    os.environ.setdefault("NCCL_DEBUG_FILE", "/dev/stderr")
    err = None
    for name in ("librccl.so", "librccl.so.1", "/opt/rocm/lib/librccl.so"):
        try:
            L = C.CDLL(name)
            break
        except OSError as e:
            err = e
    else:
        raise RcclError("cannot load librccl: %s" % err)
    VP, I, SZ = C.c_void_p, C.c_int, C.c_size_t
    L.ncclGetUniqueId.argtypes = [C.POINTER(UniqueId)]
    L.ncclCommInitRank.argtypes = [C.POINTER(VP), I, UniqueId, I]
    L.ncclCommDestroy.argtypes = [VP]
    L.ncclGetErrorString.argtypes = [I]
    L.ncclGetErrorString.restype = C.c_char_p
    L.ncclSend.argtypes = [VP, SZ, I, I, VP, VP]
    L.ncclRecv.argtypes = [VP, SZ, I, I, VP, VP]
    L.ncclBroadcast.argtypes = [VP, VP, SZ, I, I, VP, VP]
    L.ncclGetVersion.argtypes = [C.POINTER(I)]
    for f in ("ncclGetUniqueId", "ncclCommInitRank", "ncclCommDestroy", "ncclSend", "ncclRecv", "ncclBroadcast",
              "ncclGroupStart", "ncclGroupEnd", "ncclGetVersion"):
        getattr(L, f).restype = I
    _rccl = L
    return L


def _check(rc, what):
    if rc != 0:
        raise RcclError("%s: %s" % (what, load().ncclGetErrorString(rc).decode(errors="replace")))


def version():
    v = C.c_int(0)
    _check(load().ncclGetVersion(C.byref(v)), "ncclGetVersion")
    return v.value


class _stdout_to_stderr:
    """RCCL prints its version banner (NCCL_DEBUG=VERSION) on fd 1 at its first call;
    bench.py's stdout carries exactly one JSON line, so fd 1 points at fd 2 meanwhile."""

    def __enter__(self):
        import sys
        sys.stdout.flush()
        self.saved = os.dup(1)
        os.dup2(2, 1)

    def __exit__(self, *exc):
        os.dup2(self.saved, 1)
        os.close(self.saved)


def unique_id() -> bytes:
    uid = UniqueId()
    with _stdout_to_stderr():
        _check(load().ncclGetUniqueId(C.byref(uid)), "ncclGetUniqueId")
    return C.string_at(C.addressof(uid), 128)


def _addr(x, off=0):
    base = x.addr if isinstance(x, DeviceArray) else int(x)
    return C.c_void_p(base + int(off))


def gatherv_plan(rank, world, counts, root=0):
    """This rank's share of ``gatherv`` as (kind, peer, offset, nbytes) operations, in issue order:

    * on the root: ("copy", root, off_root, n) for its own bytes (send[0:n] -> recv[off:off+n]),
      then ("recv", r, off_r, n_r) for every other rank r with n_r > 0, where
      off_r = sum(counts[:r]);
    * elsewhere: ("send", root, 0, n) of send[0:n], if n = counts[rank] > 0.
    Zero-count ranks issue nothing and are expected by nobody.  The RCCL transport runs the
    send/recv ops inside one ncclGroupStart/End (lidar_slam_amd/collective.py Comm.gatherv); the
    CPU tests run the same plan over gloo (tests/test_shard.py)."""
    world, rank, root = int(world), int(rank), int(root)
    counts = [int(n) for n in counts]
    if len(counts) != world or min(counts, default=0) < 0 or not (0 <= root < world) or not (0 <= rank < world):
        raise ValueError("gatherv: need world = len(counts), counts >= 0 and ranks in [0, world)")
    offs = [0]
    for n in counts:
        offs.append(offs[-1] + n)
    if rank != root:
        return [("send", root, 0, counts[rank])] if counts[rank] else []
    ops = [("copy", root, offs[root], counts[root])] if counts[root] else []
    return ops + [("recv", r, offs[r], counts[r]) for r in range(world) if r != root and counts[r]]


class Comm:
    """One rank of an RCCL communicator bound to an lslam context (its device and stream)."""

    transport = "RCCL grouped send/recv on the lslam context stream"

    def __init__(self, ctx, world: int, rank: int, uid: bytes):
        L = load()
        self.ctx, self.world, self.rank = ctx, int(world), int(rank)
        u = UniqueId()
        C.memmove(C.addressof(u), uid, 128)
        self._comm = C.c_void_p()
        ctx.sync()  # ncclCommInitRank binds the calling thread's current device: the context's
        with _stdout_to_stderr():
            _check(L.ncclCommInitRank(C.byref(self._comm), self.world, u, self.rank), "ncclCommInitRank")

    @classmethod
    def from_process_group(cls, ctx, group=None):
        """Bootstrap over a host group (lidar_slam_amd.hostgroup.HostGroup; None = one rank):
        rank 0's unique id broadcast to all."""
        if group is None or group.world == 1:
            return cls(ctx, 1, 0, unique_id())
        uid = group.broadcast(unique_id() if group.rank == 0 else None)
        return cls(ctx, group.world, group.rank, uid)

    @property
    def _stream(self):
        return C.c_void_p(self.ctx.stream)

    def gatherv(self, send, recv, counts, root=0):
        """Rank r's first counts[r] bytes of ``send`` -> ``recv`` at sum(counts[:r]) on root."""
        ops = gatherv_plan(self.rank, self.world, counts, root)
        L = load()
        st = self._stream
        p2p = [op for op in ops if op[0] != "copy"]
        for kind, _, off, n in ops:
            if kind == "copy":
                self.ctx.copy(_addr(recv, off).value, _addr(send).value, n)
        if not p2p:
            return
        _check(L.ncclGroupStart(), "ncclGroupStart")
        try:
            for kind, peer, off, n in p2p:
                if kind == "recv":
                    _check(L.ncclRecv(_addr(recv, off), n, NCCL_UINT8, peer, self._comm, st), "ncclRecv")
                else:
                    _check(L.ncclSend(_addr(send, off), n, NCCL_UINT8, peer, self._comm, st), "ncclSend")
        except BaseException:
            L.ncclGroupEnd()  # close the group; the body's error is the one reported
            raise
        _check(L.ncclGroupEnd(), "ncclGroupEnd")

    def broadcast(self, buf, nbytes, root=0):
        """In-place broadcast of ``nbytes`` of a device buffer from ``root``."""
        a = _addr(buf)
        _check(load().ncclBroadcast(a, a, int(nbytes), NCCL_UINT8, int(root), self._comm, self._stream),
               "ncclBroadcast")

    def close(self):
        if self._comm and self._comm.value:
            self.ctx.sync()
            load().ncclCommDestroy(self._comm)
            self._comm = C.c_void_p()

    def __del__(self):
        try:
            self.close()
        except Exception:
            pass


class HostComm:
    """``Comm``'s gatherv through host memory and the host group's TCP star: for a rehearsal
    of the multi-rank launch whose ranks share ONE device (bench.py ``LSLAM_RANK_DEVICE``),
    which RCCL refuses ("Duplicate GPU detected").  It issues the same ``gatherv_plan``: a
    sending rank syncs its stream and ships its bytes; the root copies its own on the device
    and uploads each peer's at its offset.  Synchronous and PCIe + TCP bound: it checks the
    C4 leg's bookkeeping across processes, never a multi-GPU rate."""

    transport = "host TCP star (rehearsal: ranks share one device)"

    def __init__(self, ctx, group):
        self.ctx, self.group = ctx, group
        self.world = 1 if group is None else group.world
        self.rank = 0 if group is None else group.rank

    def gatherv(self, send, recv, counts, root=0):
        import numpy as np
        ops = gatherv_plan(self.rank, self.world, counts, root)
        if root != 0 and self.world > 1:
            raise ValueError("HostComm gathers to rank 0")
        for kind, peer, off, n in ops:
            if kind == "copy":
                self.ctx.copy(_addr(recv, off).value, _addr(send).value, n)
            elif kind == "send":
                buf = np.empty(send.nbytes, np.uint8)
                send.download(buf)  # syncs the stream: the pipeline call that wrote it is done
                self.group.send_to_root(buf[:n].tobytes())
            else:
                data = np.frombuffer(self.group.recv_from(peer), np.uint8)
                if data.size != n:
                    raise RcclError("HostComm: rank %d sent %d bytes, expected %d" % (peer, data.size, n))
                _lib_h2d(self.ctx, _addr(recv, off), data)

    def close(self):
        pass


def _lib_h2d(ctx, dst, data):
    from . import _lib
    _lib.check(ctx._L.lslam_h2d(ctx.handle, dst, data.ctypes.data_as(C.c_void_p), data.nbytes), "lslam_h2d")
    ctx.sync()  # data is a temporary


def available() -> bool:
    try:
        load()
        return True
    except RcclError:
        return False


__all__ = ["Comm", "HostComm", "RcclError", "available", "gatherv_plan", "load", "unique_id", "version"]
