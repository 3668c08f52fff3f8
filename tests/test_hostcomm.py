"""collective.HostComm (the C4 leg's gather for a rehearsal whose ranks share one device) on CPU:
two processes over the real HostGroup TCP star, ragged shards, every field's bytes at the
root's offsets exactly as gatherv_plan places them.  The device side is a stand-in (host
buffers behind the same calls: ctx.copy, DeviceArray.download, lslam_h2d), so this covers the
plan, the TCP transport and the placement; the GPU run is bench.py's 2-rank rehearsal
(profiles/r06a_rehearsal_2ranks_host.log)."""
import ctypes as C
import multiprocessing as mp
import os

import numpy as np

from lidar_slam_amd import _lib


class _HostArray:
    """A host buffer standing in for a DeviceArray (address, nbytes, download)."""

    def __init__(self, a):
        self.a = np.ascontiguousarray(a)
        self.nbytes = self.a.nbytes

    def __int__(self):
        return self.a.ctypes.data

    def download(self, out):
        C.memmove(out.ctypes.data, self.a.ctypes.data, self.nbytes)
        return out


class _L:
    @staticmethod
    def lslam_h2d(handle, dst, src, n):
        C.memmove(dst.value, src.value, n)
        return _lib.LSLAM_OK


class _Ctx:
    handle = None
    _L = _L

    @staticmethod
    def copy(dst, src, n):
        C.memmove(dst, src, n)

    def sync(self):
        pass


def _rank(rank, world, key, counts, q):
    from lidar_slam_amd.collective import HostComm
    from lidar_slam_amd.hostgroup import HostGroup
    g = HostGroup(rank, world, key=key, timeout=60)
    comm = HostComm(_Ctx(), g)
    send = _HostArray(np.arange(counts[rank], dtype=np.uint8) + 17 * (rank + 1))
    recv = _HostArray(np.zeros(sum(counts), np.uint8)) if rank == 0 else None
    comm.gatherv(send, recv.a.ctypes.data if recv is not None else None, counts, 0)
    g.barrier()
    if rank == 0:
        q.put(recv.a.tobytes())
    g.close()


def test_hostcomm_gatherv_two_processes():
    counts = [5, 11]
    key = "hostcomm_test_%d" % os.getpid()
    ctx = mp.get_context("fork")
    q = ctx.Queue()
    ps = [ctx.Process(target=_rank, args=(r, 2, key, counts, q)) for r in range(2)]
    for p in ps:
        p.start()
    got = q.get(timeout=60)
    for p in ps:
        p.join(60)
        assert p.exitcode == 0
    want = np.concatenate([np.arange(n, dtype=np.uint8) + 17 * (r + 1) for r, n in enumerate(counts)])
    assert got == want.tobytes()


def test_hostcomm_one_rank_is_a_copy():
    from lidar_slam_amd.collective import HostComm
    comm = HostComm(_Ctx(), None)
    send = _HostArray(np.arange(9, dtype=np.uint8))
    recv = np.zeros(9, np.uint8)
    comm.gatherv(send, recv.ctypes.data, [9], 0)
    assert np.array_equal(recv, np.arange(9, dtype=np.uint8))
