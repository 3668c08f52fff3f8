"""RPLidar express-scan packets on the GPU: the capture side of the hot path.

Reference (the measure stream the capture process consumes, and the capture
loop itself):

* ``lidar.py:55-91``  ``twos_comp`` + ``ExpressPacket.decode``: sync nibbles,
  XOR checksum, start angle, 16 cabins x 2 (distance, Q3 angle offset);
* ``lidar.py:179-187, 327-338``  ``Lidar._process_express_scan`` over the
  stream ``Lidar.scan('express')`` yields: packet p's 32 measures are
  interpolated towards packet p+1's start angle;
* ``functions.py:47-81``  ``scanning(rawPoints)``: polar -> Cartesian (A1),
  a chunk every 100 points, on the new-revolution flag the remainder if it has
  more than 2 points, then the delimiter ``0`` (A2).

Device entry points (include/lidarslam.h):

* ``express_measures(ctx, packets)``  -> the measure stream, one launch
  (``lslam_express_decode``);
* ``ExpressRevolutions(ctx, packets, skip)`` -> the completed revolutions as
  the CSR batch ``ScanPipeline`` consumes, xy left on the device
  (``lslam_express_scans``);
* ``ExpressCapture(sink)``: the ``scanning`` loop for a raw byte stream read
  from the sensor in bulk; it puts chunks and ``0`` into ``sink`` like the
  reference's ``rawPoints`` queue.

A packet that fails its sync/checksum check raises ``ValueError`` in the
reference (and ends the capture process); here its measures (and its
predecessor's, which need its start angle) are reported invalid and skipped.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import Context, DeviceArray

PACKET_BYTES = 84
MIN_NEIGHBOORS = 100  # functions.py:14


def _packets_array(packets):
    if isinstance(packets, (bytes, bytearray, memoryview)):
        a = np.frombuffer(bytes(packets), np.uint8)
    else:
        a = np.ascontiguousarray(packets, np.uint8)
    if a.size % PACKET_BYTES:
        raise ValueError("express stream is not a whole number of %d-byte packets" % PACKET_BYTES)
    return a.reshape(-1, PACKET_BYTES)


def express_measures(ctx: Context, packets, want_xy=True):
    """The measure stream of ``Lidar.scan('express')`` over M packets:
    dict of [M-1, 32] arrays ``valid``, ``new_scan``, ``angle_deg``,
    ``dist_mm`` (+ ``xy`` [M-1, 32, 2]) and ``pkt_valid`` [M]."""
    pk = _packets_array(packets)
    M = pk.shape[0]
    n = max(M - 1, 0) * 32
    dpk = ctx.to_device(pk if M else np.zeros((1, PACKET_BYTES), np.uint8))
    out = {k: ctx.empty(max(n, 1), t) for k, t in (("angle_deg", np.float64), ("dist_mm", np.float64),
                                                   ("new_scan", np.uint8), ("valid", np.uint8))}
    if want_xy:
        out["xy"] = ctx.empty((max(n, 1), 2), np.float64)
    out["pkt_valid"] = ctx.empty(max(M, 1), np.uint8)
    m = _lib.ExpressMeasures()
    for k, a in out.items():
        setattr(m, k, a.addr)
    _lib.check(_lib.load().lslam_express_decode(ctx.handle, dpk.addr, M, C.byref(m)), "lslam_express_decode")
    ctx.sync()
    res = {}
    for k, a in out.items():
        h = a.download()
        if k == "pkt_valid":
            res[k] = h[:M]
        elif k == "xy":
            res[k] = h[:n].reshape(-1, 32, 2)
        else:
            res[k] = h[:n].reshape(-1, 32)
    return res


class ExpressRevolutions:
    """Packets -> completed revolutions (E1 + A1 + A2) on the device.

    ``run(packets_device_or_host, skip=0)`` decodes the stream and leaves the
    revolutions' points in ``self.xy`` (a DeviceArray [cap, 2]); after
    ``sync`` the host gets the CSR offsets (``scan_chunk_off``,
    ``chunk_pt_off``), the point count and ``resume`` (the packet holding the
    last new-revolution flag: the stream continues from it with skip = 1).
    Capacities are sized for the worst case of M packets, so writes are never
    clipped.
    """

    def __init__(self, ctx: Context, max_packets: int):
        self.ctx = ctx
        self.max_packets = int(max_packets)
        np_ = max(self.max_packets - 1, 1)
        self.cap_points = 32 * np_
        self.cap_scans = np_
        self.cap_chunks = 32 * np_ // MIN_NEIGHBOORS + np_
        self.xy = ctx.empty((self.cap_points, 2), np.float64)
        self.d_sco = ctx.empty(self.cap_scans + 1, np.int32)
        self.d_cpo = ctx.empty(self.cap_chunks + 1, np.int32)
        self.d_counts = ctx.empty(4, np.int32)
        self.d_packets = None
        o = _lib.ExpressRevs()
        o.xy, o.scan_chunk_off, o.chunk_pt_off, o.counts = self.xy.addr, self.d_sco.addr, self.d_cpo.addr, \
            self.d_counts.addr
        o.cap_points, o.cap_scans, o.cap_chunks = self.cap_points, self.cap_scans, self.cap_chunks
        self.out = o

    def upload(self, packets):
        pk = _packets_array(packets)
        if pk.shape[0] > self.max_packets:
            raise ValueError("%d packets > max_packets %d" % (pk.shape[0], self.max_packets))
        if self.d_packets is None:
            self.d_packets = self.ctx.empty((self.max_packets, PACKET_BYTES), np.uint8)
        if pk.shape[0]:
            _lib.check(self.ctx._L.lslam_h2d(self.ctx.handle, self.d_packets.ptr, pk.ctypes.data_as(C.c_void_p),
                                             pk.nbytes), "lslam_h2d")
            self.ctx.sync()
        self.n_packets = pk.shape[0]
        return self.d_packets

    def launch(self, n_packets=None, skip=0, packets_addr=None):
        """Enqueue on the ctx stream (no sync).  Defaults to the uploaded stream."""
        n = self.n_packets if n_packets is None else int(n_packets)
        if n > self.max_packets:
            raise ValueError("%d packets > max_packets %d" % (n, self.max_packets))
        addr = self.d_packets.addr if packets_addr is None else packets_addr
        _lib.check(_lib.load().lslam_express_scans(self.ctx.handle, addr, n, int(skip), C.byref(self.out)),
                   "lslam_express_scans")

    def run(self, packets, skip=0):
        self.upload(packets)
        self.launch(skip=skip)
        return self.fetch()

    def fetch(self):
        """Sync and download the small CSR arrays (xy stays on the device)."""
        cnt = self.d_counts.download()
        S, Cn, P, resume = (int(x) for x in cnt)
        if S > self.cap_scans or Cn > self.cap_chunks or P > self.cap_points:  # cannot happen with these caps
            raise _lib.HIPLibraryError("express revolution capacity exceeded: %r" % (cnt,))
        self.n_scans, self.n_chunks, self.n_points, self.resume = S, Cn, P, resume
        self.scan_chunk_off = self.d_sco.download()[:S + 1] if S else np.zeros(1, np.int32)
        self.chunk_pt_off = self.d_cpo.download()[:Cn + 1]
        return self

    def xy_host(self):
        return self.xy.download()[:self.n_points]


class ExpressCapture:
    """functions.py:47-81 ``scanning`` for a raw express byte stream.

    ``feed(raw_bytes)`` appends bytes read from the sensor (whole or partial
    packets); every completed revolution is decoded, converted and chunked on
    the GPU and put into ``sink`` as the reference does: each chunk as a list
    of [dX, dY], then ``0``.  The open revolution is carried over (from its
    flagged packet, skip = 1) to the next ``feed``.  ``drop`` measures at the
    start stand for the reference's 1-second warm-up.
    """

    def __init__(self, sink, ctx: Context | None = None, drop=0, max_packets=4096):
        from .functions import _context
        self.sink = sink
        self.ctx = ctx or _context()
        self.buf = bytearray()
        q, r = divmod(int(drop), 32)
        self.drop_packets, self.skip = q, r
        self.rev = ExpressRevolutions(self.ctx, max_packets)

    def feed(self, raw):
        """Returns the number of revolutions put into the sink."""
        self.buf += raw
        while self.drop_packets and len(self.buf) >= PACKET_BYTES:
            del self.buf[:PACKET_BYTES]
            self.drop_packets -= 1
        done = 0
        while True:
            M = min(len(self.buf) // PACKET_BYTES, self.rev.max_packets)
            if M < 2:
                return done
            r = self.rev.run(bytes(self.buf[:M * PACKET_BYTES]), skip=self.skip)
            if r.n_scans == 0:
                if M == self.rev.max_packets:
                    raise ValueError("no new-revolution flag in %d packets (max_packets too small)" % M)
                return done
            xy = r.xy_host()
            cpo, sco = r.chunk_pt_off, r.scan_chunk_off
            for s in range(r.n_scans):
                for c in range(sco[s], sco[s + 1]):
                    self.sink.put(xy[cpo[c]:cpo[c + 1]].tolist())
                self.sink.put(0)
            done += r.n_scans
            del self.buf[:r.resume * PACKET_BYTES]
            self.skip = 1
