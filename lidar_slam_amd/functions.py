"""Drop-in pieces of ``functions.py``: the capture-side transform (A1) and the
revolution chunking (A2) that feed the hot path.

* ``polar_to_xy(theta_deg, dist)``: functions.py:59-60
  ``dX = d*cos(-theta*ANGLE_TO_RAD + PI/2)``, ``dY = d*sin(...)`` for a whole
  array of measures on the GPU (lslam_polar_to_xy).  Tolerance-level parity:
  the device cos/sin may differ from glibc's by an ulp.
* ``ScanChunker``: functions.py:56-76's per-measure state machine (drop the
  first second, a chunk every MIN_NEIGHBOORS = 100 points, on the
  new-revolution flag emit the remainder if it has more than 2 points, then
  the ``0`` delimiter).  It buffers polar measures and converts each emitted
  chunk on the GPU in one launch.
* ``scanning(rawPoints, lidar)``: the capture loop of functions.py:47-81 with
  the reference's own ``Lidar`` object passed in (hardware I/O stays the
  reference's, lidar.py is untouched).
"""
from __future__ import annotations

import time

import numpy as np

PI = np.pi
DISTANCE_LIMIT = 30       # functions.py:12 (unused by the reference too)
ANGLE_TO_RAD = PI / 180   # functions.py:13
MIN_NEIGHBOORS = 100      # functions.py:14

_ctx = None


def _context():
    global _ctx
    if _ctx is None:
        from .device import Context
        _ctx = Context(0)
    return _ctx


def polar_to_xy(theta_deg, dist, ctx=None):
    from .pipeline import polar_to_xy as _p
    return _p(ctx or _context(), theta_deg, dist)


class ScanChunker:
    """functions.py:56-76 as a push-style state machine.

    ``push(new_scan, angle_deg, dist_mm, t)`` per measure; ``sink`` gets
    ``put(list_of_[x, y])`` per chunk and ``put(0)`` per revolution, like the
    reference's ``rawPoints`` multiprocessing.Queue.
    """

    def __init__(self, sink, warmup_s=1.0, start_time=None, ctx=None):
        self.sink = sink
        self.warmup_s = warmup_s
        self.start = time.time() if start_time is None else start_time
        self.ctx = ctx
        self.th, self.d = [], []
        self.nbr_pairs = 0
        self.nbr_points = 0
        self.nbr_tours = 0

    def _emit(self):
        if self.th:
            xy = polar_to_xy(np.array(self.th), np.array(self.d), self.ctx)
            self.sink.put(xy.tolist())
        self.th, self.d = [], []

    def push(self, new_scan, angle_deg, dist_mm, t=None):
        now = time.time() if t is None else t
        if now - self.start <= self.warmup_s:   # functions.py:58
            return
        self.th.append(angle_deg)
        self.d.append(dist_mm)
        self.nbr_pairs += 1
        self.nbr_points += 1
        if self.nbr_pairs == MIN_NEIGHBOORS:    # functions.py:64-67
            self._emit()
            self.nbr_pairs = 0
        if new_scan:                            # functions.py:68-76
            self.nbr_tours += 1
            if len(self.th) > 2:
                self._emit()
            self.sink.put(0)
            self.th, self.d = [], []
            self.nbr_pairs = 0
            self.nbr_points = 0


def scanning(rawPoints, lidar):
    """functions.py:47-81 with the caller's Lidar (reference lidar.py) object."""
    chunker = ScanChunker(rawPoints)
    iterator = lidar.scan('express', max_buf_meas=False, speed=450)
    try:
        for measure in iterator:
            chunker.push(measure[0][0], measure[0][2], measure[0][3])
    except KeyboardInterrupt:
        lidar.stop_motor()
        lidar.reset()
        rawPoints.put(None)


def chunk_offsets(n_points, chunk=MIN_NEIGHBOORS):
    """CSR chunk offsets of one revolution of n_points measures (A2)."""
    sizes = [chunk] * (n_points // chunk)
    if n_points % chunk > 2:
        sizes.append(n_points % chunk)
    return np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
