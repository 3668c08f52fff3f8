"""Cross-scan landmark map feeding the UKF.

The reference keeps ONE landmark list for the whole run (``check_ransac``'s
``landmarks``, ransac_functions.py:63-93, grown by ``landmark_extraction`` at
:34-54 and ``landmarking.py:48-77``) and never connects it to the UKF it
declares (``systemClass.py:21-29``, ``UKFMethods.py:26-34`` ``hx`` over
``Landmark.pos``).  ``LandmarkMap`` is that missing glue, batched: R robots,
each with

* a persistent WORLD-frame landmark map (the reference's list, on the device),
* its own chained numpy-legacy MT19937 stream (``np.random.seed`` once, the
  stream continues over every chunk of every revolution, as in SLAM.py),
* a UKF state ``x = [x, y, theta]``, ``P``.

One ``step`` = one revolution per robot, one ``lslam_scan_pipeline`` launch in
``LSLAM_UKF_MAP`` mode: predict with ``u``; every fitted chunk line is moved
into the world frame of the predicted pose and run through the reference's
association walk against the robot's map; every chunk that matched a map
landmark becomes a range/bearing measurement against ``hx`` of that landmark's
``pos`` (the measured point is the foot of ``pos``, seen from the predicted
pose, on the chunk's fitted line: ``is_equal`` matches any segment continuing
the same wall); the UKF updates with those measurements only.  With
the pose held at 0 (no predict/update) a map step is exactly the reference's
``check_ransac`` over that revolution (tests/test_gpu_map.py).

All state stays in HBM between steps; ``xy`` may be a device array (e.g. the
output of ``express.ExpressRevolutions``), so packets -> revolutions -> map ->
filter never leave the GPU.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import Context, DeviceArray
from .pipeline import HYP, LANDMARK_DTYPE, MODEL_DTYPE

VAR_DIST, VAR_ANGLE = 0.25, 0.09  # systemClass.py:28 R = diag([0.5**2, 0.3**2] * L)


class LandmarkMap:
    """R robots' maps + filters on one GPU.  ``step`` runs one revolution per robot."""

    def __init__(self, ctx: Context, n_robots: int, *, lmk_capacity=256, slots=8, seeds=None, x0=None, P0=None,
                 R_diag=None, threshold=20.0, max_trials=100, hyp="mt19937", philox_seed=0x5EED5EED,
                 predict=True, update=True, want_yproj=False, tol_a=0.1, tol_b=10.0, tol_dist=100.0, **ukf_kw):
        R = int(n_robots)
        if R <= 0:
            raise ValueError("n_robots must be > 0")
        self.ctx, self.R, self.cap, self.slots, self.T = ctx, R, int(lmk_capacity), int(slots), int(max_trials)
        self.hyp = HYP[hyp]
        self.philox_seed = int(philox_seed)
        self.step_index = 0
        self.want_yproj = want_yproj
        self.landmarks = ctx.to_device(np.zeros((R, self.cap), LANDMARK_DTYPE))
        self.lmk_count = ctx.to_device(np.zeros(R, np.int32))
        seeds = np.arange(R) if seeds is None else np.asarray(seeds)
        if self.hyp == _lib.HYP_MT19937:
            from .pipeline import mt_seed_state
            st = np.stack([mt_seed_state(int(s)) for s in seeds])
            # double-buffered stream state: in -> out, swapped after each step
            self._mt = [ctx.to_device(st), ctx.empty((R, 625), np.uint32)]
        x0 = np.zeros((R, 3)) if x0 is None else np.asarray(x0, np.float64).reshape(R, 3)
        P0 = np.tile(np.diag([.1, .1, .05]), (R, 1, 1)) if P0 is None else np.asarray(P0, np.float64)
        self.x = ctx.to_device(np.ascontiguousarray(x0))
        self.P = ctx.to_device(np.ascontiguousarray(np.broadcast_to(P0, (R, 3, 3))).reshape(R, 9))
        self.u = ctx.to_device(np.zeros((R, 2)))
        Rd = np.array([VAR_DIST, VAR_ANGLE] * self.slots) if R_diag is None else np.asarray(R_diag, np.float64)
        if Rd.shape != (2 * self.slots,):
            raise ValueError("R_diag must hold 2 * slots entries")
        self.R_diag = ctx.to_device(Rd)
        flags = _lib.UKF_MAP | (_lib.UKF_PREDICT if predict else 0) | (_lib.UKF_UPDATE if update else 0)
        self.up = _lib.ukf_params(self.slots, flags=flags, **ukf_kw)
        # tol_*: landmarking.py:4-6 (the reference's defaults)
        self.rp = _lib.ransac_params(residual_threshold=float(threshold), max_trials=self.T, hyp_source=self.hyp,
                                     philox_seed=self.philox_seed, tol_a=float(tol_a), tol_b=float(tol_b),
                                     tol_dist=float(tol_dist))
        self.id_next = np.zeros(R, np.int64)   # landmarkNumber per robot (check_ransac :66, :77)
        self._id_base = ctx.empty(R, np.int32)  # in/out: the kernel advances it per chunk (MAP mode)
        self._id_base.fill_zero()
        self._caps = {}

    def _buf(self, name, shape, dtype):
        n = int(np.prod(shape))
        b = self._caps.get(name)
        if b is None or b.shape[0] < max(n, 1):
            b = self.ctx.empty(max(n, 1), dtype)
            self._caps[name] = b
        return b

    def upload(self, xy, scan_chunk_off, chunk_pt_off):
        """Stage one step's revolutions in HBM (reusable by ``step``)."""
        sco = np.ascontiguousarray(scan_chunk_off, np.int32)
        cpo = np.ascontiguousarray(chunk_pt_off, np.int32)
        P = int(cpo[-1])
        inp = MapInput()
        inp.sco, inp.cpo = sco, cpo
        inp.xy = xy if isinstance(xy, DeviceArray) else self.ctx.to_device(
            np.ascontiguousarray(xy, np.float64).reshape(-1, 2)[:max(P, 1)])
        inp.dsco, inp.dcpo = self.ctx.to_device(sco), self.ctx.to_device(cpo)
        return inp

    def step(self, xy, scan_chunk_off=None, chunk_pt_off=None, u=None, sync=True):
        """One revolution per robot: scan r = chunks scan_chunk_off[r]:[r+1].
        ``xy`` may be a ``MapInput`` from ``upload`` (CSR arguments then omitted)."""
        ctx = self.ctx
        staged = xy if isinstance(xy, MapInput) else None
        if staged is not None:
            xy, scan_chunk_off, chunk_pt_off = staged.xy, staged.sco, staged.cpo
        sco = np.ascontiguousarray(scan_chunk_off, np.int32)
        cpo = np.ascontiguousarray(chunk_pt_off, np.int32)
        if len(sco) != self.R + 1:
            raise ValueError("one revolution per robot: scan_chunk_off needs n_robots + 1 entries")
        Cn, P = int(sco[-1]), int(cpo[-1])
        if len(cpo) != Cn + 1:
            raise ValueError("inconsistent CSR offsets")
        per_scan = np.diff(sco)
        if per_scan.max(initial=0) > self.slots:
            raise ValueError("a revolution has %d chunks > %d measurement slots" % (per_scan.max(), self.slots))
        if isinstance(xy, DeviceArray):
            if xy.dtype != np.float64 or xy.nbytes < 16 * P:
                raise ValueError("device xy must be float64 [n, 2] with n >= chunk_pt_off[-1]")
            dxy = xy
        else:
            h = np.ascontiguousarray(xy, np.float64).reshape(-1, 2)
            if h.shape[0] < P:
                raise ValueError("xy holds fewer points than chunk_pt_off describes")
            dxy = self._buf("xy", (max(P, 1), 2), np.float64)
            dxy.upload(_pad(h[:P], dxy.shape[0]))
        if staged is not None:
            dsco, dcpo = staged.dsco, staged.dcpo
        else:
            dsco = self._buf("sco", (self.R + 1,), np.int32)
            dsco.upload(_pad(sco, dsco.shape[0]))
            dcpo = self._buf("cpo", (Cn + 1,), np.int32)
            dcpo.upload(_pad(cpo, dcpo.shape[0]))
        if u is not None:
            self.u.upload(np.ascontiguousarray(u, np.float64).reshape(self.R, 2))

        self.mask = self._buf("mask", (max(P, 1),), np.uint8)
        self.models = self._buf("models", (max(Cn, 1),), MODEL_DTYPE)
        b = _lib.ScanBatch()
        b.n_scans, b.n_chunks, b.n_points = self.R, Cn, P
        sizes = np.diff(cpo)
        b.max_chunk_points = int(sizes.max()) if Cn else 0
        b.max_scan_chunks = int(per_scan.max()) if self.R else 0
        b.lmk_capacity = self.cap
        b.xy, b.scan_chunk_off, b.chunk_pt_off = dxy.addr, dsco.addr, dcpo.addr
        if self.hyp == _lib.HYP_MT19937:
            b.mt_state_in, b.mt_state_out = self._mt[0].addr, self._mt[1].addr
        else:
            self.rp.philox_seed = (self.philox_seed + 0x9E3779B97F4A7C15 * self.step_index) & 0xFFFFFFFFFFFFFFFF
        b.id_base = self._id_base.addr
        b.landmarks, b.lmk_count = self.landmarks.addr, self.lmk_count.addr
        b.inlier_mask, b.models = self.mask.addr, self.models.addr
        if self.want_yproj:
            self.yproj = self._buf("yproj", (max(P, 1),), np.float64)
            b.y_proj = self.yproj.addr
        b.ukf_x, b.ukf_P, b.ukf_u, b.ukf_R_diag = self.x.addr, self.P.addr, self.u.addr, self.R_diag.addr
        _lib.check(_lib.load().lslam_scan_pipeline(ctx.handle, C.byref(b), C.byref(self.rp), C.byref(self.up)),
                   "lslam_scan_pipeline (map)")
        if self.hyp == _lib.HYP_MT19937:
            self._mt.reverse()
        self.id_next += per_scan
        self.step_index += 1
        self._last = (Cn, P)
        if sync:
            ctx.sync()

    def results(self):
        """Last step's per-chunk records / masks and the current map + filter state."""
        Cn, P = self._last
        out = {"mask": self.mask.download()[:P], "models": self.models.download()[:Cn],
               "landmarks": self.landmarks.download(), "lmk_count": self.lmk_count.download(),
               "x": self.x.download(), "P": self.P.download().reshape(self.R, 3, 3)}
        if self.want_yproj:
            out["y_proj"] = self.yproj.download()[:P]
        if self.hyp == _lib.HYP_MT19937:
            out["mt_state"] = self._mt[0].download()
        return out

    def robot_map(self, r):
        """Robot r's map as the reference's Landmark objects (landmarking.Landmark)."""
        from .landmarking import Landmark
        lst = self.landmarks.download()[r, :int(self.lmk_count.download()[r])]
        out = []
        for e in lst:
            L = Landmark(float(e["a"]), float(e["b"]), int(e["id"]), float(e["pos_x"]), float(e["pos_y"]),
                         float(e["end_x"]), float(e["end_y"]))
            L.life = int(e["life"])
            out.append(L)
        return out


class MapInput:
    """One step's revolutions staged in HBM (``LandmarkMap.upload``)."""
    xy = dsco = dcpo = sco = cpo = None


def _pad(a, n):
    a = np.ascontiguousarray(a).reshape(-1)
    if a.size == n:
        return a
    out = np.zeros(n, a.dtype)
    out[:a.size] = a
    return out
