"""Batched, device-resident hot path: many scans per launch on one MI355X.

This is the batched entry point the reference never had: the per-chunk
``landmark_extraction`` (ransac_functions.py:15-59) driven by ``check_ransac``
(ransac_functions.py:63-93) over every chunk of many scans, plus the intended
UKF step (systemClass.py / UKFMethods.py), in ONE library call
(``lslam_scan_pipeline``: producer, resolve, consensus, fix-up and post-pass
kernels on the device).  Semantics per scan: ``np.random.seed(seed[s])``
(or an explicit MT19937 state) chained over the scan's chunks, and the scan's
own landmark list (``landmarks[s]``), ids ``id_base[s] + chunk index``.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import Context, DeviceArray

MODEL_DTYPE = np.dtype([(n, "<f8") for n in ("ox", "oy", "ux", "uy", "a", "b", "tip_x", "tip_y", "proj_a",
                                             "proj_b")] +
                       [(n, "<i4") for n in ("n_inliers", "best_trial", "n_draws", "flags", "match_index",
                                             "landmark_id", "n_points", "reserved")])
LANDMARK_DTYPE = np.dtype([(n, "<f8") for n in ("a", "b", "pos_x", "pos_y", "end_x", "end_y")] +
                          [("id", "<i4"), ("life", "<i4")])
assert MODEL_DTYPE.itemsize == 112 and LANDMARK_DTYPE.itemsize == 56

HYP = {"mt19937": _lib.HYP_MT19937, "philox": _lib.HYP_PHILOX, "explicit": _lib.HYP_EXPLICIT}


class ScanPipeline:
    """Device-resident batch.  Build once, ``run()`` many times.

    Inputs are host numpy arrays (uploaded once).  Outputs are kept on the
    device until ``results()`` downloads them.  Points are ``xy`` [P, 2], or
    ``xy=None`` with the raw measures ``theta_deg`` / ``dist_mm`` [P]: then
    functions.py:59-60 runs inside every kernel's point load (A1 fused).
    """

    def __init__(self, ctx: Context, xy, scan_chunk_off, chunk_pt_off, *, seeds=None, mt_state=None,
                 threshold=20.0, max_trials=100, hyp="mt19937", philox_seed=0x5EED5EED, hyp_draws=None,
                 landmarks=None, lmk_count=None, lmk_capacity=None, id_base=None,
                 ukf=None, want_draws=False, want_counts=False, want_yproj=True, want_state=False,
                 theta_deg=None, dist_mm=None):
        self.ctx = ctx
        polar = xy is None
        if polar:
            if theta_deg is None or dist_mm is None:
                raise ValueError("points: xy, or theta_deg and dist_mm")
            theta_deg = np.ascontiguousarray(theta_deg, np.float64).ravel()
            dist_mm = np.ascontiguousarray(dist_mm, np.float64).ravel()
            if theta_deg.shape != dist_mm.shape:
                raise ValueError("theta_deg / dist_mm size mismatch")
            xy = np.zeros((theta_deg.size, 2))  # shape only
        dev_xy = xy if isinstance(xy, DeviceArray) else None  # e.g. ExpressRevolutions.xy: stays on the device
        if dev_xy is None:
            xy = np.ascontiguousarray(xy, np.float64).reshape(-1, 2)
        elif dev_xy.dtype != np.float64 or dev_xy.shape[-1] != 2:
            raise ValueError("device xy must be float64 [n, 2]")
        sco = np.ascontiguousarray(scan_chunk_off, np.int32)
        cpo = np.ascontiguousarray(chunk_pt_off, np.int32)
        S = len(sco) - 1
        Cn = int(sco[-1])
        P = int(cpo[-1])
        if len(cpo) != Cn + 1 or xy.shape[0] < P:
            raise ValueError("inconsistent CSR offsets")
        sizes = np.diff(cpo)
        per_scan = np.diff(sco)
        self.S, self.C, self.P, self.T = S, Cn, P, int(max_trials)
        self.sco, self.cpo = sco, cpo
        self._keep = []
        self.inputs = {}  # name -> DeviceArray of the uploaded inputs (upload_async refreshes them)
        d = self._dev
        b = _lib.ScanBatch()
        b.n_scans, b.n_chunks, b.n_points = S, Cn, P
        b.max_chunk_points = int(sizes.max()) if Cn else 0
        b.max_scan_chunks = int(per_scan.max()) if S else 0
        if polar:
            b.theta_deg = d(theta_deg[:P] if P else np.zeros(1), "theta_deg")
            b.dist_mm = d(dist_mm[:P] if P else np.zeros(1), "dist_mm")
        elif dev_xy is not None:
            self._keep.append(dev_xy)
            b.xy = dev_xy.addr
        else:
            b.xy = d(xy[:P] if P else np.zeros((1, 2)), "xy")
        b.scan_chunk_off = d(sco, "scan_chunk_off")
        b.chunk_pt_off = d(cpo, "chunk_pt_off")
        self.hyp = HYP[hyp]
        if self.hyp == _lib.HYP_MT19937:
            if isinstance(mt_state, DeviceArray):  # a device-resident chain, e.g. another call's mt_state_out
                if mt_state.dtype != np.uint32 or mt_state.nbytes != S * 625 * 4:
                    raise ValueError("device mt_state must be uint32 [n_scans, 625]")
                self._keep.append(mt_state)
                b.mt_state_in = mt_state.addr
            elif mt_state is not None:
                b.mt_state_in = d(np.ascontiguousarray(mt_state, np.uint32).reshape(S, 625))
            else:
                b.seeds = d(np.ascontiguousarray(seeds if seeds is not None else np.arange(S), np.uint32), "seeds")
            if want_state:
                self.state_out = ctx.empty((S, 625), np.uint32)
                b.mt_state_out = self.state_out.addr
        if self.hyp == _lib.HYP_EXPLICIT:
            b.hyp = d(np.ascontiguousarray(hyp_draws, np.int32).reshape(Cn, self.T + 1, 2))
        if id_base is not None:
            b.id_base = d(np.ascontiguousarray(id_base, np.int32))
        self.assoc = landmarks is not None or lmk_capacity is not None
        if self.assoc:
            cap = int(lmk_capacity or 0)
            if landmarks is None:
                landmarks = np.zeros((S, max(cap, 1)), LANDMARK_DTYPE)
                lmk_count = np.zeros(S, np.int32)
            landmarks = np.ascontiguousarray(landmarks, LANDMARK_DTYPE)
            cap = max(cap, landmarks.shape[1])
            if landmarks.shape[1] < cap:
                pad = np.zeros((S, cap), LANDMARK_DTYPE)
                pad[:, :landmarks.shape[1]] = landmarks
                landmarks = pad
            self.lmk_in = landmarks.copy()
            self.lmk_count_in = np.ascontiguousarray(lmk_count, np.int32).copy()
            self.lmk = ctx.to_device(landmarks)
            self.lmk_count = ctx.to_device(self.lmk_count_in)
            b.landmarks, b.lmk_count, b.lmk_capacity = self.lmk.addr, self.lmk_count.addr, cap
        self.mask = ctx.empty(max(P, 1), np.uint8)
        self.models = ctx.empty(max(Cn, 1), MODEL_DTYPE)
        b.inlier_mask, b.models = self.mask.addr, self.models.addr
        if want_yproj:
            self.yproj = ctx.empty(max(P, 1), np.float64)
            b.y_proj = self.yproj.addr
        if want_draws:
            self.draws = ctx.empty((max(Cn, 1), self.T + 1, 2), np.int32)
            b.draws_out = self.draws.addr
        if want_counts:
            self.counts = ctx.empty((max(Cn, 1), max(self.T, 1)), np.int32)
            b.trial_cnt_out = self.counts.addr
        self.rp = _lib.ransac_params(residual_threshold=float(threshold), max_trials=self.T,
                                     hyp_source=self.hyp, philox_seed=int(philox_seed))
        self.up = None
        if ukf is not None:
            L = int(ukf["n_landmarks"])
            self.up = _lib.ukf_params(L, **{k: v for k, v in ukf.items()
                                            if k in ("flags", "dt", "wheel_radius", "wheel_base", "alpha",
                                                     "beta", "kappa", "Q")})
            self.ukf_x0 = np.ascontiguousarray(ukf["x"], np.float64).reshape(S, 3).copy()
            self.ukf_P0 = np.ascontiguousarray(ukf["P"], np.float64).reshape(S, 9).copy()
            self.ukf_x = ctx.to_device(self.ukf_x0)
            self.ukf_P = ctx.to_device(self.ukf_P0)
            b.ukf_x, b.ukf_P = self.ukf_x.addr, self.ukf_P.addr
            b.ukf_u = d(np.ascontiguousarray(ukf["u"], np.float64).reshape(S, 2), "ukf_u")
            b.ukf_z = d(np.ascontiguousarray(ukf["z"], np.float64).reshape(S, 2 * L), "ukf_z")
            b.ukf_lmk = d(np.ascontiguousarray(ukf["lmk"], np.float64).reshape(S, L, 2), "ukf_lmk")
            b.ukf_R_diag = d(np.ascontiguousarray(ukf["R_diag"], np.float64).reshape(2 * L), "ukf_R_diag")
        self.batch = b

    def _dev(self, arr, name=None):
        a = self.ctx.to_device(arr)
        self._keep.append(a)
        if name:
            self.inputs[name] = a
        return a.addr

    def reset_state(self):
        """Restore the in/out buffers (landmark lists, UKF x/P) to their initial values."""
        if self.assoc:
            self.lmk.upload(self.lmk_in)
            self.lmk_count.upload(self.lmk_count_in)
        if self.up is not None:
            self.ukf_x.upload(self.ukf_x0)
            self.ukf_P.upload(self.ukf_P0)

    def upload_async(self, **arrays):
        """Refresh inputs on the device without a host sync (a new batch of the same shape):
        xy / theta_deg / dist_mm / seeds / ukf_u / ukf_z / ukf_lmk by name, and ukf_x / ukf_P
        (the filters' start state).  The host arrays must stay unchanged until the next
        ``ctx.sync()``; converted copies (another dtype, a strided view, a list) are held by the
        context until then.  Page-locked arrays (device.register_host) copy at PCIe rate."""
        for k, v in arrays.items():
            dst = {"ukf_x": getattr(self, "ukf_x", None), "ukf_P": getattr(self, "ukf_P", None)}.get(k) or \
                self.inputs.get(k)
            if dst is None:
                raise KeyError("no device input %r" % k)
            # a converted copy is a temporary: DeviceArray.upload_async parks it on
            # ctx._inflight until the next sync, so the copy never reads freed memory
            dst.upload_async(np.ascontiguousarray(v, dst.dtype).reshape(dst.shape))

    def clear_lists_async(self):
        """Empty every scan's landmark list on the device (lmk_count = 0), no host sync."""
        if self.assoc:
            self.lmk_count.fill_zero()

    def run(self, sync=True):
        L = _lib.load()
        _lib.check(L.lslam_scan_pipeline(self.ctx.handle, C.byref(self.batch), C.byref(self.rp),
                                         C.byref(self.up) if self.up is not None else None),
                   "lslam_scan_pipeline")
        if sync:
            self.ctx.sync()

    def run_ransac_only(self, sync=True):
        _lib.check(_lib.load().lslam_ransac(self.ctx.handle, C.byref(self.batch), C.byref(self.rp)), "lslam_ransac")
        if sync:
            self.ctx.sync()

    def run_landmarks_only(self, sync=True):
        _lib.check(_lib.load().lslam_landmarks(self.ctx.handle, C.byref(self.batch), C.byref(self.rp)),
                   "lslam_landmarks")
        if sync:
            self.ctx.sync()

    def run_ukf_only(self, sync=True):
        _lib.check(_lib.load().lslam_ukf_step(self.ctx.handle, C.byref(self.batch), C.byref(self.up)),
                   "lslam_ukf_step")
        if sync:
            self.ctx.sync()

    def run_ukf_trace(self):
        """lslam_ukf_trace (a test/diagnostic form of run_ukf_only): the step's intermediate values
        per scan, as a dict of arrays (include/lidarslam.h: sigma points, residual_x, hx(sigma_k),
        zp, residual_h(z, zp), residual_h(hx(sigma_k), zp))."""
        L = int(self.up.n_landmarks)
        m, n = 2 * L, 42 + 32 * L
        tr = self.ctx.empty((max(self.S, 1), n), np.float64)
        tr.upload(np.full((max(self.S, 1), n), np.nan))   # inactive slots stay NaN
        _lib.check(_lib.load().lslam_ukf_trace(self.ctx.handle, C.byref(self.batch), C.byref(self.up), tr.ptr),
                   "lslam_ukf_trace")
        t = tr.download()[:self.S]
        return {"sigmas": t[:, :21].reshape(-1, 7, 3), "dx": t[:, 21:42].reshape(-1, 7, 3),
                "hx": t[:, 42:42 + 7 * m].reshape(-1, 7, m), "zp": t[:, 42 + 7 * m:42 + 8 * m],
                "y": t[:, 42 + 8 * m:42 + 9 * m], "rz": t[:, 42 + 9 * m:].reshape(-1, 7, m)}

    def results(self):
        out = {"mask": self.mask.download()[:self.P], "models": self.models.download()[:self.C]}
        if hasattr(self, "yproj"):
            out["y_proj"] = self.yproj.download()[:self.P]
        if hasattr(self, "draws"):
            out["draws"] = self.draws.download()[:self.C]
        if hasattr(self, "counts"):
            out["counts"] = self.counts.download()[:self.C, :self.T]
        if hasattr(self, "state_out"):
            out["mt_state"] = self.state_out.download()
        if self.assoc:
            out["landmarks"] = self.lmk.download()
            out["lmk_count"] = self.lmk_count.download()
        if self.up is not None:
            out["ukf_x"] = self.ukf_x.download()
            out["ukf_P"] = self.ukf_P.download().reshape(self.S, 3, 3)
        return out


def hyp_mt19937(ctx: Context, scan_chunk_off, chunk_pt_off, seeds=None, mt_state=None, max_trials=100):
    """A3 alone: the choice(N, 2, replace=False) draws each chunk's ransac makes
    (assuming no early stop).  Returns (draws [C][T+1][2], state_out [S][625])."""
    sco = np.ascontiguousarray(scan_chunk_off, np.int32)
    cpo = np.ascontiguousarray(chunk_pt_off, np.int32)
    S, Cn = len(sco) - 1, int(sco[-1])
    keep = []

    def d(a, name=None):
        x = ctx.to_device(a)
        keep.append(x)
        return x.addr

    b = _lib.ScanBatch()
    b.n_scans, b.n_chunks, b.n_points = S, Cn, int(cpo[-1])
    sizes = np.diff(cpo)
    b.max_chunk_points = int(sizes.max()) if Cn else 0
    b.max_scan_chunks = int(np.diff(sco).max()) if S else 0
    b.scan_chunk_off, b.chunk_pt_off = d(sco), d(cpo)
    if mt_state is not None:
        b.mt_state_in = d(np.ascontiguousarray(mt_state, np.uint32).reshape(S, 625))
    else:
        b.seeds = d(np.ascontiguousarray(seeds if seeds is not None else np.arange(S), np.uint32), "seeds")
    draws = ctx.empty((max(Cn, 1), max_trials + 1, 2), np.int32)
    st = ctx.empty((S, 625), np.uint32)
    b.draws_out, b.mt_state_out = draws.addr, st.addr
    _lib.check(_lib.load().lslam_hyp_mt19937(ctx.handle, C.byref(b), int(max_trials)), "lslam_hyp_mt19937")
    ctx.sync()
    return draws.download()[:Cn], st.download()


def polar_to_xy(ctx: Context, theta_deg, dist):
    """A1 (functions.py:59-60) on the device; returns (n, 2) fp64."""
    th = np.ascontiguousarray(theta_deg, np.float64).ravel()
    di = np.ascontiguousarray(dist, np.float64).ravel()
    if th.shape != di.shape:
        raise ValueError("theta/dist size mismatch")
    n = th.size
    dth, ddi = ctx.to_device(th), ctx.to_device(di)
    out = ctx.empty((max(n, 1), 2), np.float64)
    _lib.check(_lib.load().lslam_polar_to_xy(ctx.handle, dth.ptr, ddi.ptr, out.ptr, n), "lslam_polar_to_xy")
    ctx.sync()
    return out.download()[:n]


def mt_seed_state(seed):
    st = np.zeros(625, np.uint32)
    _lib.load().lslam_mt_seed_state(int(seed) & 0xFFFFFFFF, st.ctypes.data_as(C.POINTER(C.c_uint32)))
    return st


def inlier_cutoff(thr):
    return _lib.load().lslam_inlier_cutoff(float(thr))


def ukf_weights(up):
    Wm = (C.c_double * 7)()
    Wc = (C.c_double * 7)()
    lpn = C.c_double(0)
    _lib.load().lslam_ukf_weights(C.byref(up), Wm, Wc, C.byref(lpn))
    return np.array(Wm[:]), np.array(Wc[:]), lpn.value
