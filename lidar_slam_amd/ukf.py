"""GPU-backed Unscented Kalman Filter with the interface systemClass.py wires up.

``UnscentedKalmanFilter`` exposes what the reference's ``System.ukf`` (a
filterpy 1.4.5 ``UnscentedKalmanFilter``, systemClass.py:21-29) exposes to its
callers: ``predict(u=[vl, vr])``, ``update(z, landmarks=...)``, and the
attributes ``x`` (3,), ``P`` (3,3), ``Q``, ``R``, ``Wm``, ``Wc``, ``dt``.  The
process/measurement models are UKFMethods.py's intended ``transition_function``
/ ``transfer_function`` with its angle-aware means and residuals; every step
runs on the GPU (lslam_ukf_step, U1-U8).  ``landmarks`` may be Landmark objects
(their ``get_pos()``, as UKFMethods.py:32 uses) or (x, y) pairs.

Difference from filterpy, by design: ``update`` re-draws the sigma points from
the current (x, P) instead of reusing ``sigmas_f`` cached by ``predict``; the
two coincide whenever ``update`` follows ``predict`` (filterpy's own usage).
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import Context
from .pipeline import ukf_weights


class UnscentedKalmanFilter:
    def __init__(self, dim_x=3, dim_z=16, dt=0.005, alpha=1e-4, beta=2.0, kappa=0.0, device=0, ctx=None):
        if dim_x != 3:
            raise ValueError("dim_x must be 3 ([x, y, theta], robot.py:6-7)")
        if dim_z % 2:
            raise ValueError("dim_z must be 2 * number of landmarks")
        self.ctx = ctx or Context(device)
        self._dim_x, self._dim_z = dim_x, dim_z
        self.L = dim_z // 2
        self.dt = dt
        self.up = _lib.ukf_params(self.L, dt=float(dt), alpha=float(alpha), beta=float(beta), kappa=float(kappa))
        self.Wm, self.Wc, _ = ukf_weights(self.up)
        self.x = np.zeros(3)
        self.P = np.eye(3)
        self.Q = np.eye(3)
        self.R = np.eye(dim_z)
        c = self.ctx
        self._dx, self._dP = c.empty(3, np.float64), c.empty(9, np.float64)
        self._du, self._dz = c.empty(2, np.float64), c.empty(max(dim_z, 1), np.float64)
        self._dl, self._dR = c.empty(max(dim_z, 1), np.float64), c.empty(max(dim_z, 1), np.float64)
        self._dsco = c.to_device(np.array([0, 0], np.int32))
        self._dcpo = c.to_device(np.array([0], np.int32))
        self._z_zero = np.zeros(dim_z)
        self._l_zero = np.zeros(dim_z)

    def _step(self, flags, u, z, lmk):
        for i in range(9):
            self.up.Q[i] = float(np.asarray(self.Q, np.float64).reshape(9)[i])
        self.up.dt = float(self.dt)
        self.up.flags = flags
        self._dx.upload(np.asarray(self.x, np.float64).reshape(3))
        self._dP.upload(np.asarray(self.P, np.float64).reshape(9))
        self._du.upload(np.asarray(u, np.float64).reshape(2))
        self._dz.upload(np.asarray(z, np.float64).reshape(self._dim_z))
        self._dl.upload(np.asarray(lmk, np.float64).reshape(self._dim_z))
        self._dR.upload(np.ascontiguousarray(np.diag(np.asarray(self.R, np.float64))))
        b = _lib.ScanBatch()
        b.n_scans = 1
        b.scan_chunk_off, b.chunk_pt_off = self._dsco.addr, self._dcpo.addr
        b.ukf_x, b.ukf_P, b.ukf_u = self._dx.addr, self._dP.addr, self._du.addr
        b.ukf_z, b.ukf_lmk, b.ukf_R_diag = self._dz.addr, self._dl.addr, self._dR.addr
        _lib.check(_lib.load().lslam_ukf_step(self.ctx.handle, C.byref(b), C.byref(self.up)), "lslam_ukf_step")
        self.x = self._dx.download()
        self.P = self._dP.download().reshape(3, 3)

    def predict(self, dt=None, u=(0.0, 0.0), **kw):
        """filterpy UKF.predict(u=...) with fx = UKFMethods.transition_function."""
        if dt is not None:
            self.dt = dt
        self._step(_lib.UKF_PREDICT, u, self._z_zero, self._l_zero)
        self.x_prior, self.P_prior = self.x.copy(), self.P.copy()

    def update(self, z, R=None, landmarks=None, **kw):
        """filterpy UKF.update(z, landmarks=...) with hx = UKFMethods.transfer_function."""
        if z is None:
            return
        if R is not None:
            self.R = np.eye(self._dim_z) * R if np.isscalar(R) else R
        if landmarks is None:
            raise ValueError("update needs landmarks= (UKFMethods.transfer_function's second argument)")
        pos = [np.asarray(l.get_pos() if hasattr(l, "get_pos") else l, np.float64)[:2] for l in landmarks]
        if len(pos) != self.L:
            raise ValueError("expected %d landmarks for dim_z=%d, got %d" % (self.L, self._dim_z, len(pos)))
        self._step(_lib.UKF_UPDATE, (0.0, 0.0), z, np.concatenate(pos))
        self.x_post, self.P_post = self.x.copy(), self.P.copy()
