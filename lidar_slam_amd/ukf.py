"""GPU-backed Unscented Kalman Filter with the interface systemClass.py wires up.

``UnscentedKalmanFilter`` exposes what the reference's ``System.ukf`` (a
filterpy 1.4.5 ``UnscentedKalmanFilter``, systemClass.py:21-29) exposes to its
callers: ``predict(u=[vl, vr])``, ``update(z, landmarks=...)``, and the
attributes ``x`` (3,), ``P`` (3,3), ``Q``, ``R``, ``Wm``, ``Wc``, ``dt`` and
``sigmas_f``.  The process/measurement models are UKFMethods.py's intended
``transition_function`` / ``transfer_function`` with its angle-aware means and
residuals; every step runs on the GPU (lslam_ukf_step, U1-U8).  ``landmarks``
may be Landmark objects (their ``get_pos()``, as UKFMethods.py:30 uses) or
(x, y) pairs.

filterpy's state is kept as filterpy keeps it:
* ``sigmas_f`` starts as zeros; ``predict`` leaves the sigma points re-drawn from
  the predicted (x, P) there, and ``update`` uses THOSE with the current ``x`` and
  ``P`` (lslam_scan_batch.ukf_sigmas + LSLAM_UKF_SIGMAS_IN), so assigning ``x`` or
  ``P`` between the two calls, or calling ``update`` twice, behaves as in filterpy.
* ``predict(dt=...)`` and ``update(R=...)`` apply to that call only.
What the GPU path cannot represent raises instead of being dropped: a
non-diagonal ``R`` (the kernel takes R's diagonal, systemClass.py:28 builds a
diagonal one), custom ``UT`` / ``fx`` / ``hx`` callables, a predict without
``u`` (transition_function's third argument, UKFMethods.py:17) and an update
without ``landmarks`` (transfer_function's second, UKFMethods.py:26) raise
``TypeError`` as those calls would.
"""
from __future__ import annotations

import ctypes as C

import numpy as np

from . import _lib
from .device import Context
from .pipeline import ukf_weights


def _diag_of(R, dim_z):
    R = np.asarray(R, np.float64)
    if R.shape != (dim_z, dim_z):
        raise ValueError("R must be %d x %d, got %s" % (dim_z, dim_z, R.shape))
    d = np.diag(R)
    if np.any(R - np.diag(d)):
        raise ValueError("R must be diagonal: the GPU UKF takes R's diagonal (systemClass.py:28 builds a "
                         "diagonal R)")
    return np.ascontiguousarray(d)


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
        self.sigmas_f = np.zeros((7, 3))
        c = self.ctx
        self._dx, self._dP = c.empty(3, np.float64), c.empty(9, np.float64)
        self._du, self._dz = c.empty(2, np.float64), c.empty(max(dim_z, 1), np.float64)
        self._dl, self._dR = c.empty(max(dim_z, 1), np.float64), c.empty(max(dim_z, 1), np.float64)
        self._ds = c.empty(21, np.float64)
        self._dsco = c.to_device(np.array([0, 0], np.int32))
        self._dcpo = c.to_device(np.array([0], np.int32))
        self._z_zero = np.zeros(dim_z)
        self._l_zero = np.zeros(dim_z)
        self._r_unused = np.ones(dim_z)

    def _step(self, flags, u, z, lmk, R_diag, dt):
        Q = np.asarray(self.Q, np.float64).reshape(9)
        for i in range(9):
            self.up.Q[i] = float(Q[i])
        self.up.dt = float(dt)
        self.up.flags = flags
        self._dx.upload(np.asarray(self.x, np.float64).reshape(3))
        self._dP.upload(np.asarray(self.P, np.float64).reshape(9))
        self._du.upload(np.asarray(u, np.float64).reshape(2))
        self._dz.upload(np.asarray(z, np.float64).reshape(self._dim_z))
        self._dl.upload(np.asarray(lmk, np.float64).reshape(self._dim_z))
        self._dR.upload(R_diag)
        self._ds.upload(np.asarray(self.sigmas_f, np.float64).reshape(21))
        b = _lib.ScanBatch()
        b.n_scans = 1
        b.scan_chunk_off, b.chunk_pt_off = self._dsco.addr, self._dcpo.addr
        b.ukf_x, b.ukf_P, b.ukf_u = self._dx.addr, self._dP.addr, self._du.addr
        b.ukf_z, b.ukf_lmk, b.ukf_R_diag = self._dz.addr, self._dl.addr, self._dR.addr
        b.ukf_sigmas = self._ds.addr
        _lib.check(_lib.load().lslam_ukf_step(self.ctx.handle, C.byref(b), C.byref(self.up)), "lslam_ukf_step")
        self.x = self._dx.download()
        self.P = self._dP.download().reshape(3, 3)
        self.sigmas_f = self._ds.download().reshape(7, 3)

    def predict(self, dt=None, UT=None, fx=None, **fx_args):
        """filterpy UKF.predict(dt=None, UT=None, fx=None, **fx_args) with fx =
        UKFMethods.transition_function(x, dt, u): ``u`` is required."""
        u, dt = predict_args(dt, UT, fx, fx_args, self.dt)
        self._step(_lib.UKF_PREDICT, u, self._z_zero, self._l_zero, self._r_unused, dt)  # predict reads no R
        self.x_prior, self.P_prior = self.x.copy(), self.P.copy()

    def update(self, z, R=None, UT=None, hx=None, **hx_args):
        """filterpy UKF.update(z, R=None, UT=None, hx=None, **hx_args) with hx =
        UKFMethods.transfer_function(x, landmarks): ``landmarks`` is required."""
        if z is None:
            self.x_post, self.P_post = self.x.copy(), self.P.copy()
            return
        Rd, lmk = update_args(R, UT, hx, hx_args, self.R, self._dim_z)
        self._step(_lib.UKF_UPDATE | _lib.UKF_SIGMAS_IN, (0.0, 0.0), z, lmk, Rd, self.dt)
        self.x_post, self.P_post = self.x.copy(), self.P.copy()


def predict_args(dt, UT, fx, fx_args, default_dt):
    """(u, dt) of a predict call, or the error filterpy's call would raise."""
    if UT is not None or fx is not None:
        raise ValueError("custom UT / fx are not supported: the GPU step implements UKFMethods.py's models")
    if "u" not in fx_args:
        raise TypeError("transition_function() missing 1 required positional argument: 'u'")
    extra = set(fx_args) - {"u"}
    if extra:
        raise TypeError("transition_function() got unexpected keyword arguments %s" % sorted(extra))
    return np.asarray(fx_args["u"], np.float64).reshape(2), (default_dt if dt is None else dt)


def update_args(R, UT, hx, hx_args, R_attr, dim_z):
    """(R diagonal, flattened landmark positions) of an update call, or the error."""
    if UT is not None or hx is not None:
        raise ValueError("custom UT / hx are not supported: the GPU step implements UKFMethods.py's models")
    if "landmarks" not in hx_args:
        raise TypeError("transfer_function() missing 1 required positional argument: 'landmarks'")
    extra = set(hx_args) - {"landmarks"}
    if extra:
        raise TypeError("transfer_function() got unexpected keyword arguments %s" % sorted(extra))
    if R is None:
        R = R_attr
    elif np.isscalar(R):
        R = np.eye(dim_z) * R
    Rd = _diag_of(R, dim_z)
    pos = [np.asarray(l.get_pos() if hasattr(l, "get_pos") else l, np.float64)[:2] for l in hx_args["landmarks"]]
    if len(pos) * 2 != dim_z:
        raise ValueError("expected %d landmarks for dim_z=%d, got %d" % (dim_z // 2, dim_z, len(pos)))
    return Rd, np.concatenate(pos)
