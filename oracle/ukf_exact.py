"""ORACLE — TEST INFRASTRUCTURE ONLY.  The UKF of ``oracle/ukf.py`` evaluated with
50 significant digits (mpmath), the reference point of every float64 UKF here.

PARITY UNPINNED, as for oracle/ukf.py: the reference UKF does not parse
(UKFMethods.py:40, systemClass.py:4) and filterpy is absent, so no output of the
reference exists.  What this module pins is the ROUNDING: it runs the same
steps as oracle/ukf.py (same formulas, same sigma order, the mathematical pi)
in 50-digit arithmetic, so the difference between a float64 implementation
(the NumPy oracle, the HIP kernel) and this is that implementation's own error.

  weights          systemClass.py:20   MerweScaledSigmaPoints(3, alpha, beta, kappa)
  sigma points     filterpy            U = chol((n+lambda) P) upper; x, x + U[k], x - U[k]
  transition (fx)  UKFMethods.py:17-24 x + dt B(theta) u, R = 50, L = 200
  transfer (hx)    UKFMethods.py:26-34 [dist, wrap(atan2 - theta)] per landmark
  means            UKFMethods.py:37-57 weighted sums, angles via atan2 of weighted sin / cos
  residuals        UKFMethods.py:10-14,60-71 (floor-mod by 2 pi, then -2 pi above pi)
  predict/update   filterpy 1.4.5 UnscentedKalmanFilter:
                   x, P = UT(fx(sigmas)) + Q; sigmas_f re-drawn from (x, P);
                   S = sum Wc rz rz^T + R; Pxz = sum Wc rx rz^T; K = Pxz S^-1;
                   x += K residual_h(z, zp); P -= K S K^T = Pxz S^-1 Pxz^T.

Inputs are float64 numbers taken exactly (alpha etc. are the float64 constants'
exact values).  S^-1 is applied through the Woodbury identity
S^-1 = R^-1 - R^-1 Y (W^-1 + Y^T R^-1 Y)^-1 Y^T R^-1 (Y = [rz_0 .. rz_6],
W = diag(Wc)), which equals the dense inverse in exact arithmetic (checked
against mpmath's dense LU solve in tests/test_ukf_exact.py) and keeps L = 200
(dim_z = 400) cheap.
"""
from __future__ import annotations

import mpmath as mp
import numpy as np

DPS = 50
R_WHEEL = 50.0   # UKFMethods.py:6
L_BASE = 200.0   # UKFMethods.py:7
DT = 0.005       # systemClass.py:10


def _f(v):
    return mp.mpf(float(v))


def normalize_angle(a):
    tp = 2 * mp.pi
    a = a - tp * mp.floor(a / tp)
    if a > mp.pi:
        a -= tp
    return a


def weights(alpha=1e-4, beta=2.0, kappa=0.0, n=3):
    al, be, ka = _f(alpha), _f(beta), _f(kappa)
    lam = al ** 2 * (n + ka) - n
    c = mp.mpf(1) / (2 * (n + lam))
    Wm = [c] * (2 * n + 1)
    Wc = [c] * (2 * n + 1)
    Wm[0] = lam / (n + lam)
    Wc[0] = Wm[0] + (1 - al ** 2 + be)
    return Wm, Wc, lam + n


def sigma_points(x, P, lpn):
    A = mp.matrix(3, 3)
    for i in range(3):
        for j in range(3):
            A[i, j] = lpn * P[i][j]
    Lo = mp.cholesky(A)           # A = Lo Lo^T; filterpy's upper factor U = Lo^T, U[k] = column k of Lo
    sig = [list(x)]
    for k in range(3):
        sig.append([x[j] + Lo[j, k] for j in range(3)])
    for k in range(3):
        sig.append([x[j] - Lo[j, k] for j in range(3)])
    return sig


def fx(s, dt, u):
    c = _f(R_WHEEL) / 2 * mp.cos(s[2])
    sn = _f(R_WHEEL) / 2 * mp.sin(s[2])
    k0, k1 = -_f(R_WHEEL) / _f(L_BASE), _f(R_WHEEL) / _f(L_BASE)
    return [s[0] + dt * (c * u[0] + c * u[1]), s[1] + dt * (sn * u[0] + sn * u[1]), s[2] + dt * (k0 * u[0] + k1 * u[1])]


def hx(s, lmk):
    out = []
    for px, py in lmk:
        dx, dy = px - s[0], py - s[1]
        out.append(mp.sqrt(dx * dx + dy * dy))
        out.append(normalize_angle(mp.atan2(dy, dx) - s[2]))
    return out


def _wsum(vals, W):
    return mp.fsum(w * v for w, v in zip(W, vals))


def state_mean(sig, Wm):
    return [_wsum([s[0] for s in sig], Wm), _wsum([s[1] for s in sig], Wm),
            mp.atan2(_wsum([mp.sin(s[2]) for s in sig], Wm), _wsum([mp.cos(s[2]) for s in sig], Wm))]


def z_mean(sh, Wm):
    m = len(sh[0])
    out = []
    for j in range(0, m, 2):
        out.append(_wsum([s[j] for s in sh], Wm))
        out.append(mp.atan2(_wsum([mp.sin(s[j + 1]) for s in sh], Wm), _wsum([mp.cos(s[j + 1]) for s in sh], Wm)))
    return out


def residual_x(a, b):
    return [a[0] - b[0], a[1] - b[1], normalize_angle(a[2] - b[2])]


def residual_h(a, b):
    return [normalize_angle(ai - bi) if j % 2 else ai - bi for j, (ai, bi) in enumerate(zip(a, b))]


def _solve7(M, v):
    return list(mp.lu_solve(M, mp.matrix(v)))


def step(x, P, u, z, lmk, R_diag, dt=DT, Q=None, alpha=1e-4, beta=2.0, kappa=0.0, predict=True, update=True,
         dense=False, sigmas=None):
    """One predict + update (either may be skipped) of one filter.  Arguments are float64
    arrays; returns (x[3], P[3][3]) as mpf lists.  ``dense`` applies S^-1 by an LU solve of
    the 2L x 2L S instead of the Woodbury form (the cross-check).  ``sigmas`` (7 x 3 float64,
    update only): filterpy's cached sigmas_f, used with the given x and P instead of sigma
    points drawn from them (filterpy's update after x or P was reassigned)."""
    with mp.workdps(DPS):
        Wm, Wc, lpn = weights(alpha, beta, kappa)
        xs = [_f(v) for v in np.asarray(x, np.float64).reshape(3)]
        Ps = [[_f(v) for v in row] for row in np.asarray(P, np.float64).reshape(3, 3)]
        Qm = np.eye(3) * 0.001 if Q is None else np.asarray(Q, np.float64).reshape(3, 3)
        Qs = [[_f(v) for v in row] for row in Qm]
        dts = _f(dt)
        us = [_f(v) for v in np.asarray(u, np.float64).reshape(2)]
        if predict:
            sf = [fx(s, dts, us) for s in sigma_points(xs, Ps, lpn)]
            xs = state_mean(sf, Wm)
            Pn = [[mp.mpf(0)] * 3 for _ in range(3)]
            for k in range(7):
                y = residual_x(sf[k], xs)
                for i in range(3):
                    for j in range(3):
                        Pn[i][j] += Wc[k] * (y[i] * y[j])
            Ps = [[Pn[i][j] + Qs[i][j] for j in range(3)] for i in range(3)]
        if not update:
            return xs, Ps
        if sigmas is not None and not predict:
            sf = [[_f(v) for v in row] for row in np.asarray(sigmas, np.float64).reshape(7, 3)]
        else:
            sf = sigma_points(xs, Ps, lpn)
        lm = [(_f(px), _f(py)) for px, py in np.asarray(lmk, np.float64).reshape(-1, 2)]
        sh = [hx(s, lm) for s in sf]
        zp = z_mean(sh, Wm)
        m = len(zp)
        Rd = [_f(v) for v in np.asarray(R_diag, np.float64).reshape(m)]
        rz = [residual_h(sh[k], zp) for k in range(7)]      # Y columns
        rx = [residual_x(sf[k], xs) for k in range(7)]
        Pxz = [[mp.fsum(Wc[k] * rx[k][i] * rz[k][q] for k in range(7)) for q in range(m)] for i in range(3)]
        y = residual_h([_f(v) for v in np.asarray(z, np.float64).reshape(m)], zp)
        if dense:
            S = mp.matrix(m, m)
            for a in range(m):
                for c in range(m):
                    S[a, c] = mp.fsum(Wc[k] * rz[k][a] * rz[k][c] for k in range(7)) + (Rd[a] if a == c else 0)

            def sinv(v):
                return list(mp.lu_solve(S, mp.matrix(v)))
        else:
            Ri = [1 / r for r in Rd]
            M = mp.matrix(7, 7)
            for k in range(7):
                for l2 in range(7):
                    M[k, l2] = mp.fsum(rz[k][q] * Ri[q] * rz[l2][q] for q in range(m)) + (1 / Wc[k] if k == l2 else 0)

            def sinv(v):
                t = [Ri[q] * v[q] for q in range(m)]
                w = _solve7(M, [mp.fsum(rz[k][q] * t[q] for q in range(m)) for k in range(7)])
                return [t[q] - Ri[q] * mp.fsum(rz[k][q] * w[k] for k in range(7)) for q in range(m)]

        Kt = [sinv(Pxz[i]) for i in range(3)]                 # rows of K = Pxz S^-1 (S symmetric)
        xn = [xs[i] + mp.fsum(Kt[i][q] * y[q] for q in range(m)) for i in range(3)]
        Pn = [[Ps[i][j] - mp.fsum(Kt[i][q] * Pxz[j][q] for q in range(m)) for j in range(3)] for i in range(3)]
        return xn, Pn


def to_float(xs, Ps):
    return np.array([float(v) for v in xs]), np.array([[float(v) for v in row] for row in Ps])


def ukf_batch_exact(x, P, u, z, lmk, R_diag, **kw):
    """``oracle.ukf.ukf_batch`` in 50 digits: (x[S,3], P[S,3,3]) rounded once to float64."""
    S = x.shape[0]
    xo, Po = np.zeros((S, 3)), np.zeros((S, 3, 3))
    for s in range(S):
        xo[s], Po[s] = to_float(*step(x[s], P[s], u[s], z[s], lmk[s], R_diag, **kw))
    return xo, Po


def component_errors(x, P, x_ref, P_ref):
    """Per-scan error components against a reference (the exact values):
    x, y relative to |x_ref|, theta absolute (wrapped), P relative to max|P_ref|."""
    x, P, x_ref, P_ref = (np.asarray(a, np.float64) for a in (x, P, x_ref, P_ref))
    rel_xy = np.abs(x[:, :2] - x_ref[:, :2]) / np.maximum(np.abs(x_ref[:, :2]), 1.0)
    dth = np.abs((x[:, 2] - x_ref[:, 2] + np.pi) % (2 * np.pi) - np.pi)
    scale = np.max(np.abs(P_ref.reshape(len(P_ref), -1)), axis=1)
    rel_P = np.max(np.abs((P - P_ref).reshape(len(P), -1)), axis=1) / scale
    return {"x_rel": float(rel_xy[:, 0].max()), "y_rel": float(rel_xy[:, 1].max()), "theta_abs": float(dth.max()),
            "P_rel": float(rel_P.max())}
