"""ORACLE — TEST INFRASTRUCTURE ONLY.  NumPy restatement of the intended UKF.

PARITY UNPINNED.  The reference UKF cannot run: ``UKFMethods.py`` is a
SyntaxError at line 40 and ``systemClass.py`` at line 4, nothing imports
``systemClass`` (SLAM.py:1-4), and filterpy (the third-party engine it
configures, version 1.4.5 era, not vendored) is absent from the container.
This module restates, as literally as NumPy allows:

* UKFMethods.py:10-14   normalize_angle (Python float %, then -2pi above pi)
* UKFMethods.py:17-24   transition_function, intended: x + dt * B(theta) u
* UKFMethods.py:26-34   transfer_function: per landmark [dist, wrap(atan2 - theta)]
* UKFMethods.py:37-57   state_mean / z_mean, intended: weighted sums, angles via
                        atan2(sum W sin, sum W cos)
* UKFMethods.py:60-71   residual_x / residual_h (wrap angle components)
* systemClass.py:7-29   n=3, MerweScaledSigmaPoints(alpha=1e-4, beta=2, kappa=0),
                        dt = DT = 0.005, P0 = diag(.1,.1,.05), R = diag([.25,.09]*L),
                        Q = 1e-3 I
* filterpy 1.4.5        MerweScaledSigmaPoints.sigma_points/_compute_weights,
                        unscented_transform (loop form when residual_fn given),
                        UnscentedKalmanFilter.predict/update/cross_variance,
                        scipy.linalg.cholesky (upper), np.linalg.inv for S^-1.

Self-pinned by known-answer tests (tests/test_ukf_oracle.py): linear models
reduce to the Kalman filter, the weights of systemClass.py:20, wrap edge cases.
"""
from __future__ import annotations

import math

import numpy as np
import scipy.linalg

R_WHEEL = 50.0   # UKFMethods.py:6
L_BASE = 200.0   # UKFMethods.py:7
DT = 0.005       # systemClass.py:10
VAR_DIST = 0.5 ** 2   # systemClass.py:8
VAR_ANGLE = 0.3 ** 2  # systemClass.py:9


def normalize_angle(angle):
    angle = angle % (2 * np.pi)
    if angle > np.pi:
        angle -= 2 * np.pi
    return angle


def transition_function(x, dt, u):
    c = R_WHEEL / 2.0 * math.cos(x[2])
    s = R_WHEEL / 2.0 * math.sin(x[2])
    bx = np.array([[c, c], [s, s], [-1.0 * R_WHEEL / L_BASE, 1.0 * R_WHEEL / L_BASE]])
    return np.dot(np.identity(x.shape[0]), x) + dt * np.dot(bx, u)


def transfer_function(x, landmarks):
    hx = []
    for (px, py) in landmarks:
        dist = math.sqrt((px - x[0]) ** 2 + (py - x[1]) ** 2)
        angle = math.atan2(py - x[1], px - x[0])
        hx.extend([dist, normalize_angle(angle - x[2])])
    return np.array(hx)


def state_mean(sigmas, Wm):
    x = np.zeros(3)
    sum_sin = np.dot(np.sin(sigmas[:, 2]), Wm)
    sum_cos = np.dot(np.cos(sigmas[:, 2]), Wm)
    x[0] = np.dot(sigmas[:, 0], Wm)
    x[1] = np.dot(sigmas[:, 1], Wm)
    x[2] = math.atan2(sum_sin, sum_cos)
    return x


def z_mean(sigmas, Wm):
    n = sigmas.shape[1]
    x = np.zeros(n)
    for z in range(0, n, 2):
        sum_sin = np.dot(np.sin(sigmas[:, z + 1]), Wm)
        sum_cos = np.dot(np.cos(sigmas[:, z + 1]), Wm)
        x[z] = np.dot(sigmas[:, z], Wm)
        x[z + 1] = math.atan2(sum_sin, sum_cos)
    return x


# The same means evaluated about sigma point 0: sum W s = s_0 + sum W (s - s_0) and
# atan2(sum W sin a, sum W cos a) = a_0 + atan2(sum W sin(a - a_0), sum W cos(a - a_0)),
# identical in exact arithmetic (the weights sum to 1).  In float64 the alpha = 1e-4
# weights (~-1e8, 1.7e7) sum to 1 - 1.1e-8, which biases the literal sums by 1.1e-8 |s|
# and, through the (Wc0 - Wm0) term of the covariance, P by ~1e-5 relative
# (tests/test_ukf_exact.py measures both forms against a 50-digit evaluation).  The HIP
# kernel (lslam_ukf.h) uses this form.
def state_mean_centred(sigmas, Wm):
    d = sigmas - sigmas[0]
    x = np.zeros(3)
    x[0] = sigmas[0, 0] + np.dot(d[:, 0], Wm)
    x[1] = sigmas[0, 1] + np.dot(d[:, 1], Wm)
    x[2] = normalize_angle(sigmas[0, 2] + math.atan2(np.dot(np.sin(d[:, 2]), Wm), np.dot(np.cos(d[:, 2]), Wm)))
    return x


def z_mean_centred(sigmas, Wm):
    n = sigmas.shape[1]
    d = sigmas - sigmas[0]
    x = np.zeros(n)
    for z in range(0, n, 2):
        x[z] = sigmas[0, z] + np.dot(d[:, z], Wm)
        x[z + 1] = normalize_angle(sigmas[0, z + 1] + math.atan2(np.dot(np.sin(d[:, z + 1]), Wm),
                                                                 np.dot(np.cos(d[:, z + 1]), Wm)))
    return x


def residual_x(a, b):
    y = a - b
    y[2] = normalize_angle(y[2])
    return y


def residual_h(a, b):
    y = a - b
    for i in range(0, len(y), 2):
        y[i + 1] = normalize_angle(y[i + 1])
    return y


class MerweScaledSigmaPoints:
    def __init__(self, n, alpha, beta, kappa):
        self.n, self.alpha, self.beta, self.kappa = n, alpha, beta, kappa
        lambda_ = alpha ** 2 * (n + kappa) - n
        c = .5 / (n + lambda_)
        self.Wc = np.full(2 * n + 1, c)
        self.Wm = np.full(2 * n + 1, c)
        self.Wc[0] = lambda_ / (n + lambda_) + (1 - alpha ** 2 + beta)
        self.Wm[0] = lambda_ / (n + lambda_)

    def sigma_points(self, x, P):
        n = self.n
        lambda_ = self.alpha ** 2 * (n + self.kappa) - n
        U = scipy.linalg.cholesky((lambda_ + n) * P)
        sigmas = np.zeros((2 * n + 1, n))
        sigmas[0] = x
        for k in range(n):
            sigmas[k + 1] = np.subtract(x, -U[k])
            sigmas[n + k + 1] = np.subtract(x, U[k])
        return sigmas


def unscented_transform(sigmas, Wm, Wc, noise_cov, mean_fn, residual_fn):
    kmax, n = sigmas.shape
    x = mean_fn(sigmas, Wm)
    P = np.zeros((n, n))
    for k in range(kmax):
        y = residual_fn(sigmas[k], x)
        P += Wc[k] * np.outer(y, y)
    if noise_cov is not None:
        P += noise_cov
    return x, P


class UKF:
    """filterpy UnscentedKalmanFilter as configured by systemClass.py:21-29."""

    def __init__(self, n_landmarks, dt=DT, alpha=1e-4, beta=2.0, kappa=0.0, fx=transition_function,
                 hx=transfer_function, x_mean=state_mean_centred, z_mean_fn=z_mean_centred, res_x=residual_x,
                 res_z=residual_h):
        self.points = MerweScaledSigmaPoints(3, alpha, beta, kappa)
        self.Wm, self.Wc = self.points.Wm, self.points.Wc
        self.dt = dt
        self.fx, self.hx = fx, hx
        self.x_mean, self.z_mean = x_mean, z_mean_fn
        self.residual_x, self.residual_z = res_x, res_z
        self.x = np.zeros(3)
        self.P = np.diag([.1, .1, 0.05])
        self.R = np.diag([VAR_DIST, VAR_ANGLE] * n_landmarks)
        self.Q = np.eye(3) * 0.001
        self.sigmas_f = np.zeros((7, 3))

    def predict(self, u):
        sigmas = self.points.sigma_points(self.x, self.P)
        for i, s in enumerate(sigmas):
            self.sigmas_f[i] = self.fx(s, self.dt, u)
        self.x, self.P = unscented_transform(self.sigmas_f, self.Wm, self.Wc, self.Q, self.x_mean,
                                             self.residual_x)
        self.sigmas_f = self.points.sigma_points(self.x, self.P)

    def update(self, z, landmarks):
        sigmas_h = np.atleast_2d([self.hx(s, landmarks) for s in self.sigmas_f])
        zp, S = unscented_transform(sigmas_h, self.Wm, self.Wc, self.R, self.z_mean, self.residual_z)
        SI = np.linalg.inv(S)
        Pxz = np.zeros((3, sigmas_h.shape[1]))
        for i in range(sigmas_h.shape[0]):
            dx = self.residual_x(self.sigmas_f[i], self.x)
            dz = self.residual_z(sigmas_h[i], zp)
            Pxz += self.Wc[i] * np.outer(dx, dz)
        K = np.dot(Pxz, SI)
        y = self.residual_z(np.asarray(z, np.float64), zp)
        self.x = np.add(self.x, np.dot(K, y))
        self.P = self.P - np.dot(K, np.dot(S, K.T))


def ukf_batch(x, P, u, z, lmk, R_diag, dt=DT, predict=True, update=True, Q=None, centred=True):
    """Run one predict/update per scan; returns (x[S,3], P[S,3,3]).  ``centred=False``: filterpy's
    literal float64 means (state_mean / z_mean above) instead of the centred form."""
    S = x.shape[0]
    L = lmk.shape[1]
    xo = np.zeros((S, 3))
    Po = np.zeros((S, 3, 3))
    means = {} if centred else dict(x_mean=state_mean, z_mean_fn=z_mean)
    for s in range(S):
        f = UKF(L, dt=dt, **means)
        f.x = np.array(x[s], np.float64)
        f.P = np.array(P[s], np.float64).reshape(3, 3)
        f.R = np.diag(np.asarray(R_diag, np.float64))
        if Q is not None:
            f.Q = np.asarray(Q, np.float64).reshape(3, 3)
        if predict:
            f.predict(np.asarray(u[s], np.float64))
        else:
            f.sigmas_f = f.points.sigma_points(f.x, f.P)
        if update:
            f.update(z[s], [tuple(p) for p in lmk[s]])
        xo[s] = f.x
        Po[s] = f.P
    return xo, Po
