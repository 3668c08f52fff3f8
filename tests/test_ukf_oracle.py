"""Self-pinning of the UKF oracle (PARITY UNPINNED: the reference UKF does not
parse and filterpy is absent).  Known answers: the weights of systemClass.py:20,
normalize_angle edge cases, linear models reduce to the Kalman filter, and the
rounding-noise floor that bounds every UKF parity tolerance."""
import math

import numpy as np

from oracle import ukf as oukf


def test_weights_systemclass():
    pts = oukf.MerweScaledSigmaPoints(3, 1e-4, 2.0, 0.0)
    assert abs(pts.Wm[0] - (-99999999.6077)) < 1e-3
    assert abs(pts.Wc[0] - (-99999996.6077)) < 1e-3
    assert abs(pts.Wm[1] - 16666666.768) < 1e-3
    assert abs(np.sum(pts.Wm) - 1.0) < 1e-7


def test_normalize_angle_edges():
    f = oukf.normalize_angle
    assert f(0.0) == 0.0
    assert f(np.pi) == np.pi
    assert abs(f(-np.pi) - np.pi) < 1e-15          # -pi maps to +pi: range (-pi, pi]
    assert f(2 * np.pi) == 0.0
    assert abs(f(3 * np.pi / 2) + np.pi / 2) < 1e-15
    assert abs(f(-3 * np.pi / 2) - np.pi / 2) < 1e-15
    assert abs(f(7.0) - (7.0 - 2 * np.pi)) < 1e-15


def test_linear_ukf_equals_kalman():
    """With linear fx/hx and identity residuals the UT is exact: UKF == KF."""
    A = np.array([[1.0, 0.1, 0.0], [0.0, 1.0, 0.1], [0.0, 0.0, 1.0]])
    H = np.array([[1.0, 0.0, 0.0], [0.0, 0.0, 1.0]])
    f = oukf.UKF(1, alpha=1.0, beta=2.0, kappa=0.0,
                 fx=lambda x, dt, u: A @ x, hx=lambda x, lm: H @ x,
                 x_mean=lambda s, W: W @ s, z_mean_fn=lambda s, W: W @ s,
                 res_x=np.subtract, res_z=np.subtract)
    f.x = np.array([1.0, 2.0, 0.3])
    f.P = np.array([[0.5, 0.1, 0.0], [0.1, 0.4, 0.05], [0.0, 0.05, 0.3]])
    f.R = np.diag([0.2, 0.1])
    x, P = f.x.copy(), f.P.copy()
    f.predict(np.zeros(2))
    x = A @ x
    P = A @ P @ A.T + f.Q
    assert np.allclose(f.x, x, atol=1e-12) and np.allclose(f.P, P, atol=1e-12)
    z = np.array([1.5, 0.1])
    f.update(z, None)
    S = H @ P @ H.T + f.R
    K = P @ H.T @ np.linalg.inv(S)
    x = x + K @ (z - H @ x)
    P = P - K @ S @ K.T
    assert np.allclose(f.x, x, atol=1e-10) and np.allclose(f.P, P, atol=1e-10)


def _exact_state_mean(sigmas, Wm):
    x = np.zeros(3)
    x[0] = math.fsum(sigmas[:, 0] * Wm)
    x[1] = math.fsum(sigmas[:, 1] * Wm)
    x[2] = math.atan2(math.fsum(np.sin(sigmas[:, 2]) * Wm), math.fsum(np.cos(sigmas[:, 2]) * Wm))
    return x


def test_noise_floor_of_alpha_1e4():
    """Two summation orders of the SAME algorithm differ at the level the GPU
    parity tolerance allows (|dx| ~1e-6..1e-4, |dP| ~1e-8): the floor is the
    cancellation of the +-1e8 weights, not an implementation error."""
    rng = np.random.default_rng(11)
    dxs, dPs = [], []
    for s in range(16):
        L = 20
        x0 = np.array([rng.uniform(800, 3200), rng.uniform(800, 2200), rng.uniform(-np.pi, np.pi)])
        lmk = [tuple(p) for p in rng.uniform(-3000, 3000, (L, 2))]
        z = oukf.transfer_function(x0, lmk) + rng.normal(0, 0.3, 2 * L)
        outs = []
        for mean_fn in (oukf.state_mean, _exact_state_mean):
            f = oukf.UKF(L, x_mean=mean_fn)
            f.x = x0.copy()
            f.predict(np.array([2.0, 2.5]))
            f.update(z, lmk)
            outs.append((f.x.copy(), f.P.copy()))
        dxs.append(np.max(np.abs(outs[0][0] - outs[1][0])))
        dPs.append(np.max(np.abs(outs[0][1] - outs[1][1])))
    assert max(dPs) < 1e-6 and max(dxs) < 1e-4
    assert max(dPs) > 1e-10  # the spread is real, not zero
