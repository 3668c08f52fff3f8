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


def test_centred_means_equal_literal_up_to_the_weight_sum():
    """state_mean_centred and state_mean are the same mean; in float64 they differ by the
    literal form's bias (1 - sum Wm) * s (sum Wm = 1 - 1.1e-8 for alpha = 1e-4)."""
    rng = np.random.default_rng(11)
    pts = oukf.MerweScaledSigmaPoints(3, 1e-4, 2.0, 0.0)
    bias = 1.0 - math.fsum(pts.Wm)
    for _ in range(16):
        x0 = np.array([rng.uniform(800, 3200), rng.uniform(800, 2200), rng.uniform(-3.0, 3.0)])
        sig = pts.sigma_points(x0, np.diag([.1, .1, .05]))
        lit, cen = oukf.state_mean(sig, pts.Wm), oukf.state_mean_centred(sig, pts.Wm)
        assert np.all(np.abs(lit[:2] - cen[:2]) <= 3 * abs(bias) * np.abs(x0[:2]) + 1e-9)
        assert abs(lit[2] - cen[2]) < 1e-7
