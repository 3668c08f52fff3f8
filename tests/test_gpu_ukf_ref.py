"""U4 / U6 on the GPU against the reference's own functions (tests/golden/ukf_ref.npz:
UKFMethods.py normalize_angle :10-14, transfer_function :26-34, residual_x :60-63,
residual_h :66-71, run as written; tests/test_ukf_ref.py pins oracle/ukf.py to them bit
for bit).  The kernel's intermediate values come from lslam_ukf_trace, which runs the
lane-group UKF step of lslam_ukf_step with extra stores.

Bounds, all stated here:
* hx(sigma_0) against the fixture (update-only step: sigma_0 = x exactly): distances
  within 1 ulp, and bit-exact for at least 99 % of them: the kernel squares with one
  correctly rounded multiply, the reference with ``(px - x[0])**2`` (UKFMethods.py:31),
  i.e. glibc's pow(d, 2), which is 1 ulp off d*d for a few arguments (3 of the 800 c5
  distances); the sum and the square root round identically;
  bearings within BEARING_ULP ulp of max(pi, |theta|), compared modulo 2 pi (the GPU's
  atan2 is OCML's, the reference's glibc's; both are faithful, not correctly rounded:
  fl(atan2 - theta) then differs by at most a unit of theta's spacing).  Headings beyond
  BIG_THETA = 1e6 (the edge case's +-1e15 and +-1e300), where that spacing approaches or
  exceeds 2 pi and the modulo-2-pi check would be vacuous, are held bit-exact instead:
  there fl(atan2 - theta) absorbs atan2's last bits except at a rounding boundary, with
  probability ~ 2 ulp(pi) / spacing(theta) per bearing (7e-15 at 1e15; it would be 8e-6 at
  1e6 and 5e-4 at 1e4, so headings up to 1e6 take the tolerance check, 2.3e-10 at 1e6).
  The edge case's landmarks dead ahead / dead behind (atan2 = +0 / pi exactly on both
  sides) are bit-exact: there the bearing IS normalize_angle(a) for the edge angles a.
* the wraps inside the step, BIT-EXACT against the oracle's restatement (pinned to the
  reference) evaluated on the kernel's own inputs: residual_x(sigma_k, x),
  residual_h(z, zp), residual_h(hx(sigma_k), zp).
* hx(sigma_k) for k = 1..6 against the oracle's transfer_function on the kernel's
  sigma points, at the same bounds as sigma_0.
"""
import numpy as np
import pytest

from oracle import ukf as oukf

pytestmark = pytest.mark.gpu

BEARING_ULP = 2
BIG_THETA = 1e6


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def _bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def _trace(ctx, g, case):
    from lidar_slam_amd import _lib
    from lidar_slam_amd.pipeline import ScanPipeline
    x, lm = g[case + "_x"], g[case + "_lmk"]
    S, L = lm.shape[:2]
    p = ScanPipeline(ctx, np.zeros((1, 2)), np.zeros(S + 1, np.int32), np.zeros(1, np.int32),
                     ukf=dict(n_landmarks=L, x=x, P=g[case + "_P"], u=np.zeros((S, 2)), z=g[case + "_z"], lmk=lm,
                              R_diag=g[case + "_R_diag"], flags=_lib.UKF_UPDATE))
    return p.run_ukf_trace()


def _bearing_err(a, b):
    d = np.abs(a - b)
    return np.minimum(d, 2 * np.pi - d)


def _check_hx(hx_gpu, hx_ref, theta):
    """distances within 1 ulp, bearings within BEARING_ULP ulp of max(pi, |theta|) modulo
    2 pi; returns (bit-exact distances, distances) for the caller's >= 99 % check"""
    dg, dr = hx_gpu[..., 0::2], hx_ref[..., 0::2]
    assert np.all(np.abs(dg - dr) <= np.spacing(dr))
    theta = np.asarray(theta, np.float64)
    big = np.abs(theta) > BIG_THETA
    bg, br = hx_gpu[..., 1::2], hx_ref[..., 1::2]
    assert np.array_equal(_bits(bg[big]), _bits(br[big]))
    tol = BEARING_ULP * np.spacing(np.maximum(np.pi, np.abs(theta[~big])))
    assert np.all(tol < 1e-9)  # never vacuous
    err = _bearing_err(bg[~big], br[~big])
    assert np.all(err <= tol[..., None]), float(np.max(err / tol[..., None]))
    return int(np.sum(dg == dr)), dg.size


@pytest.mark.parametrize("case", ["c3", "c5", "edge"])
def test_hx_sigma0_vs_reference(ctx, golden, case):
    g = golden("ukf_ref.npz")
    t = _trace(ctx, g, case)
    x = g[case + "_x"]
    assert np.array_equal(_bits(t["sigmas"][:, 0]), _bits(x))  # update-only: sigma_0 = x
    same, n = _check_hx(t["hx"][:, 0], g[case + "_hx"], x[:, 2])
    assert same >= 0.99 * n, (same, n)
    if case == "edge":
        # dead ahead: bearing = normalize_angle(a); dead behind: normalize_angle(pi + a) -- bit-exact
        assert np.array_equal(_bits(t["hx"][:, 0, 1]), _bits(g["edge_hx"][:, 1]))
        assert np.array_equal(_bits(t["hx"][:, 0, 3]), _bits(g["edge_hx"][:, 3]))


@pytest.mark.parametrize("case", ["c3", "c5", "edge"])
def test_wraps_bitwise_on_kernel_inputs(ctx, golden, case):
    g = golden("ukf_ref.npz")
    t = _trace(ctx, g, case)
    x, z = g[case + "_x"], g[case + "_z"]
    with np.errstate(invalid="ignore"):
        for s in range(len(x)):
            for k in range(7):
                assert np.array_equal(_bits(t["dx"][s, k]), _bits(oukf.residual_x(t["sigmas"][s, k].copy(), x[s])))
                assert np.array_equal(_bits(t["rz"][s, k]), _bits(oukf.residual_h(t["hx"][s, k].copy(), t["zp"][s])))
            assert np.array_equal(_bits(t["y"][s]), _bits(oukf.residual_h(z[s].copy(), t["zp"][s])))


@pytest.mark.parametrize("case", ["c3", "c5"])
def test_hx_all_sigmas_vs_oracle(ctx, golden, case):
    g = golden("ukf_ref.npz")
    t = _trace(ctx, g, case)
    lm = g[case + "_lmk"]
    same = n = 0
    for s in range(len(lm)):
        want = np.stack([oukf.transfer_function(t["sigmas"][s, k], [tuple(p) for p in lm[s]]) for k in range(7)])
        a, b = _check_hx(t["hx"][s], want, t["sigmas"][s, :, 2])
        same, n = same + a, n + b
    assert same >= 0.99 * n, (same, n)
