"""U4 / U6 pinned to the reference's own code: tests/golden/ukf_ref.npz holds the outputs
of UKFMethods.py's normalize_angle (:10-14), transfer_function (:26-34), residual_x
(:60-63) and residual_h (:66-71), run as written on reference landmarking.Landmark
objects (tests/golden/make_ukf_ref.py).

* oracle/ukf.py must reproduce every output BIT FOR BIT (it is the checker the GPU
  tests use for the kernel's sigma points, tests/test_gpu_ukf_ref.py).
* oracle/ukf_exact.py evaluates the same formulas in 50 digits with the mathematical
  pi, so it cannot be bit-exact: its rounded values are held to 1 ulp on distances and
  4 ulp of max(pi, |theta|) on bearings (the reference's angle - theta and its floor-mod
  by the float64 2 pi round at theta's scale), for headings |theta| <= 1e4.  Beyond that the
  reference's floor-mod by the float64 2 pi and the exact one drift apart (at 1e15 rad
  the two wraps differ by O(1)), which is the reference's own float semantics.
"""
import mpmath as mp
import numpy as np
import pytest

from oracle import ukf as oukf
from oracle import ukf_exact as ux

DIST_REL = 2.0 ** -52      # 1 ulp


def _bits(a):
    return np.asarray(a, np.float64).view(np.int64)


def test_fixture_records_what_ran(golden):
    g = golden("ukf_ref.npz")
    spans = [s.split()[0] for s in g["meta_blocks"]]
    # the four functions (10-14, 26-34, 60-63, 66-71), numpy / math imports, R, L, dt (6-8)
    for want in ("10-", "26-", "60-", "66-", "1-", "2-", "6-", "7-", "8-"):
        assert any(s.startswith(want) for s in spans), (want, spans)
    assert not any(s.startswith(("3-", "4-", "37-", "47-")) for s in spans), spans  # filterpy, state_mean, z_mean


def test_normalize_angle_bitwise(golden):
    g = golden("ukf_ref.npz")
    with np.errstate(invalid="ignore"):
        mine = np.array([oukf.normalize_angle(float(v)) for v in g["norm_in"]])
        mine64 = np.array([oukf.normalize_angle(np.float64(v)) for v in g["norm_in"]])
    assert np.array_equal(_bits(mine), _bits(g["norm_out"]))
    assert np.array_equal(_bits(mine64), _bits(g["norm_out"]))
    # the edges are in there: -0.0 -> +0.0, pi stays, pi + 1 ulp wraps, 2 pi -> 0
    ea, out = g["edge_angles"], g["norm_out"]
    idx = {float(v): i for i, v in enumerate(ea) if v != 0}
    assert _bits(out[1]) == 0 and out[idx[np.pi]] == np.pi and out[idx[float(np.nextafter(np.pi, 4))]] < 0
    assert out[idx[2 * np.pi]] == 0.0


@pytest.mark.parametrize("case", ["c3", "c5", "edge"])
def test_transfer_function_bitwise(golden, case):
    g = golden("ukf_ref.npz")
    x, lm = g[case + "_x"], g[case + "_lmk"]
    mine = np.stack([oukf.transfer_function(np.array(x[s]), [tuple(p) for p in lm[s]]) for s in range(len(x))])
    assert np.array_equal(_bits(mine), _bits(g[case + "_hx"]))


def test_edge_bearings_are_the_wrap(golden):
    """Landmark 0 dead ahead: bearing = normalize_angle(edge angle); landmark 1 dead behind:
    normalize_angle(pi + edge angle) (the fixture's own construction)."""
    g = golden("ukf_ref.npz")
    ea, hx = g["edge_angles"], g["edge_hx"]
    want0 = np.array([oukf.normalize_angle(0.0 - (-a)) for a in ea])
    assert np.array_equal(_bits(hx[:, 1]), _bits(want0))
    want1 = np.array([oukf.normalize_angle(np.pi - (-a)) for a in ea])
    assert np.array_equal(_bits(hx[:, 3]), _bits(want1))


def test_residuals_bitwise(golden):
    g = golden("ukf_ref.npz")
    with np.errstate(invalid="ignore"):
        rx = np.stack([oukf.residual_x(a.copy(), b.copy()) for a, b in zip(g["resx_a"], g["resx_b"])])
        rh = np.stack([oukf.residual_h(a.copy(), b.copy()) for a, b in zip(g["resh_a"], g["resh_b"])])
    assert np.array_equal(_bits(rx), _bits(g["resx_out"]))
    assert np.array_equal(_bits(rh), _bits(g["resh_out"]))


def _exact_hx(x, lm):
    with mp.workdps(ux.DPS):
        return np.array([float(v) for v in ux.hx([mp.mpf(float(t)) for t in x],
                                                 [(mp.mpf(float(px)), mp.mpf(float(py))) for px, py in lm])])


@pytest.mark.parametrize("case", ["c3", "c5", "edge"])
def test_exact_evaluator_within_rounding(golden, case):
    g = golden("ukf_ref.npz")
    x, lm, hx = g[case + "_x"], g[case + "_lmk"], g[case + "_hx"]
    keep = np.abs(x[:, 2]) <= 1e4
    assert keep.sum() >= len(x) - 8
    for s in np.nonzero(keep)[0][:16]:
        ex = _exact_hx(x[s], lm[s])
        d = np.abs(ex[0::2] - hx[s, 0::2]) / np.abs(hx[s, 0::2])
        b = np.abs(ex[1::2] - hx[s, 1::2])
        b = np.minimum(b, 2 * np.pi - b)   # the two wraps may land on either side of +-pi
        tol_b = 4 * np.spacing(max(np.pi, abs(float(x[s, 2]))))
        assert d.max() <= DIST_REL and b.max() <= tol_b, (case, s, d.max(), b.max())
