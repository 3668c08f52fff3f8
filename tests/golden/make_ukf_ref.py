"""Generate tests/golden/ukf_ref.npz: the reference's OWN UKF measurement and residual
functions run on this build's test inputs.

    /opt/conda/bin/python3.9 tests/golden/make_ukf_ref.py

``/root/reference/UKFMethods.py`` does not parse as a whole (``state_mean`` /
``z_mean`` at :37-57 are SyntaxErrors) and imports the absent filterpy (:3-4),
but four of its functions need only numpy and math and run as written:

    normalize_angle     UKFMethods.py:10-14
    transfer_function   UKFMethods.py:26-34   (hx: [dist, wrap(atan2 - theta)] per landmark)
    residual_x          UKFMethods.py:60-63
    residual_h          UKFMethods.py:66-71

The module's text is split into its top-level statements; each is parsed on its own
(``ast``), and only these four ``def``s, the ``import numpy as np`` / ``from math
import ...`` lines and the module constants (:6-8) are compiled and executed, in file
order.  The filterpy imports and the two unparseable functions are left out.  Nothing of
the reference's text is stored: the archive holds inputs and outputs only, plus the
sha256 and line span of each statement that ran (``meta_blocks``).

Landmarks are stand-ins for reference ``landmarking.Landmark`` objects holding what
``transfer_function`` reads: ``get_pos()``, the ``np.array([x, y])`` of landmarking.py:17, :36-37
(the reference module itself is not imported: only the ast-selected functions above run).  Poses are numpy float64 rows, as filterpy
passes sigma points, so the angle arithmetic runs on np.float64 as it would in the UKF.

Cases (S filters x L landmarks, inputs made with numpy's default_rng here):
  c3     48 x 20: uniform poses plus 8 headings within 1e-9..1e-6 of +-pi
  c5     4 x 200
  edge   one filter per edge angle a (heading -a): landmark 0 dead ahead (atan2 = +0,
         so bearing 0 = normalize_angle(a)), landmark 1 dead behind (atan2 = pi),
         landmarks 2.. uniform; a in {+-0, +-pi, pi +- 1 ulp, 2pi, 3pi, 4pi +- 1 ulp,
         +-pi +- 1e-9, tiny and huge magnitudes, ...}
  norm   normalize_angle on the edge list, random |a| <= 20 and |a| <= 1e4, inf / nan,
         called with Python floats and with np.float64 (the two must agree)
  resx   residual_x(a, b) on 3-vectors whose angle differences hit the edges
  resh   residual_h(a, b) on 40-vectors, likewise
Each hx case also carries the update-only UKF inputs the GPU trace test runs
(P = diag(.1, .1, .05), R = [.25, .09] per landmark, z = hx + noise).
"""
import ast
import hashlib
import os
import sys

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import blaspin  # noqa: E402  (pins OPENBLAS_CORETYPE; must precede numpy)
import numpy as np  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("LSLAM_GOLDEN_OUT", HERE)
sys.path.insert(0, REF)


WANT_DEFS = ("normalize_angle", "transfer_function", "residual_x", "residual_h")
WANT_CONSTS = ("R", "L", "dt")


def _top_level_blocks(text):
    """(first_line, last_line, source) of each top-level statement: a block starts at a
    non-blank, non-comment line with no indentation and runs until the next one."""
    lines = text.splitlines(keepends=True)
    starts = [i for i, ln in enumerate(lines) if ln.strip() and not ln[0].isspace() and not ln.startswith("#")]
    out = []
    for n, i in enumerate(starts):
        j = starts[n + 1] if n + 1 < len(starts) else len(lines)
        out.append((i + 1, j, "".join(lines[i:j])))
    return out


def load_reference_functions(path=os.path.join(REF, "UKFMethods.py")):
    with open(path) as f:
        text = f.read()
    ns, ran = {}, []
    for first, last, src in _top_level_blocks(text):
        try:
            mod = ast.parse(src)
        except SyntaxError:
            continue  # state_mean / z_mean (UKFMethods.py:37-57)
        keep = []
        for node in mod.body:
            if isinstance(node, ast.FunctionDef) and node.name in WANT_DEFS:
                keep.append(node)
            elif isinstance(node, ast.Import) and all(a.name == "numpy" for a in node.names):
                keep.append(node)
            elif isinstance(node, ast.ImportFrom) and node.module == "math":
                keep.append(node)
            elif (isinstance(node, ast.Assign) and len(node.targets) == 1 and isinstance(node.targets[0], ast.Name)
                  and node.targets[0].id in WANT_CONSTS):
                keep.append(node)
        if not keep:
            continue
        exec(compile(ast.Module(body=keep, type_ignores=[]), path, "exec"), ns)
        ran.append("%d-%d %s" % (first, last, hashlib.sha256(src.encode()).hexdigest()[:16]))
    missing = [n for n in WANT_DEFS if n not in ns]
    assert not missing, missing
    return ns, ran


class _Landmark:
    """What transfer_function reads of a reference landmarking.Landmark: get_pos(), the
    np.array([x, y]) the constructor stores (landmarking.py:17, :36-37).  A local stand-in, so
    that no reference module runs beyond the ast-selected UKFMethods.py functions."""

    def __init__(self, x, y):
        self.pos = np.array([x, y])

    def get_pos(self):
        return self.pos


def _landmarks(pts):
    return [_Landmark(float(px), float(py)) for px, py in pts]


def edge_angles():
    pi, tp = np.pi, 2 * np.pi
    up, dn = (lambda v: np.nextafter(v, np.inf)), (lambda v: np.nextafter(v, -np.inf))
    a = [0.0, -0.0, pi, -pi, up(pi), dn(pi), up(-pi), dn(-pi), tp, -tp, up(tp), dn(tp), -up(tp), -dn(tp),
         3 * pi, -3 * pi, 2 * tp, -2 * tp, up(2 * tp), dn(2 * tp), -up(2 * tp), -dn(2 * tp), 5 * pi, -5 * pi,
         pi + 1e-9, pi - 1e-9, -pi + 1e-9, -pi - 1e-9, pi / 2, -pi / 2, 1e-300, -1e-300, 5e-324, -5e-324,
         1e-9, -1e-9, 1e6, -1e6, 1e15, -1e15, 1e300, -1e300, 7.0, -7.0, 12.566370614359172, -12.566370614359172]
    return np.array(a, np.float64)


def hx_case(ns, rng, name, x, lmk, noise=0.3):
    S, L = lmk.shape[:2]
    hx = np.stack([ns["transfer_function"](np.array(x[s], np.float64), _landmarks(lmk[s])) for s in range(S)])
    assert hx.dtype == np.float64 and hx.shape == (S, 2 * L)
    z = hx + rng.normal(0, noise, (S, 2 * L))
    P = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    Rd = np.array([0.5 ** 2, 0.3 ** 2] * L)
    return {name + "_x": x, name + "_lmk": lmk, name + "_hx": hx, name + "_z": z, name + "_P": P, name + "_R_diag": Rd}


def _poses(rng, S):
    return np.stack([rng.uniform(800, 3200, S), rng.uniform(800, 2200, S), rng.uniform(-np.pi, np.pi, S)], 1)


def main():
    ns, ran = load_reference_functions()
    rng = np.random.default_rng(20261017)
    out = {}
    # c3: L = 20, headings near +-pi included
    x = _poses(rng, 48)
    x[:8, 2] = [np.pi - 1e-6, -np.pi + 1e-6, np.pi - 1e-9, -np.pi + 1e-9, np.pi, -np.pi, 3.0, -3.0]
    out.update(hx_case(ns, rng, "c3", x, rng.uniform(-3000, 3000, (48, 20, 2))))
    # c5: L = 200
    out.update(hx_case(ns, rng, "c5", _poses(rng, 4), rng.uniform(-3000, 3000, (4, 200, 2))))
    # edge: heading -a, landmark 0 dead ahead (atan2(+0, +) = +0), landmark 1 dead behind (atan2(+0, -) = pi)
    ea = edge_angles()
    S = len(ea)
    x = _poses(rng, S)
    x[:, 2] = -ea
    lm = rng.uniform(-3000, 3000, (S, 20, 2))
    lm[:, 0, 0], lm[:, 0, 1] = x[:, 0] + 1000.0, x[:, 1]
    lm[:, 1, 0], lm[:, 1, 1] = x[:, 0] - 1000.0, x[:, 1]
    out.update(hx_case(ns, rng, "edge", x, lm))
    out["edge_angles"] = ea
    # normalize_angle on Python floats and on np.float64
    na = np.concatenate([ea, rng.uniform(-20, 20, 1000), rng.uniform(-1e4, 1e4, 1000), [np.inf, -np.inf, np.nan]])
    with np.errstate(invalid="ignore"):
        nf = np.array([ns["normalize_angle"](float(v)) for v in na], np.float64)
        nn = np.array([ns["normalize_angle"](np.float64(v)) for v in na], np.float64)
    assert np.array_equal(nf, nn, equal_nan=True)
    out["norm_in"], out["norm_out"] = na, nf
    # residual_x / residual_h: angle differences on the edges, the rest random
    n = len(ea)
    b3 = _poses(rng, n)
    a3 = b3 + rng.normal(0, 5, (n, 3))
    a3[:, 2] = b3[:, 2] + ea
    a3 = np.concatenate([a3, _poses(rng, 200)])
    b3 = np.concatenate([b3, _poses(rng, 200)])
    with np.errstate(invalid="ignore"):
        rx = np.stack([ns["residual_x"](a3[i].copy(), b3[i].copy()) for i in range(len(a3))])
    out["resx_a"], out["resx_b"], out["resx_out"] = a3, b3, rx
    m = 40
    ah = rng.uniform(-4, 4, (64, m))
    bh = rng.uniform(-4, 4, (64, m))
    ah[:, 0::2] *= 1000.0
    bh[:, 0::2] *= 1000.0
    k = np.arange(64 * (m // 2)) % n
    ah.reshape(-1, 2)[:, 1] = bh.reshape(-1, 2)[:, 1] + ea[k]
    with np.errstate(invalid="ignore"):
        rh = np.stack([ns["residual_h"](ah[i].copy(), bh[i].copy()) for i in range(len(ah))])
    out["resh_a"], out["resh_b"], out["resh_out"] = ah, bh, rh
    out["meta_blocks"] = np.array(ran)
    blaspin.save_npz(os.path.join(OUT, "ukf_ref.npz"), **out)
    print("ukf_ref.npz", os.path.getsize(os.path.join(OUT, "ukf_ref.npz")), "bytes; ran UKFMethods.py blocks:", ran)


if __name__ == "__main__":
    main()
