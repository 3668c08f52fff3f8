"""Generate tests/golden/ukf_exact.npz: UKF steps evaluated in 50-digit arithmetic.

    python tests/golden/make_ukf_exact.py

PARITY UNPINNED (the reference UKF does not parse, filterpy is absent): these
vectors pin the rounding of the float64 implementations, not the algorithm.
Each case is a batch of filters with its inputs (x, P, u, z, landmark
positions, R diagonal) and the exact step's (x, P) rounded once to float64
(oracle/ukf_exact.py).  Cases:
  c3       48 filters, L = 20 (C3's dim_z = 40), P0 = diag(.1, .1, .05), R = [.25, .09]
           (systemClass.py:8-9,27-28), headings uniform plus 8 within 1e-6 of +-pi
  c5       4 filters, L = 200 (C5's dim_z = 400)
  bench    8 filters exactly as bench.py's make_workload feeds the timed C3 step
  map      8 filters, L = 8, the landmark-map tuning P0 = diag(25, 25, 1e-4), R = [25, 1e-4]
  predict  8 filters, predict only (flags = LSLAM_UKF_PREDICT)
"""
import os
import sys
import time

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import blaspin  # noqa: E402  (pins OPENBLAS_CORETYPE; must precede numpy)
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("LSLAM_GOLDEN_OUT", HERE)  # the dispatch census writes elsewhere
ROOT = os.path.abspath(os.path.join(HERE, "..", ".."))
sys.path.insert(0, ROOT)

from oracle import ukf as oukf  # noqa: E402
from oracle import ukf_exact as ux  # noqa: E402


def _filters(rng, S, L, noise=0.3, headings=None):
    x = np.stack([rng.uniform(800, 3200, S), rng.uniform(800, 2200, S), rng.uniform(-np.pi, np.pi, S)], 1)
    if headings is not None:
        x[:len(headings), 2] = headings
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)]) + rng.normal(0, noise, (S, 2 * L))
    return x, lmk, z


def case(name, x, P, u, z, lmk, Rd, predict=True, update=True):
    t = time.time()
    xe, Pe = ux.ukf_batch_exact(x, P, u, z, lmk, Rd, predict=predict, update=update)
    print("%-8s %3d filters, L=%3d: %.1fs" % (name, len(x), lmk.shape[1], time.time() - t), flush=True)
    flags = (1 if predict else 0) | (2 if update else 0)
    return {name + "_" + k: v for k, v in dict(x=x, P=P, u=u, z=z, lmk=lmk, R_diag=Rd, x_exact=xe, P_exact=Pe,
                                               flags=np.int32(flags)).items()}


def main():
    out = {}
    rng = np.random.default_rng(20261016)
    # c3
    S, L = 48, 20
    heads = [np.pi - 1e-6, -np.pi + 1e-6, np.pi - 1e-9, -np.pi + 1e-9, np.pi, 3.0, -3.0, 1e-7]
    x, lmk, z = _filters(rng, S, L, headings=heads)
    P0 = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    u = np.tile([2.0, 2.5], (S, 1))
    Rd = np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)
    out.update(case("c3", x, P0, u, z, lmk, Rd))
    # c5
    S, L = 4, 200
    x, lmk, z = _filters(rng, S, L)
    out.update(case("c5", x, np.tile(np.diag([.1, .1, .05]), (S, 1, 1)), np.tile([2.0, 2.5], (S, 1)), z, lmk,
                    np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)))
    # bench (the timed step's inputs: bench.make_workload, scans 0..7)
    import bench
    _, wk = bench.make_workload(list(range(8)), 720, 20)
    out.update(case("bench", wk["x"], wk["P"], wk["u"], wk["z"], wk["lmk"], wk["R_diag"]))
    # map tuning
    S, L = 8, 8
    x, lmk, z = _filters(rng, S, L, noise=1.0)
    out.update(case("map", x, np.tile(np.diag([25.0, 25.0, 1e-4]), (S, 1, 1)), np.tile([2.0, 2.5], (S, 1)), z, lmk,
                    np.array([25.0, 1e-4] * L)))
    # predict only
    S, L = 8, 20
    x, lmk, z = _filters(rng, S, L)
    out.update(case("predict", x, np.tile(np.diag([.1, .1, .05]), (S, 1, 1)), np.tile([2.0, 2.5], (S, 1)), z, lmk,
                    np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L), update=False))
    blaspin.save_npz(os.path.join(OUT, "ukf_exact.npz"), **out)
    print("ukf_exact.npz", os.path.getsize(os.path.join(OUT, "ukf_exact.npz")), "bytes")


if __name__ == "__main__":
    main()
