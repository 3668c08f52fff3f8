"""The HIP UKF (U1-U8, lslam_ukf.h) against the 50-digit evaluation of the same
algorithm (tests/golden/ukf_exact.npz, oracle/ukf_exact.py), per component, at
north_star's 1e-5: x and y relative, theta absolute, P relative to max|P|.
PARITY UNPINNED for the algorithm itself (see tests/test_ukf_exact.py)."""
import numpy as np
import pytest

from oracle import ukf_exact as ux

pytestmark = pytest.mark.gpu

TOL = {"x_rel": 1e-5, "y_rel": 1e-5, "theta_abs": 1e-5, "P_rel": 1e-5}


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def case(golden, name):
    g = golden("ukf_exact.npz")
    return {k[len(name) + 1:]: v for k, v in g.items() if k.startswith(name + "_")}


def _ukf_only(ctx, c):
    from lidar_slam_amd.pipeline import ScanPipeline
    S, L = c["x"].shape[0], c["lmk"].shape[1]
    p = ScanPipeline(ctx, np.zeros((1, 2)), np.zeros(S + 1, np.int32), np.zeros(1, np.int32),
                     ukf=dict(n_landmarks=L, x=c["x"], P=c["P"], u=c["u"], z=c["z"], lmk=c["lmk"],
                              R_diag=c["R_diag"], flags=int(c["flags"])))
    p.run_ukf_only()
    r = p.results()
    return r["ukf_x"], r["ukf_P"]


@pytest.mark.parametrize("name", ["c3", "c5", "bench", "map", "predict"])
def test_hip_ukf_rounding_per_component(ctx, golden, name):
    c = case(golden, name)
    x, P = _ukf_only(ctx, c)
    err = ux.component_errors(x, P, c["x_exact"], c["P_exact"])
    for k, tol in TOL.items():
        assert err[k] <= tol, (name, err)


def test_fused_pipeline_ukf_on_the_bench_workload(ctx, golden):
    """The UKF inside the fused C3 pipeline call (post pass after RANSAC + association) on
    the bench's own scans and UKF inputs."""
    import bench
    from lidar_slam_amd.pipeline import ScanPipeline
    c = case(golden, "bench")
    ids = list(range(8))
    b, wk = bench.make_workload(ids, 720, 20)
    assert np.array_equal(wk["z"], c["z"]) and np.array_equal(wk["x"], c["x"])
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                     lmk_capacity=64, ukf=wk)
    p.run()
    r = p.results()
    err = ux.component_errors(r["ukf_x"], r["ukf_P"], c["x_exact"], c["P_exact"])
    for k, tol in TOL.items():
        assert err[k] <= tol, err
