"""bench.py's C4 leg (BASELINE configs[3]) at world size 1 on a reduced shared batch.

The leg is the replacement for the reference's hand-off of scans through one
``multiprocessing.Queue`` (/root/reference/SLAM.py:13,18-23): one host batch in node shared
memory, page-locked, the rank's shard uploaded, the fused pipeline, the RCCL gather of the
per-scan results to rank 0's HBM and the copy to its host.  Here one rank runs the whole path
(a one-rank communicator: the gather is its device copy) and the gathered arrays must equal a
direct ScanPipeline call on the same inputs byte for byte, and the oracle on a sample."""
import types

import numpy as np
import pytest

pytestmark = pytest.mark.gpu

SCANS = 8192     # one C4 shard's size (65,536 / 8)
L = 20


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


@pytest.fixture(scope="module")
def leg(ctx):
    import bench
    args = types.SimpleNamespace(c4_scans=SCANS, beams=720, trials=100, lmk_capacity=64, c4_steps=2, warmup=1,
                                c4_transport="rccl")
    keep = {}
    res = bench.run_guarded(lambda segs: bench.c4_leg(args, 0, 1, None, ctx, L, segs, keep=keep), 120, 0, {})
    return res, keep


def test_leg_runs_consistent(leg):
    res, keep = leg
    assert "error" not in res, res
    assert res["consistent"] is True
    assert res["capacity_overflows"] == 0
    assert res["total_scans"] == SCANS
    assert res["host_batch"].endswith("page-locked")
    assert set(keep) == {"mask", "models", "ukf_x", "ukf_P", "lmk_count"}


def test_gathered_equals_direct_pipeline(ctx, leg):
    import bench
    from lidar_slam_amd.pipeline import ScanPipeline
    _, keep = leg
    ids = list(range(SCANS))
    b, wk = bench.make_workload(ids, 720, L, seed_base=1000)   # rank 0's shard generator in the leg
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                     max_trials=100, lmk_capacity=64, want_yproj=False, ukf=wk)
    p.run()
    r = p.results()
    for k in ("mask", "models", "ukf_x", "ukf_P", "lmk_count"):
        assert np.ascontiguousarray(keep[k]).tobytes() == np.ascontiguousarray(r[k]).tobytes(), k


def test_gathered_sample_vs_oracle(leg):
    import bench
    from lidar_slam_amd import synth
    from oracle import cpu as orc
    from oracle import ukf as oukf
    _, keep = leg
    sample = [0, 1, 4095, 4096, SCANS - 1]
    sb = synth.make_batch(sample)
    mask, _, models, _ = orc.run_batch(sb["xy"], sb["scan_chunk_off"], sb["chunk_pt_off"], sample)
    nch = int(np.diff(sb["scan_chunk_off"])[0])
    npt = int(sb["chunk_pt_off"][nch])
    got_mask = np.concatenate([keep["mask"][s * npt:(s + 1) * npt] for s in sample])
    assert np.array_equal(got_mask, mask)
    got = np.concatenate([keep["models"][s * nch:(s + 1) * nch] for s in sample])
    assert np.array_equal(got["n_inliers"], np.array([m["n_inliers"] for m in models]))
    assert np.array_equal(got["best_trial"], np.array([m["best_trial"] for m in models]))
    assert np.allclose(got["a"], np.array([m["a"] for m in models]), rtol=1e-9, atol=0)
    # the UKF rows of the sample against the NumPy restatement (U1-U8, 1e-5 as elsewhere)
    _, wk = bench.make_workload(list(range(SCANS)), 720, L, seed_base=1000)
    idx = np.array(sample)
    xo, Po = oukf.ukf_batch(wk["x"][idx], wk["P"][idx], wk["u"][idx], wk["z"][idx], wk["lmk"][idx], wk["R_diag"])
    assert np.allclose(keep["ukf_x"][idx], xo, rtol=1e-5, atol=1e-5)
    assert np.allclose(keep["ukf_P"][idx], Po, rtol=1e-5, atol=1e-9)
