"""An understated ``max_scan_chunks`` (include/lidarslam.h lslam_scan_batch) through the C ABI.

``max_scan_chunks`` sizes the post pass's LDS staging of a scan's chunk records.  A scan with
more chunks than the batch declares must still get the reference's per-chunk semantics
(``check_ransac`` calling ``landmark_extraction`` once per chunk, ransac_functions.py:34-54,
63-93): its chunk records are walked in place instead of staged, and the fix-up's early-stop
rewind restores a snapshot of the stream taken at the chunk's start instead of replaying a
per-chunk history of max_scan_chunks entries.  So an understated call must be bit-identical to
the correct one, for every scan, in every output.

The batch: 24 synthetic scans in which scans 5 and 6 are merged into one scan of 16 chunks,
whose chunk 12 is collinear (y == 0 exactly: the first trial's residual sum is 0, so skimage's
ransac stops after one trial, fit.py:862-869, and the fix-up replays the scan).
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


def _batch():
    from lidar_slam_amd import synth
    ids = list(range(24))
    b = synth.make_batch(ids)
    xy = b["xy"].copy()
    sco = np.delete(b["scan_chunk_off"], 6)  # scans 5 and 6 -> one scan of 16 chunks
    cpo = b["chunk_pt_off"]
    c = sco[5] + 12
    p0, p1 = cpo[c], cpo[c + 1]
    xy[p0:p1, 0] = 50.0 * np.arange(p1 - p0)
    xy[p0:p1, 1] = 0.0
    seeds = np.array([s for s in ids if s != 6], np.int64)
    return xy, sco, cpo, seeds


def _run(ctx, xy, sco, cpo, seeds, msc, cap, ukf):
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import ukf as oukf
    S = len(sco) - 1
    kw = {}
    if ukf:
        L = 20
        rng = np.random.default_rng(3)
        lmk = rng.uniform(-3000, 3000, (S, L, 2))
        x = np.tile([100.0, 200.0, 0.3], (S, 1))
        z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)])
        kw["ukf"] = dict(n_landmarks=L, x=x, P=np.tile(np.diag([.1, .1, .05]), (S, 1, 1)),
                         u=np.tile([2.0, 2.5], (S, 1)), z=z, lmk=lmk,
                         R_diag=np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L), flags=7)
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=seeds, lmk_capacity=cap, want_state=True, want_draws=True, **kw)
    assert p.batch.max_scan_chunks == 16
    p.batch.max_scan_chunks = msc
    p.run()
    return p.results()


@pytest.mark.parametrize("cap,ukf", [(32, False), (80, False), (32, True)])
def test_understated_max_scan_chunks_is_bit_identical(cap, ukf):
    """cap 32: the association keeps the list in registers (post_assoc_reg); cap 80: the LDS
    list (per-chunk loop); ukf: + the lane-group UKF fed by the chunk origins (LMK_FROM_RANSAC)."""
    from lidar_slam_amd.device import Context
    ctx = Context(0)
    xy, sco, cpo, seeds = _batch()
    good = _run(ctx, xy, sco, cpo, seeds, 16, cap, ukf)
    low = _run(ctx, xy, sco, cpo, seeds, 8, cap, ukf)
    assert good["models"]["flags"][sco[5] + 12] & 16  # the early stop is there (LSLAM_EARLY_STOP)
    for k in good:
        if good[k].dtype.names:
            for f in good[k].dtype.names:
                assert np.array_equal(good[k][f], low[k][f], equal_nan=True), (k, f)
        else:
            assert np.array_equal(good[k], low[k], equal_nan=True), k
    assert not np.any(low["models"]["flags"] & 512)  # LSLAM_CHUNK_BOUND: only map mode sets it


def test_understated_max_scan_chunks_vs_oracle():
    """The merged scan's masks, line parameters, projected y and MT end state against the
    oracle's sequential restatement (oracle/cpu.py, pinned to the reference's fixtures)."""
    from lidar_slam_amd.device import Context
    from oracle import cpu as orc
    ctx = Context(0)
    xy, sco, cpo, seeds = _batch()
    low = _run(ctx, xy, sco, cpo, seeds, 8, 32, False)
    mask, yproj, models, _ = orc.run_batch(xy, sco, cpo, seeds)
    assert np.array_equal(low["mask"], mask)
    a = np.array([m["a"] for m in models])
    assert np.array_equal(low["models"]["a"], a, equal_nan=True)
    np.testing.assert_allclose(low["y_proj"], yproj, rtol=1e-9, atol=1e-9)
