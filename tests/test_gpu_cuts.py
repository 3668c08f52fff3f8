"""The consensus's box terms, cutoffs and owning scan computed ahead (cut_lane_kernel, launched with
seed_kernel on the seeding stream in a fresh-stream pipeline call) against the consensus computing
them itself (explicit draws: no seeding, so no cut kernel): the same draws through both paths must
give byte-identical masks, chunk records and trial counts.  The batches are ragged (chunk sizes
1..128, scans of 0..9 chunks), so the cut kernel's owning-scan search leaves its proportional
guess, and one batch is polar (points converted on load in both kernels).  Repeated calls on one
pipeline cycle the four-buffer cut ring."""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def _ragged(rng, S):
    per = rng.integers(0, 10, S)
    per[0] = max(per[0], 1)
    sco = np.concatenate([[0], np.cumsum(per)]).astype(np.int32)
    C = int(sco[-1])
    sizes = rng.integers(1, 129, C)
    sizes[rng.random(C) < 0.6] = 100  # mostly C3-sized chunks, ragged around them
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    return sco, cpo


def _walls(rng, cpo):
    """Per chunk: a noisy segment of a line plus a few outliers (mm)."""
    P = int(cpo[-1])
    xy = np.empty((P, 2))
    for c in range(len(cpo) - 1):
        p0, p1 = cpo[c], cpo[c + 1]
        n = p1 - p0
        ang = rng.uniform(0, np.pi)
        t = np.linspace(-1500, 1500, n)
        o = rng.uniform(-4000, 4000, 2)
        pts = o + np.outer(t, [np.cos(ang), np.sin(ang)]) + rng.normal(0, 8, (n, 2))
        k = rng.random(n) < 0.15
        pts[k] += rng.normal(0, 600, (int(k.sum()), 2))
        xy[p0:p1] = pts
    return xy


def _fields(r):
    m = r["models"]
    return r["mask"].tobytes(), m.tobytes(), r["counts"].tobytes()


@pytest.mark.parametrize("polar", [False, True])
def test_precomputed_cuts_equal_in_kernel(ctx, polar):
    from lidar_slam_amd import pipeline as pl
    rng = np.random.default_rng(7 + polar)
    S = 600
    sco, cpo = _ragged(rng, S)
    xy = _walls(rng, cpo)
    kw = dict(max_trials=100, want_counts=True, want_yproj=False)
    if polar:
        th = np.degrees(np.arctan2(xy[:, 1], xy[:, 0]))
        dd = np.hypot(xy[:, 0], xy[:, 1])
        pts = dict(xy=None, theta_deg=th, dist_mm=dd)
    else:
        pts = dict(xy=xy)
    seeds = rng.integers(0, 2**32, S, dtype=np.uint64).astype(np.uint32)
    mt = pl.ScanPipeline(ctx, scan_chunk_off=sco, chunk_pt_off=cpo, seeds=seeds, want_draws=True, **pts, **kw)
    runs = []
    for _ in range(6):  # the cut ring has four buffers: wrap it
        mt.run(sync=False)
        ctx.sync()
        runs.append(mt.results())
    a = runs[0]
    for r in runs[1:]:
        assert _fields(r) == _fields(a)
    ex = pl.ScanPipeline(ctx, scan_chunk_off=sco, chunk_pt_off=cpo, hyp="explicit", hyp_draws=a["draws"], **pts, **kw)
    ex.run()
    b = ex.results()
    assert a["mask"].tobytes() == b["mask"].tobytes()
    assert a["counts"].tobytes() == b["counts"].tobytes()
    am, bm = a["models"], b["models"]
    for f in am.dtype.names:
        assert am[f].tobytes() == bm[f].tobytes(), f
