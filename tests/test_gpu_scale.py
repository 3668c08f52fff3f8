"""GPU checks at BASELINE.json's full sizes through size-independent
properties, plus a bit-exact oracle comparison on a sample of the batch.

C3: 4096 x 720-pt scans (RANSAC + association + UKF, L=20)
C4 shard: 8192 scans (one GPU's share of 65,536)
C5: 4096-pt scans, 2048 hypotheses, UKF with L=200 (sampled)
"""
import numpy as np
import pytest

pytestmark = pytest.mark.gpu


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def _run(ctx, b, ids, ukf=None, **kw):
    from lidar_slam_amd.pipeline import ScanPipeline
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                     lmk_capacity=32, ukf=ukf, want_state=True, **kw)
    p.run()
    return p.results()


def test_c3_full_batch_properties(ctx):
    import bench
    from oracle import cpu as orc
    ids = list(range(4096))
    b, ukf = bench.make_workload(ids, 720, 20)
    r1 = _run(ctx, b, ids, ukf)
    r2 = _run(ctx, b, ids, ukf)
    # determinism
    for k in ("mask", "y_proj", "mt_state", "landmarks", "lmk_count", "ukf_x", "ukf_P"):
        assert np.array_equal(r1[k], r2[k]), k
    assert r1["models"].tobytes() == r2["models"].tobytes()
    m = r1["models"]
    cpo = b["chunk_pt_off"]
    # every chunk fitted; mask popcount == n_inliers; draws = T+1 (no exact-collinear chunk)
    assert np.all(m["flags"] & 1)
    pop = np.add.reduceat(r1["mask"].astype(np.int64), cpo[:-1])
    assert np.array_equal(pop, m["n_inliers"])
    assert np.all(m["n_draws"] == 101)
    assert np.all(np.isfinite(r1["ukf_x"])) and np.all(np.isfinite(r1["ukf_P"]))
    # shard invariance: two halves == the whole
    for lo, hi in ((0, 2048), (2048, 4096)):
        sub = list(range(lo, hi))
        c0, c1 = b["scan_chunk_off"][lo], b["scan_chunk_off"][hi]
        bb = {"xy": b["xy"][cpo[c0]:cpo[c1]], "scan_chunk_off": b["scan_chunk_off"][lo:hi + 1] - c0,
              "chunk_pt_off": cpo[c0:c1 + 1] - cpo[c0]}
        uk = {k: (v[lo:hi] if isinstance(v, np.ndarray) and v.shape[:1] == (4096,) else v) for k, v in ukf.items()}
        rs = _run(ctx, bb, sub, uk)
        assert np.array_equal(rs["mask"], r1["mask"][cpo[c0]:cpo[c1]])
        assert rs["models"].tobytes() == r1["models"][c0:c1].tobytes()
        assert np.array_equal(rs["ukf_x"], r1["ukf_x"][lo:hi])
    # bit-exact against the oracle on a random sample of scans
    rng = np.random.default_rng(0)
    for s in rng.choice(4096, 24, replace=False):
        c0, c1 = b["scan_chunk_off"][s], b["scan_chunk_off"][s + 1]
        xy = b["xy"][cpo[c0]:cpo[c1]]
        mask, yproj, models, lists = orc.run_batch(xy, np.array([0, c1 - c0]), cpo[c0:c1 + 1] - cpo[c0], [s])
        assert np.array_equal(mask, r1["mask"][cpo[c0]:cpo[c1]]), s
        assert np.array_equal(np.array([d["a"] for d in models]), m["a"][c0:c1]), s
        assert [L["id"] for L in lists[0]] == list(r1["landmarks"][s, :r1["lmk_count"][s]]["id"]), s


def test_c2_full_batch_ransac_only(ctx):
    """C2: 4096 x 720-pt scans through the RANSAC-only entry point (lslam_ransac, the
    ransac_functions.py:23-31 leg: skimage ransac + a, b, tip per chunk).  Masks, every RANSAC
    field of the chunk records and the MT streams equal the fused C3 run's; bit-exact against
    the oracle on a sample of scans."""
    import bench
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import cpu as orc
    ids = list(range(4096))
    b, ukf = bench.make_workload(ids, 720, 20)
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                     want_state=True)
    p.run_ransac_only()
    r2 = p.results()
    r3 = _run(ctx, b, ids, ukf)
    m2, m3 = r2["models"], r3["models"]
    assert np.array_equal(r2["mask"], r3["mask"])
    assert np.array_equal(r2["mt_state"], r3["mt_state"])
    for f in ("ox", "oy", "ux", "uy", "a", "b", "tip_x", "tip_y", "n_inliers", "best_trial", "n_draws",
              "landmark_id", "n_points"):
        assert np.array_equal(m2[f], m3[f]), f
    assert np.array_equal(m2["flags"] & 63, m3["flags"] & 63)       # the RANSAC flags (no association bits)
    assert np.all(m2["flags"] & 1) and not np.any(m2["flags"] & (64 | 128))
    cpo, sco = b["chunk_pt_off"], b["scan_chunk_off"]
    pop = np.add.reduceat(r2["mask"].astype(np.int64), cpo[:-1])
    assert np.array_equal(pop, m2["n_inliers"])
    # y_proj on the chunk's own line (no association pass)
    sel = r2["mask"].astype(bool)
    c_of_pt = np.repeat(np.arange(len(cpo) - 1), np.diff(cpo))
    assert np.array_equal(r2["y_proj"][sel], m2["a"][c_of_pt[sel]] * b["xy"][sel, 0] + m2["b"][c_of_pt[sel]])
    assert not np.any(r2["y_proj"][~sel])
    for s in np.random.default_rng(2).choice(4096, 32, replace=False):
        st = orc.MTState(seed=int(s))
        for c in range(sco[s], sco[s + 1]):
            mo, md, _ = orc.ransac(b["xy"][cpo[c]:cpo[c + 1]], 20.0, 100, state=st)
            assert np.array_equal(r2["mask"][cpo[c]:cpo[c + 1]], mo), (s, c)
            for f in ("best_trial", "n_draws", "flags", "n_inliers", "ox", "oy", "ux", "uy", "a", "b"):
                assert m2[f][c] == md[f], (s, c, f)
        assert np.array_equal(r2["mt_state"][s, :624], st.key) and r2["mt_state"][s, 624] == st.pos.value, s


def test_c4_shard_8192(ctx):
    """Rank 1's shard of C4 (65,536 scans over 8 GPUs, `bench.py --gpus 8 --scans 8192`) equals
    the same scans run as two 4096-scan launches (ranks 2 and 3 of the default bench), and the
    oracle on a sample."""
    import bench
    from oracle import cpu as orc
    ids = list(range(8192, 16384))
    b, ukf = bench.make_workload(ids, 720, 20, seed_base=1)
    r = _run(ctx, b, ids, ukf)
    m = r["models"]
    cpo = b["chunk_pt_off"]
    assert np.all(m["flags"] & 1)
    pop = np.add.reduceat(r["mask"].astype(np.int64), cpo[:-1])
    assert np.array_equal(pop, m["n_inliers"])
    for lo, hi in ((0, 4096), (4096, 8192)):
        c0, c1 = b["scan_chunk_off"][lo], b["scan_chunk_off"][hi]
        bb = {"xy": b["xy"][cpo[c0]:cpo[c1]], "scan_chunk_off": b["scan_chunk_off"][lo:hi + 1] - c0,
              "chunk_pt_off": cpo[c0:c1 + 1] - cpo[c0]}
        uk = {k: (v[lo:hi] if isinstance(v, np.ndarray) and v.shape[:1] == (8192,) else v) for k, v in ukf.items()}
        rs = _run(ctx, bb, ids[lo:hi], uk)
        assert np.array_equal(rs["mask"], r["mask"][cpo[c0]:cpo[c1]])
        assert rs["models"].tobytes() == m[c0:c1].tobytes()
        for k in ("mt_state", "landmarks", "lmk_count", "ukf_x", "ukf_P"):
            assert np.array_equal(rs[k], r[k][lo:hi]), k
    for i in np.random.default_rng(4).choice(8192, 8, replace=False):
        c0, c1 = b["scan_chunk_off"][i], b["scan_chunk_off"][i + 1]
        mask, _, models, lists = orc.run_batch(b["xy"][cpo[c0]:cpo[c1]], np.array([0, c1 - c0]),
                                               cpo[c0:c1 + 1] - cpo[c0], [ids[i]])
        assert np.array_equal(mask, r["mask"][cpo[c0]:cpo[c1]]), i
        assert [L["id"] for L in lists[0]] == list(r["landmarks"][i, :r["lmk_count"][i]]["id"]), i


def test_c5_dense_scans_and_l200_ukf(ctx):
    """4096-point scans as ONE chunk each, 2048 hypotheses, UKF with L=200."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import cpu as orc
    from oracle import ukf as oukf
    from oracle import ukf_exact
    S, Np, L = 6, 4096, 200
    xys = [synth.polar_to_xy_ref(*synth.scan_polar(9000 + s, n_beams=Np, cfg=5)[:2]) for s in range(S)]
    xy = np.concatenate(xys)
    sco = np.arange(S + 1, dtype=np.int32)
    cpo = (np.arange(S + 1) * Np).astype(np.int32)
    rng = np.random.default_rng(3)
    x = np.stack([rng.uniform(800, 3200, S), rng.uniform(800, 2200, S), rng.uniform(-np.pi, np.pi, S)], 1)
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)]) + rng.normal(0, 0.3, (S, 2 * L))
    Rd = np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)
    P0 = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    u = np.tile([2.0, 2.5], (S, 1))
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=np.arange(S) + 9000, max_trials=2048, lmk_capacity=8,
                     ukf=dict(n_landmarks=L, x=x, P=P0, u=u, z=z, lmk=lmk, R_diag=Rd))
    p.run()
    r = p.results()
    for s in range(2):
        mo, md, _ = orc.ransac(xys[s], 20.0, 2048, state=orc.MTState(seed=9000 + s))
        assert np.array_equal(r["mask"][s * Np:(s + 1) * Np], mo)
        assert r["models"]["best_trial"][s] == md["best_trial"]
    xo, Po = oukf.ukf_batch(x, P0, u, z, lmk, Rd)
    err = ukf_exact.component_errors(r["ukf_x"], r["ukf_P"], xo, Po)  # 1e-5 per component
    assert max(err.values()) <= 1e-5, err
