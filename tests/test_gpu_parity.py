"""GPU parity: the HIP path (through the C ABI) against the reference golden
vectors and the CPU oracle, on the same seeded inputs.

Bit-exact: MT19937 draws/state, per-trial counts, winning trial, inlier masks,
origins, directions and line parameters vs the oracle (same closed-form refit),
landmark ids/lives, projected y vs the oracle.  Against the reference's own
numbers (LAPACK direction): directions <= 1e-11, a/b/tip_y/y_proj <= 1e-9 rel.
"""
import numpy as np
import pytest

from oracle import cpu as orc

pytestmark = pytest.mark.gpu

REL = 1e-9


@pytest.fixture(scope="module")
def ctx():
    from lidar_slam_amd.device import Context
    if Context.device_count() < 1:
        pytest.skip("no HIP device")
    return Context(0)


def _rel(a, b):
    a = np.asarray(a, np.float64)
    b = np.asarray(b, np.float64)
    return np.abs(a - b) / np.maximum(np.abs(b), 1.0)


def _ukf_close(x, P, xo, Po, tol=1e-5):
    from oracle import ukf_exact
    err = ukf_exact.component_errors(x, P, xo, Po)
    assert max(err.values()) <= tol, err


def _dir_ok(ux, uy, ref, tol=1e-11):
    u = np.stack([ux, uy], -1)
    return np.all(np.minimum(np.max(np.abs(u - ref), -1), np.max(np.abs(u + ref), -1)) <= tol)


def test_hyp_mt19937_matches_reference_draws(ctx, golden):
    from lidar_slam_amd import pipeline as pl
    g = golden("batch.npz")
    assert np.all(g["draws_used"] == 101)
    draws, state = pl.hyp_mt19937(ctx, g["scan_chunk_off"], g["chunk_pt_off"], seeds=g["seeds"])
    assert np.array_equal(draws, g["draws"])
    last = g["scan_chunk_off"][1:] - 1
    assert np.array_equal(state[:, :624], g["state_after_key"][last])
    assert np.array_equal(state[:, 624], g["state_after_pos"][last])


def test_hyp_mt19937_small_n(ctx, golden):
    from lidar_slam_amd import pipeline as pl
    g = golden("mt_choice.npz")
    for j, n in enumerate(g["ns"]):
        S = len(g["seeds"])
        ndraw = g["draws"].shape[2]
        # one chunk of n points per scan, max_trials = ndraw - 1
        sco = np.arange(S + 1, dtype=np.int32)
        cpo = (np.arange(S + 1) * int(n)).astype(np.int32)
        draws, state = pl.hyp_mt19937(ctx, sco, cpo, seeds=g["seeds"], max_trials=ndraw - 1)
        assert np.array_equal(draws, g["draws"][:, j]), n
        assert np.array_equal(state[:, :624], g["after_key"][:, j]), n
        assert np.array_equal(state[:, 624], g["after_pos"][:, j]), n


def _run_batch(ctx, g, seeds=None, mt_state=None, threshold=20.0, trials=100, assoc=True, cap=64, **kw):
    from lidar_slam_amd.pipeline import ScanPipeline
    p = ScanPipeline(ctx, g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], seeds=seeds, mt_state=mt_state,
                     threshold=threshold, max_trials=trials, lmk_capacity=cap if assoc else None,
                     want_draws=True, want_counts=True, want_state=True, **kw)
    p.run()
    return p.results()


def _check_vs_golden(g, r):
    m = r["models"]
    assert np.array_equal(r["draws"], g["draws"])
    assert np.array_equal(r["counts"], g["trial_cnt"])
    assert np.array_equal(m["best_trial"], g["best_trial"])
    assert np.array_equal(m["n_draws"], g["draws_used"])
    assert np.array_equal(r["mask"], g["mask"])
    assert np.array_equal(m["ox"], g["origin"][:, 0]) and np.array_equal(m["oy"], g["origin"][:, 1])
    assert _dir_ok(m["ux"], m["uy"], g["direction"])
    assert np.all(_rel(m["a"], g["a"]) < REL) and np.all(_rel(m["b"], g["b"]) < REL)
    assert np.array_equal(m["tip_x"], g["tip"][:, 0]) and np.all(_rel(m["tip_y"], g["tip"][:, 1]) < REL)
    assert np.array_equal((m["flags"] & 64) != 0, g["new_landmark"].astype(bool))
    sel = r["mask"].astype(bool)
    assert np.array_equal(g["xy"][sel, 0], g["q_x"])
    assert np.all(_rel(r["y_proj"][sel], g["q_y"]) < REL)


@pytest.mark.parametrize("n,trials", [(100, 250), (200, 100), (256, 70), (300, 60), (1000, 40)])
def test_hyp_mt19937_resolve_paths(ctx, n, trials):
    """Draws of chunks whose steps exceed the 16 KiB LDS stage (u8 steps for N <= 256, u16
    above): the tiled resolve_big_kernel path, chained over 3 chunks per scan, vs the
    oracle's choice(N, 2) sequence."""
    from lidar_slam_amd import pipeline as pl
    seeds = [11, 12, 13]
    S = len(seeds)
    sizes = [n, n - 7, n + 3]
    sco = np.arange(0, 3 * S + 1, 3, dtype=np.int32)
    cpo = np.concatenate([[0], np.cumsum(sizes * S)]).astype(np.int32)
    draws, state = pl.hyp_mt19937(ctx, sco, cpo, seeds=seeds, max_trials=trials)
    for s, seed in enumerate(seeds):
        st = orc.MTState(seed=seed)
        for k, nk in enumerate(sizes):
            ref = np.array([st.choice2(nk) for _ in range(trials + 1)])
            assert np.array_equal(draws[3 * s + k], ref), (n, trials, s, k)
        assert np.array_equal(state[s, :624], st.key) and state[s, 624] == st.pos.value


def test_batch_pipeline_vs_reference(ctx, golden):
    g = golden("batch.npz")
    r = _run_batch(ctx, g, seeds=g["seeds"])
    _check_vs_golden(g, r)
    # per-scan landmark lists after the scan's last chunk
    for s in range(len(g["seeds"])):
        c = g["scan_chunk_off"][s + 1] - 1
        l0, l1 = g["lm_off"][c], g["lm_off"][c + 1]
        n = r["lmk_count"][s]
        lst = r["landmarks"][s, :n]
        assert list(lst["id"]) == list(g["lm_id"][l0:l1])
        assert list(lst["life"]) == list(g["lm_life"][l0:l1])
        assert np.all(_rel(lst["a"], g["lm_a"][l0:l1]) < REL)
    # state after each scan
    last = g["scan_chunk_off"][1:] - 1
    assert np.array_equal(r["mt_state"][:, :624], g["state_after_key"][last])


def test_batch_pipeline_vs_oracle_bitexact(ctx, golden):
    g = golden("batch.npz")
    r = _run_batch(ctx, g, seeds=g["seeds"])
    mask, yproj, models, lists = orc.run_batch(g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], g["seeds"])
    m = r["models"]
    assert np.array_equal(r["mask"], mask)
    for f in ("ox", "oy", "ux", "uy", "a", "b", "tip_x", "tip_y", "proj_a", "proj_b"):
        assert np.array_equal(m[f], np.array([d[f] for d in models])), f
    for f in ("n_inliers", "best_trial", "n_draws", "flags", "match_index", "landmark_id"):
        assert np.array_equal(m[f], np.array([d[f] for d in models])), f
    assert np.array_equal(r["y_proj"], yproj)


def test_live_chain_one_stream_one_list(ctx, golden):
    """SLAM.py live semantics: one np.random.seed, one landmark list, 112 chunks."""
    g = golden("live.npz")
    gg = dict(g)
    gg["scan_chunk_off"] = np.array([0, len(g["a"])], np.int32)
    r = _run_batch(ctx, gg, seeds=g["seed"], cap=128)
    _check_vs_golden(gg, r)
    c = len(g["a"]) - 1
    l0, l1 = g["lm_off"][c], g["lm_off"][c + 1]
    lst = r["landmarks"][0, :r["lmk_count"][0]]
    assert list(lst["id"]) == list(g["lm_id"][l0:l1])
    assert list(lst["life"]) == list(g["lm_life"][l0:l1])
    assert np.array_equal(r["mt_state"][0, :624], g["state_after_key"][c])
    assert r["mt_state"][0, 624] == g["state_after_pos"][c]


def test_mt_state_in_continues_stream(ctx, golden):
    """Explicit state in/out (the drop-in shim path): chunk-by-chunk calls with
    the fixture's entry states reproduce the chained run."""
    g = golden("live.npz")
    C = 12
    st = np.concatenate([g["state_before_key"][:C], g["state_before_pos"][:C, None].astype(np.uint32)], 1)
    gg = {"xy": g["xy"], "chunk_pt_off": g["chunk_pt_off"][:C + 1],
          "scan_chunk_off": np.arange(C + 1, dtype=np.int32)}
    r = _run_batch(ctx, gg, mt_state=st, assoc=False)
    assert np.array_equal(r["mask"], g["mask"][:g["chunk_pt_off"][C]])
    assert np.array_equal(r["mt_state"][:, :624], g["state_after_key"][:C])
    assert np.array_equal(r["mt_state"][:, 624], g["state_after_pos"][:C])


def test_early_stop_rewinds_stream(ctx, golden):
    g = golden("edge_chain.npz")
    r = _run_batch(ctx, g, seeds=g["seed"])
    assert list(r["models"]["n_draws"]) == [101, 2, 101]
    assert r["models"]["flags"][1] & 16
    assert np.array_equal(r["mask"], g["mask"])
    assert np.array_equal(r["draws"][2], g["draws"][2])
    assert np.array_equal(r["mt_state"][0, :624], g["state_after_key"][-1])
    assert r["mt_state"][0, 624] == g["state_after_pos"][-1]


def test_edge_cases(ctx, golden):
    g = golden("edge.npz")
    for k, name in enumerate(g["names"]):
        xy = g["xy"][g["off"][k]:g["off"][k + 1]]
        gg = {"xy": xy, "scan_chunk_off": np.array([0, 1], np.int32),
              "chunk_pt_off": np.array([0, len(xy)], np.int32)}
        r = _run_batch(ctx, gg, seeds=g["seeds"][k:k + 1], threshold=float(g["thr"][k]),
                       trials=int(g["trials"][k]), assoc=False)
        m = r["models"][0]
        err = g["err"][k]
        if err == 1:
            assert m["flags"] & (2 | 8), name
        elif err == 2:
            assert m["flags"] & 4, name
        else:
            assert m["flags"] & 1, name
            p = g["params"][k]
            assert np.array_equal(r["mask"], g["mask"][g["off"][k]:g["off"][k + 1]]), name
            assert m["ox"] == p[0] and m["oy"] == p[1], name
            assert _dir_ok(m["ux"], m["uy"], p[2:4]), name
        assert np.array_equal(r["mt_state"][0, :624], g["after_key"][k]), name
        assert r["mt_state"][0, 624] == g["after_pos"][k], name
        # and bit-exact with the oracle
        mo, md, _ = orc.ransac(xy, float(g["thr"][k]), int(g["trials"][k]), state=orc.MTState(seed=int(g["seeds"][k])))
        assert np.array_equal(r["mask"], mo), name
        for f in ("ox", "oy", "ux", "uy", "a", "b"):
            assert np.array_equal(m[f], md[f]) or (np.isnan(m[f]) and np.isnan(md[f])), (name, f)


def test_assoc_crafted_lists(ctx, golden):
    from lidar_slam_amd.pipeline import LANDMARK_DTYPE, ScanPipeline
    g = golden("assoc.npz")
    K = len(g["names"])
    cap = 16
    lm = np.zeros((K, cap), LANDMARK_DTYPE)
    cnt = np.zeros(K, np.int32)
    for k in range(K):
        i0, i1 = g["lm_in_off"][k], g["lm_in_off"][k + 1]
        n = i1 - i0
        cnt[k] = n
        lm[k, :n]["a"], lm[k, :n]["b"] = g["lm_in_a"][i0:i1], g["lm_in_b"][i0:i1]
        lm[k, :n]["pos_x"], lm[k, :n]["pos_y"] = g["lm_in_pos"][i0:i1, 0], g["lm_in_pos"][i0:i1, 1]
        lm[k, :n]["end_x"], lm[k, :n]["end_y"] = g["lm_in_end"][i0:i1, 0], g["lm_in_end"][i0:i1, 1]
        lm[k, :n]["id"], lm[k, :n]["life"] = g["lm_in_id"][i0:i1], g["lm_in_life"][i0:i1]
    xy = np.tile(g["xy"], (K, 1))
    n = len(g["xy"])
    p = ScanPipeline(ctx, xy, np.arange(K + 1, dtype=np.int32), (np.arange(K + 1) * n).astype(np.int32),
                     seeds=np.full(K, g["seed"][0]), landmarks=lm, lmk_count=cnt,
                     id_base=np.full(K, 99, np.int32))
    p.run()
    r = p.results()
    for k, name in enumerate(g["names"]):
        o0, o1 = g["lm_out_off"][k], g["lm_out_off"][k + 1]
        lst = r["landmarks"][k, :r["lmk_count"][k]]
        assert list(lst["id"]) == list(g["lm_out_id"][o0:o1]), name
        assert list(lst["life"]) == list(g["lm_out_life"][o0:o1]), name
        assert bool(r["models"]["flags"][k] & 64) == bool(g["new_landmark"][k]), name
        q0, q1 = g["q_off"][k], g["q_off"][k + 1]
        sel = r["mask"][k * n:(k + 1) * n].astype(bool)
        assert np.all(_rel(r["y_proj"][k * n:(k + 1) * n][sel], g["q_y"][q0:q1]) < REL), name


def test_big_c5_chunks(ctx, golden):
    g = golden("big.npz")
    S = len(g["seeds"])
    gg = {"xy": g["xy"], "scan_chunk_off": np.arange(S + 1, dtype=np.int32), "chunk_pt_off": g["off"]}
    r = _run_batch(ctx, gg, seeds=g["seeds"], trials=int(g["trials"]), assoc=False)
    assert np.array_equal(r["mask"], g["mask"])
    assert np.array_equal(r["models"]["best_trial"], g["best_trial"])
    assert np.array_equal(r["mt_state"][:, :624], g["after_key"])


def test_philox_and_explicit_vs_oracle(ctx, golden):
    from lidar_slam_amd.pipeline import ScanPipeline
    g = golden("batch.npz")
    p = ScanPipeline(ctx, g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], hyp="philox", want_draws=True,
                     lmk_capacity=64)
    p.run()
    r = p.results()
    d = r["draws"]
    sizes = np.diff(g["chunk_pt_off"])
    assert np.all(d[..., 0] != d[..., 1])
    assert np.all((d >= 0) & (d < sizes[:, None, None]))
    # the same draws through the explicit path and through the oracle
    p2 = ScanPipeline(ctx, g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], hyp="explicit", hyp_draws=d)
    p2.run()
    r2 = p2.results()
    assert np.array_equal(r2["mask"], r["mask"])
    for c in range(len(sizes)):
        p0, p1 = g["chunk_pt_off"][c], g["chunk_pt_off"][c + 1]
        mo, md, _ = orc.ransac(g["xy"][p0:p1], 20.0, 100, hyp=d[c])
        assert np.array_equal(r["mask"][p0:p1], mo), c
        assert r["models"]["a"][c] == md["a"] and r["models"]["best_trial"][c] == md["best_trial"]


def test_philox_pipeline_with_side_ukf_and_assoc(ctx, golden):
    """Philox hypotheses + association + UKF: the UKF (it reads nothing of the RANSAC) runs on
    the side stream beside the consensus, the association pass in the waves_per_eu(4) build.
    Two chained calls: x/P in/out vs the oracle UKF, masks/lists vs the explicit-draw path and
    the stand-alone association entry point."""
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import ukf as oukf
    g = golden("batch.npz")
    S = len(g["scan_chunk_off"]) - 1
    L = 8
    rng = np.random.default_rng(17)
    x0 = np.column_stack([rng.uniform(500, 3500, S), rng.uniform(500, 2500, S), rng.uniform(-3, 3, S)])
    P0 = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    z = np.stack([oukf.transfer_function(x0[s], lmk[s]) for s in range(S)]) + rng.normal(0, 0.2, (S, 2 * L))
    u = np.tile([2.0, 2.5], (S, 1))
    Rd = np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)
    ukf = dict(n_landmarks=L, x=x0, P=P0, u=u, z=z, lmk=lmk, R_diag=Rd)
    p = ScanPipeline(ctx, g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], hyp="philox", want_draws=True,
                     lmk_capacity=64, ukf=ukf)
    p.run(sync=False)
    p.run()  # the second call chains x/P from the first
    r = p.results()
    xo, Po = oukf.ukf_batch(x0, P0, u, z, lmk, Rd)
    xo, Po = oukf.ukf_batch(xo, Po, u, z, lmk, Rd)
    _ukf_close(r["ukf_x"], r["ukf_P"], xo, Po)
    # association: the explicit path with the same draws, fresh lists, one call
    p2 = ScanPipeline(ctx, g["xy"], g["scan_chunk_off"], g["chunk_pt_off"], hyp="explicit", hyp_draws=r["draws"],
                      lmk_capacity=64)
    p2.run()
    r2 = p2.results()
    assert np.array_equal(r2["mask"], r["mask"])
    # stand-alone association entry point over the models of the explicit call, fresh lists
    p2.reset_state()
    p2.run_landmarks_only()
    r3 = p2.results()
    for k in ("lmk_count",):
        assert np.array_equal(r3[k], r2[k])
    assert np.array_equal(r3["landmarks"]["id"], r2["landmarks"]["id"])
    assert np.array_equal(r3["y_proj"], r2["y_proj"])


@pytest.mark.parametrize("hyp,n_beams,chunk", [("mt19937", 720, None), ("philox", 600, 600)])
def test_fused_polar_loads_equal_polar_kernel_then_xy(ctx, hyp, n_beams, chunk):
    """A1 fused into every point load (xy = NULL, theta/dist given): the whole pipeline (small
    chunks with association + UKF, and > 128-point chunks through the model / count / select
    kernels) gives exactly the outputs of lslam_polar_to_xy followed by the xy pipeline."""
    from lidar_slam_amd import pipeline as pl
    from lidar_slam_amd import synth
    from oracle import ukf as oukf
    ids = list(range(24))
    b = synth.make_batch(ids, n_beams)
    if chunk:  # one chunk per scan
        S = len(ids)
        b["scan_chunk_off"] = np.arange(S + 1, dtype=np.int32)
        b["chunk_pt_off"] = (np.arange(S + 1) * n_beams).astype(np.int32)
    S = len(b["scan_chunk_off"]) - 1
    L = 8
    rng = np.random.default_rng(3)
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    ukf = dict(n_landmarks=L, x=b["poses"].copy(), P=np.tile(np.diag([.1, .1, .05]), (S, 1, 1)),
               u=np.tile([2.0, 2.5], (S, 1)), z=np.stack([oukf.transfer_function(b["poses"][s], lmk[s])
                                                        for s in range(S)]),
               lmk=lmk, R_diag=np.array([0.25, 0.09] * L), flags=7)
    xy_dev = pl.polar_to_xy(ctx, b["theta_deg"], b["dist_mm"])
    kw = dict(seeds=np.array(ids), hyp=hyp, lmk_capacity=32, ukf=ukf, max_trials=100 if not chunk else 256)
    pa = pl.ScanPipeline(ctx, xy_dev, b["scan_chunk_off"], b["chunk_pt_off"], **kw)
    pb = pl.ScanPipeline(ctx, None, b["scan_chunk_off"], b["chunk_pt_off"], theta_deg=b["theta_deg"],
                         dist_mm=b["dist_mm"], **kw)
    pa.run()
    pb.run()
    ra, rb = pa.results(), pb.results()
    assert int(np.sum(ra["models"]["flags"] & 1)) > 0
    for k in ("mask", "y_proj", "lmk_count", "ukf_x", "ukf_P"):
        assert np.array_equal(ra[k], rb[k]), k
    assert ra["models"].tobytes() == rb["models"].tobytes()
    assert ra["landmarks"].tobytes() == rb["landmarks"].tobytes()


def test_polar_to_xy(ctx):
    from lidar_slam_amd import pipeline as pl
    from lidar_slam_amd import synth
    th, d, _ = synth.scan_polar(3)
    xy = pl.polar_to_xy(ctx, th, d)
    ref = synth.polar_to_xy_ref(th, d)
    assert np.max(np.abs(xy - ref)) < 1e-9


def test_ukf_vs_oracle(ctx):
    from lidar_slam_amd.pipeline import ScanPipeline
    from oracle import ukf as oukf
    rng = np.random.default_rng(11)
    S, L = 96, 20
    x = np.stack([rng.uniform(800, 3200, S), rng.uniform(800, 2200, S), rng.uniform(-np.pi, np.pi, S)], 1)
    P = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    u = np.tile([2.0, 2.5], (S, 1))
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)]) + rng.normal(0, 0.3, (S, 2 * L))
    Rd = np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)
    xo, Po = oukf.ukf_batch(x, P, u, z, lmk, Rd)
    # UKF only: no chunks
    p = ScanPipeline(ctx, np.zeros((1, 2)), np.zeros(S + 1, np.int32), np.zeros(1, np.int32),
                     ukf=dict(n_landmarks=L, x=x, P=P, u=u, z=z, lmk=lmk, R_diag=Rd))
    p.run_ukf_only()
    r = p.results()
    # north_star's 1e-5 per component (x, y relative; theta absolute; P relative to max|P|).
    # Both sides are float64 evaluations of the same steps; each is within 1e-5 of the
    # 50-digit evaluation (tests/test_ukf_exact.py, tests/test_gpu_ukf_exact.py).
    _ukf_close(r["ukf_x"], r["ukf_P"], xo, Po)


@pytest.mark.parametrize("L", [20, 4])
def test_fused_ukf_landmarks_from_ransac_vs_oracle(ctx, L):
    """flags = PREDICT | UPDATE | LMK_FROM_RANSAC in the fused pipeline: landmark slot j of
    scan s becomes chunk j's fitted origin (Landmark.pos, ransac_functions.py:31) wherever that
    chunk is LSLAM_VALID, the rest keep ukf_lmk.  The kernel's (x, P) must equal the oracle's UKF
    run on exactly that substituted landmark set (1e-5 per component).  L = 4 < 8 chunks: only
    the first L chunks feed slots.  (The one-wave UKF form runs in map mode: test_gpu_map.py.)"""
    from lidar_slam_amd.pipeline import ScanPipeline
    from lidar_slam_amd import synth
    from lidar_slam_amd.device import Context
    from oracle import ukf as oukf
    ids = list(range(40))
    b = synth.make_batch(ids)
    S = len(ids)
    rng = np.random.default_rng(17)
    lmk = rng.uniform(-3000, 3000, (S, L, 2))
    x = b["poses"].copy()
    z = np.stack([oukf.transfer_function(x[s], lmk[s]) for s in range(S)]) + rng.normal(0, 0.3, (S, 2 * L))
    P = np.tile(np.diag([.1, .1, .05]), (S, 1, 1))
    u = np.tile([2.0, 2.5], (S, 1))
    Rd = np.array([oukf.VAR_DIST, oukf.VAR_ANGLE] * L)
    p = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                     ukf=dict(n_landmarks=L, x=x, P=P, u=u, z=z, lmk=lmk, R_diag=Rd, flags=7))
    p.run()
    r = p.results()
    m = r["models"]
    sco = b["scan_chunk_off"]
    lmk2 = lmk.copy()
    replaced = 0
    for s in range(S):
        for j in range(min(L, sco[s + 1] - sco[s])):
            c = sco[s] + j
            if m["flags"][c] & 1:
                lmk2[s, j] = (m["ox"][c], m["oy"][c])
                replaced += 1
    assert replaced >= S * min(L, 8) * 0.9
    xo, Po = oukf.ukf_batch(x, P, u, z, lmk2, Rd)
    _ukf_close(r["ukf_x"], r["ukf_P"], xo, Po)
    # and it is not the un-substituted step
    xn, _ = oukf.ukf_batch(x, P, u, z, lmk, Rd)
    assert np.max(np.abs(r["ukf_x"] - xn)) > 1e-3


def _border_batch():
    """Chunks whose residuals sit on the inlier threshold (r^2 within ulps of
    the cutoff, where the consensus kernel's cheap cross-product test defers to
    the exact residual), duplicated points (degenerate hypotheses, u = d), and
    mixtures of both."""
    thr2 = [20.0, np.nextafter(20.0, 0), np.nextafter(20.0, 40), 19.999999999999996, 20.000000000000004]
    chunks = []
    xs = np.arange(0.0, 60.0, 1.5)
    # 1) axis-aligned line + points at exactly/near the threshold distance
    ys = np.zeros_like(xs)
    ys[1::4] = [thr2[k % 5] * (1 if k % 2 else -1) for k in range(len(ys[1::4]))]
    chunks.append(np.stack([xs, ys], 1))
    # 2) the same rotated by 90 degrees, shifted
    chunks.append(np.stack([ys + 1000.0, xs - 500.0], 1))
    # 3) many duplicates: draws of two copies give a zero direction
    d = np.array([[3.0, 4.0]] * 30 + [[3.0, 24.0]] * 10 + [[23.0, 4.0]] * 10 + [[100.0, 100.0]] * 5)
    chunks.append(d)
    # 4) duplicates on a line plus threshold-distance points
    e = np.concatenate([np.stack([xs[:20], 2 * xs[:20]], 1), np.repeat([[7.0, 14.0]], 15, 0),
                        np.stack([xs[:12], 2 * xs[:12] + 20.0 * np.sqrt(5.0)], 1)])
    chunks.append(e)
    # 5) every point on a slanted line: residuals ~1e-15, all 100 trials tied
    chunks.append(np.stack([xs, 0.5 * xs + 3.0], 1))
    # 6) every point on y = 7: residuals exactly 0, the zero-sum early stop
    #    (the producer's draws for the following chunks are then replayed)
    chunks.append(np.stack([xs, np.full_like(xs, 7.0)], 1))
    chunks.append(chunks[0][::-1].copy())
    return chunks


def _border_batch_large():
    """The border chunks grown past 128 points (the count/select kernels): copies
    shifted along each chunk's own line keep the threshold distances; chunk 3
    repeats its duplicates."""
    c = _border_batch()
    along = [(60.0, 0.0), (0.0, 60.0), None, (30.0, 60.0), (60.0, 30.0), (60.0, 0.0), (-60.0, 0.0)]
    out = []
    for ch, v in zip(c, along):
        reps = [ch + (0.0 if v is None else np.array(v) * k) for k in range(5)]
        out.append(np.concatenate(reps))
    return out


@pytest.mark.parametrize("large", [False, True])
def test_border_band_and_degenerate_hypotheses(ctx, large):
    chunks = _border_batch_large() if large else _border_batch()
    if large:
        assert min(len(ch) for ch in chunks) > 128
    seeds = np.arange(40, dtype=np.uint32) * 7919 + 11
    S = len(seeds)
    xy = np.concatenate([np.concatenate(chunks)] * S)
    sizes = [len(c) for c in chunks] * S
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    sco = (np.arange(S + 1) * len(chunks)).astype(np.int32)
    g = {"xy": xy, "scan_chunk_off": sco, "chunk_pt_off": cpo}
    r = _run_batch(ctx, g, seeds=seeds, assoc=False)
    m = r["models"]
    c = 0
    for s in range(S):
        st = orc.MTState(seed=int(seeds[s]))
        for ch in chunks:
            p0, p1 = cpo[c], cpo[c + 1]
            mo, md, ex = orc.ransac(ch, 20.0, 100, state=st, want_trials=True)
            assert np.array_equal(r["mask"][p0:p1], mo), (s, c)
            assert np.array_equal(r["counts"][c], ex["cnt"]), (s, c)
            for f in ("best_trial", "n_draws", "flags", "n_inliers"):
                assert m[f][c] == md[f], (s, c, f)
            for f in ("ox", "oy", "ux", "uy", "a", "b"):
                assert m[f][c] == md[f] or (np.isnan(m[f][c]) and np.isnan(md[f])), (s, c, f)
            c += 1
        assert np.array_equal(r["mt_state"][s, :624], st.key) and r["mt_state"][s, 624] == st.pos.value, s


def test_batch256_pipeline_vs_reference(ctx, golden):
    """The 256-scan reference batch (tests/golden/batch256.npz) through the fused pipeline:
    masks, per-trial counts, winners, draws used, origins exact; directions <= 1e-11; a, b,
    tip_y <= 1e-9 relative; new-landmark decisions, each scan's final list (ids, lives) and
    final MT state (hash) exact."""
    import hashlib

    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    g = golden("batch256.npz")
    S = int(g["n_scans"])
    b = synth.make_batch(list(range(S)))
    assert hashlib.sha256(b["xy"].tobytes()).digest() == g["xy_sha256"].tobytes()
    p = ScanPipeline(ctx, b["xy"], g["scan_chunk_off"], g["chunk_pt_off"], seeds=g["seeds"], lmk_capacity=64,
                     want_counts=True, want_state=True)
    p.run()
    r = p.results()
    m = r["models"]
    assert np.array_equal(r["mask"], g["mask"])
    assert np.array_equal(r["counts"].astype(np.uint8), g["trial_cnt"])
    assert np.array_equal(m["best_trial"], g["best_trial"]) and np.array_equal(m["n_draws"], g["draws_used"])
    assert np.array_equal(m["n_inliers"], g["n_inl"])
    assert np.array_equal(m["ox"], g["origin"][:, 0]) and np.array_equal(m["oy"], g["origin"][:, 1])
    assert _dir_ok(m["ux"], m["uy"], g["direction"])
    assert np.all(_rel(m["a"], g["a"]) < REL) and np.all(_rel(m["b"], g["b"]) < REL)
    assert np.array_equal(m["tip_x"], g["tip"][:, 0]) and np.all(_rel(m["tip_y"], g["tip"][:, 1]) < REL)
    assert np.array_equal((m["flags"] & 64) != 0, g["new_landmark"].astype(bool))
    for s in range(S):
        c = g["scan_chunk_off"][s + 1] - 1
        l0, l1 = g["lm_out_off"][c], g["lm_out_off"][c + 1]
        lst = r["landmarks"][s, :r["lmk_count"][s]]
        assert list(lst["id"]) == list(g["lm_out_id"][l0:l1]) and list(lst["life"]) == list(g["lm_out_life"][l0:l1])
        st = r["mt_state"][s]
        h = int.from_bytes(hashlib.sha256(st[:624].tobytes() + np.int32(st[624]).tobytes()).digest()[:8], "little")
        assert h == int(g["state_after_hash"][s]), s


@pytest.mark.parametrize("cap", [64, 24])
def test_assoc_lists_stress_vs_oracle(ctx, cap):
    """The association-only post pass (its landmark list in registers when lmk_capacity <= 64,
    post_assoc_reg) against the oracle's chained landmark_extraction
    (ransac_functions.py:15-59, landmarking.py:48-77): input lists of 0..cap entries mixing
    near-copies of the scan's own walls (matches), junk lines and lives of 1..3 (runs of
    removals, skip-after-remove), full lists (a new landmark dropped: LSLAM_CAPACITY).  Final
    lists (ids, lives, lines), per-chunk new/matched/capacity flags and y_proj exact."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import LANDMARK_DTYPE, ScanPipeline
    S = 48
    ids = list(range(300, 300 + S))
    b = synth.make_batch(ids, 720)
    xy, sco, cpo = b["xy"], b["scan_chunk_off"], b["chunk_pt_off"]
    rng = np.random.default_rng(7)
    # the scans' own fitted walls (oracle, empty lists) seed plausible matches
    walls = []
    for s in range(S):
        st = orc.MTState(seed=s)
        ws = []
        for k, c in enumerate(range(sco[s], sco[s + 1])):
            _, _, mod, _ = orc.landmark_extraction(xy[cpo[c]:cpo[c + 1]], k, [], st, cap=1)
            if mod["flags"] & 1:
                ws.append(mod)
        walls.append(ws)
    lm = np.zeros((S, cap), LANDMARK_DTYPE)
    cnt = np.zeros(S, np.int32)
    lists_in = []
    for s in range(S):
        full = s % 5 == 0  # a full list of long-lived junk: nothing matches or dies, nothing fits
        n = cap if full else int(rng.integers(0, cap + 1))
        lst = []
        for i in range(n):
            if walls[s] and not full and rng.random() < 0.5:
                w = walls[s][int(rng.integers(len(walls[s])))]
                a, bb = w["a"] + rng.normal(0, 0.01), w["b"] + rng.normal(0, 2.0)
                pos, end = (w["ox"], w["oy"]), (w["tip_x"], w["tip_y"])
            else:
                a, bb = rng.normal(0, 3), rng.normal(0, 3000)
                pos, end = tuple(rng.uniform(-5000, 5000, 2)), tuple(rng.uniform(-5000, 5000, 2))
            life = 40 if full else int(rng.choice([1, 1, 2, 3, 40]))
            lst.append({"a": float(a), "b": float(bb), "pos": (float(pos[0]), float(pos[1])),
                        "end": (float(end[0]), float(end[1])), "id": 5000 + i, "life": life})
        lists_in.append(lst)
        cnt[s] = n
        for i, L in enumerate(lst):
            lm[s, i] = (L["a"], L["b"], L["pos"][0], L["pos"][1], L["end"][0], L["end"][1], L["id"], L["life"])
    id_base = (np.arange(S) * 100).astype(np.int32)
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=np.arange(S, dtype=np.uint32), landmarks=lm, lmk_count=cnt,
                     lmk_capacity=cap, id_base=id_base)
    p.run()
    r = p.results()
    m = r["models"]
    n_cap = 0
    for s in range(S):
        st = orc.MTState(seed=s)
        lst = [dict(L) for L in lists_in[s]]
        for k, c in enumerate(range(sco[s], sco[s + 1])):
            p0, p1 = cpo[c], cpo[c + 1]
            mask, yp, mod, lst = orc.landmark_extraction(xy[p0:p1], int(id_base[s]) + k, lst, st, cap=cap)
            assert np.array_equal(r["mask"][p0:p1], mask), (s, k)
            assert np.array_equal(r["y_proj"][p0:p1], yp), (s, k)
            for f in (64, 128, 256):
                assert bool(m["flags"][c] & f) == bool(mod["flags"] & f), (s, k, f)
            n_cap += bool(m["flags"][c] & 256)
        got = r["landmarks"][s, :r["lmk_count"][s]]
        assert r["lmk_count"][s] == len(lst), s
        assert list(got["id"]) == [L["id"] for L in lst], s
        assert list(got["life"]) == [L["life"] for L in lst], s
        assert np.array_equal(got["a"], [L["a"] for L in lst]) and np.array_equal(got["end_y"], [L["end"][1] for L in lst])
    assert n_cap > 0  # the full-list case was exercised


@pytest.mark.gpu
@pytest.mark.parametrize("cap", [8, 80])
def test_assoc_distance_at_tolerance_vs_oracle(ctx, cap):
    """is_equal's distance tests (landmarking.py:57-72, sqrt(e) <= TOL_DIST) at the tolerance itself:
    the kernel compares e against the last value whose rounded square root is <= TOL_DIST
    (lslam_host_math.h sqrt_le_bound), the oracle takes the square root.  Each scan's list holds
    one landmark on its first fitted wall's line whose end lies k ulps around TOL_DIST from the
    wall's origin (k = -3..2), so some match and some do not; flags, lists and y_proj must equal
    the oracle's.  cap = 8 runs the post pass's register list (is_equal_reg, lmk_cap <= 64),
    cap = 80 its LDS list (is_equal)."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import LANDMARK_DTYPE, ScanPipeline
    S = 12
    b = synth.make_batch(list(range(700, 700 + S)), 720)
    xy, sco, cpo = b["xy"], b["scan_chunk_off"], b["chunk_pt_off"]
    tol = 100.0
    lm = np.zeros((S, cap), LANDMARK_DTYPE)
    cnt = np.zeros(S, np.int32)
    lists_in = []
    for s in range(S):
        st = orc.MTState(seed=s)
        w = None
        for k, c in enumerate(range(sco[s], sco[s + 1])):
            _, _, mod, _ = orc.landmark_extraction(xy[cpo[c]:cpo[c + 1]], k, [], st, cap=1)
            if mod["flags"] & 1:
                w = mod
                break
        assert w is not None
        # the end: ox + (tol moved by k ulps), same y, so e = fl(vx * vx) with vx = fl(end_x - ox)
        ex = w["ox"] + tol
        for _ in range(abs(s % 6 - 3)):
            ex = np.nextafter(ex, np.inf if s % 6 - 3 > 0 else -np.inf)
        L = {"a": float(w["a"]), "b": float(w["b"]), "pos": (float(w["tip_x"]) + 5000.0, float(w["tip_y"]) + 5000.0),
             "end": (float(ex), float(w["oy"])), "id": 9000 + s, "life": 40}
        lists_in.append([L])
        cnt[s] = 1
        lm[s, 0] = (L["a"], L["b"], L["pos"][0], L["pos"][1], L["end"][0], L["end"][1], L["id"], L["life"])
    id_base = (np.arange(S) * 100).astype(np.int32)
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=np.arange(S, dtype=np.uint32), landmarks=lm, lmk_count=cnt,
                     lmk_capacity=cap, id_base=id_base)
    p.run()
    r = p.results()
    m = r["models"]
    outcomes = set()
    for s in range(S):
        st = orc.MTState(seed=s)
        lst = [dict(L) for L in lists_in[s]]
        first = True
        for k, c in enumerate(range(sco[s], sco[s + 1])):
            p0, p1 = cpo[c], cpo[c + 1]
            mask, yp, mod, lst = orc.landmark_extraction(xy[p0:p1], int(id_base[s]) + k, lst, st, cap=cap)
            assert np.array_equal(r["y_proj"][p0:p1], yp), (s, k)
            for f in (64, 128, 256):
                assert bool(m["flags"][c] & f) == bool(mod["flags"] & f), (s, k, f)
            if first and mod["flags"] & 1:
                outcomes.add(bool(mod["flags"] & 128))
                first = False
        got = r["landmarks"][s, :r["lmk_count"][s]]
        assert list(got["id"]) == [L["id"] for L in lst], s
        assert list(got["life"]) == [L["life"] for L in lst], s
    assert outcomes == {True, False}  # both sides of the tolerance were exercised


@pytest.mark.gpu
def test_register_resolve_every_chunk_size_vs_oracle(ctx):
    """The packed register resolve (resolve_reg8_kernel: 64 (chunk, draw) items per wave, rows of
    different K in one wave poisoned past their K; full 16-step groups as SDWA byte compares, the
    XOR-64 domain from step 65) over every chunk size 3..128 in one pipeline call: each scan's
    chunks run through a different rotation of the sizes, so waves mix neighbouring sizes.  The
    draws (draw T included: draws_out) and end states against the oracle's choice(N, 2)."""
    from lidar_slam_amd import synth
    from lidar_slam_amd.pipeline import ScanPipeline
    trials = 30
    sizes_all = list(range(3, 129))
    S = 3
    sizes = [sizes_all[(s * 41 + i) % len(sizes_all)] for s in range(S) for i in range(len(sizes_all))]
    rng = np.random.default_rng(3)
    # noisy walls: every fit has >= 3 inliers with nonzero residuals, so no chunk stops early and
    # every chunk consumes exactly trials + 1 draws
    xs = rng.uniform(-3000.0, 3000.0, size=sum(sizes))
    xy = np.stack([xs, 0.3 * xs + 500.0 + rng.normal(0.0, 5.0, size=xs.size)], axis=1)
    per = len(sizes_all)
    sco = np.arange(0, S * per + 1, per, dtype=np.int32)
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    seeds = np.array([21, 22, 23], np.uint32)
    p = ScanPipeline(ctx, xy, sco, cpo, seeds=seeds, max_trials=trials, want_draws=True, want_state=True)
    p.run()
    r = p.results()
    draws = r["draws"]
    for s in range(S):
        st = orc.MTState(seed=int(seeds[s]))
        for k in range(per):
            c = s * per + k
            n = sizes[c]
            ref = np.array([st.choice2(n) for _ in range(trials + 1)])
            assert np.array_equal(draws[c], ref), (s, k, n)
            assert r["models"]["n_draws"][c] == trials + 1 and not r["models"]["flags"][c] & 16, (s, k)
        assert np.array_equal(r["mt_state"][s, :624], st.key) and r["mt_state"][s, 624] == st.pos.value, s
