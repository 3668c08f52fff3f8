"""Drop-in surface tests.  CPU: the modules import and mirror the reference's
names/constants; chunking (A2) follows functions.py:56-76.  GPU: the shim's
landmark_extraction reproduces the reference run chunk by chunk on numpy's
global RNG; System.ukf runs predict/update on the device."""
import numpy as np
import pytest

from lidar_slam_amd import functions, landmarking, ransac_functions, systemClass


def test_constants_mirror_reference():
    assert (ransac_functions.THRESHOLD, ransac_functions.MAX_TRIALS, ransac_functions.MIN_SAMPLES) == (20, 100, 2)
    assert (landmarking.LIFE, landmarking.TOLERANCE_A, landmarking.TOLERANCE_B, landmarking.TOLERANCE) == \
        (40, 0.1, 10, 100)
    assert systemClass.LANDMARK_NUMBER == 8 and systemClass.DT == 0.005
    assert functions.MIN_NEIGHBOORS == 100


def test_landmark_value_object():
    L = landmarking.Landmark(0.5, 3.0, 7, 1.0, 2.0, 50.0, 28.0)
    assert L.get_life() == 40 and L.get_id() == 7
    for _ in range(39):
        assert L.decrease_life() is None
    assert L.decrease_life() is True and L.get_life() == 0
    assert L.decrease_life() is True and L.get_life() == 0
    L.reset_life()
    assert L.get_life() == 40
    M = landmarking.Landmark(0.55, 3.0, 8, 50.0, 28.0, 500.0, 250.0)
    assert L.is_equal(M)  # ||pos_M - end_L|| = 0
    M.a = 0.7
    assert not L.is_equal(M)
    M.a = float("nan")
    assert not L.is_equal(M)
    sysm = systemClass.PoseHolder()
    assert sysm.get_dim_x() == 3 and np.array_equal(sysm.get_pos(), np.zeros(3))


def test_chunker_matches_functions_py():
    class Q(list):
        def put(self, x):
            self.append(x)

    q = Q()
    ch = functions.ScanChunker(q, warmup_s=0.0, start_time=-1.0)
    ch._emit = lambda: (q.put(len(ch.th)), ch.th.clear(), ch.d.clear())   # count instead of converting
    for k in range(720):
        ch.push(k == 719, k * 0.5, 1000.0, t=0.0)
    # 7 chunks of 100; the flagged 720th measure joins the remainder (20 > 2); then the delimiter
    assert q == [100] * 7 + [20, 0]
    q.clear()
    for k in range(701):
        ch.push(k == 700, k * 0.5, 1000.0, t=0.0)
    assert q == [100] * 7 + [0]      # remainder of 1 point is dropped (functions.py:71)
    assert list(functions.chunk_offsets(720)) == [0, 100, 200, 300, 400, 500, 600, 700, 720]


@pytest.mark.gpu
def test_shim_replays_live_reference_run(golden):
    """The live fixture (one global RNG stream, one landmark list, 112 chunks)
    replayed through ransac_functions.landmark_extraction on numpy's global state."""
    g = golden("live.npz")
    np.random.seed(int(g["seed"][0]))
    landmarks = []
    number = 0
    for c in range(len(g["a"])):
        p0, p1 = g["chunk_pt_off"][c], g["chunk_pt_off"][c + 1]
        pts = [g["xy"][p0:p1].tolist()]
        q, fitted, new = ransac_functions.landmark_extraction(pts, number, landmarks)
        assert pts == []
        if new:
            landmarks.append(fitted)
        number += 1
        st = np.random.get_state()
        assert np.array_equal(st[1], g["state_after_key"][c]) and st[2] == g["state_after_pos"][c]
        q0, q1 = g["q_off"][c], g["q_off"][c + 1]
        assert [p.x() for p in q] == list(g["q_x"][q0:q1])
        assert np.allclose([p.y() for p in q], g["q_y"][q0:q1], rtol=1e-9, atol=1e-9)
        assert bool(new) == bool(g["new_landmark"][c])
        l0, l1 = g["lm_off"][c], g["lm_off"][c + 1]
        assert [L.id for L in landmarks] == list(g["lm_id"][l0:l1])
        assert [L.life for L in landmarks] == list(g["lm_life"][l0:l1])


@pytest.mark.gpu
def test_shim_errors_match_reference():
    np.random.seed(3)
    with pytest.raises(ValueError):
        ransac_functions.landmark_extraction([[[0.0, 0.0], [1.0, 1.0]]], 0, [])
    st = np.random.get_state()
    assert np.array_equal(st[1], np.random.RandomState(3).get_state()[1])  # nothing consumed


@pytest.mark.gpu
def test_system_ukf_vs_oracle():
    from oracle import ukf as oukf
    sysm = systemClass.System([])
    sysm.ukf.x = np.array([1000.0, 800.0, 0.3])
    rng = np.random.default_rng(2)
    lm = [tuple(p) for p in rng.uniform(-3000, 3000, (8, 2))]
    z = oukf.transfer_function(np.array([1000.0, 800.0, 0.3]), lm) + 0.05
    sysm.ukf.predict(u=[2.0, 2.5])
    sysm.ukf.update(z, landmarks=lm)
    f = oukf.UKF(8)
    f.x = np.array([1000.0, 800.0, 0.3])
    f.predict(np.array([2.0, 2.5]))
    f.update(z, lm)
    from oracle import ukf_exact
    err = ukf_exact.component_errors(sysm.ukf.x[None], sysm.ukf.P[None], f.x[None], f.P[None])
    assert max(err.values()) <= 1e-5, err


@pytest.mark.gpu
def test_revolution_dispatcher_replays_live_reference_run(golden):
    """The live fixture's 112 chunks grouped into revolutions of 8 and run one
    launch per revolution (process_revolution) end in the reference's RNG
    state, landmark list and projected points after every revolution."""
    g = golden("live.npz")
    np.random.seed(int(g["seed"][0]))
    landmarks = []
    number = 0
    C = len(g["a"])
    for r0 in range(0, C, 8):
        cs = range(r0, min(r0 + 8, C))
        chunks = [g["xy"][g["chunk_pt_off"][c]:g["chunk_pt_off"][c + 1]] for c in cs]
        pts, number = ransac_functions.process_revolution(chunks, number, landmarks)
        last = cs[-1]
        st = np.random.get_state()
        assert np.array_equal(st[1], g["state_after_key"][last]) and st[2] == g["state_after_pos"][last]
        q0, q1 = g["q_off"][cs[0]], g["q_off"][last + 1]
        assert len(pts) == q1 - q0
        assert list(pts.x) == list(g["q_x"][q0:q1])
        assert np.allclose(pts.y, g["q_y"][q0:q1], rtol=1e-9, atol=1e-9)
        assert [p.x() for p in pts[:3]] == list(g["q_x"][q0:q0 + 3])
        l0, l1 = g["lm_off"][last], g["lm_off"][last + 1]
        assert [L.id for L in landmarks] == list(g["lm_id"][l0:l1])
        assert [L.life for L in landmarks] == list(g["lm_life"][l0:l1])
    assert number == C


@pytest.mark.gpu
def test_revolution_dispatcher_thread_and_error_replay():
    import threading
    import time as _t
    rng = np.random.default_rng(4)
    line = lambda n, s: np.stack([np.arange(n) * 10.0, s * np.arange(n) * 10.0 + rng.normal(0, 2, n)], 1)
    pts, pairs, allp, temp, lms = [], [], [], [], []
    ev, stop = threading.Event(), threading.Event()
    th = threading.Thread(target=ransac_functions.check_ransac_revolution,
                          args=(pairs, temp, allp, pts, lms, ev), kwargs={"stop": stop})
    np.random.seed(9)
    th.start()
    chunks = [line(100, 0.5), line(100, -1.0), line(20, 2.0)]
    for c in chunks:
        temp.append(c)
        pts.append(c.tolist())
    pts.append(0)
    t0 = _t.time()
    while not ev.is_set() and _t.time() - t0 < 60:
        _t.sleep(0.01)
    stop.set()
    th.join(10)
    assert ev.is_set() and len(pairs) == 1 and len(allp) == 1
    assert len(allp[0]) == 220 and len(pairs[0]) > 0
    # the per-chunk path from the same state gives the same points and list
    np.random.seed(9)
    lm2, q_all, n = [], [], 0
    for c in chunks:
        q, f, new = ransac_functions.landmark_extraction([c.tolist()], n, lm2)
        q_all += q
        if new:
            lm2.append(f)
        n += 1
    assert [p.x() for p in q_all] == list(pairs[0].x)
    assert [(L.id, L.life) for L in lm2] == [(L.id, L.life) for L in lms]
    # a 2-point chunk raises ValueError at that chunk, as in the reference
    with pytest.raises(ValueError):
        ransac_functions.process_revolution([line(50, 1.0), line(2, 1.0)], 0, [])


def test_ukf_dropin_arguments_are_strict():
    """filterpy's call surface (systemClass.py:21-29): per-call dt / R, required u / landmarks,
    and what the GPU step cannot represent raises instead of being dropped (CPU: the argument
    handling of lidar_slam_amd/ukf.py, no device)."""
    from lidar_slam_amd import ukf
    u, dt = ukf.predict_args(None, None, None, {"u": [2.0, 2.5]}, 0.005)
    assert dt == 0.005 and np.array_equal(u, [2.0, 2.5])
    assert ukf.predict_args(0.01, None, None, {"u": (0, 0)}, 0.005)[1] == 0.01
    with pytest.raises(TypeError):
        ukf.predict_args(None, None, None, {}, 0.005)           # transition_function needs u
    with pytest.raises(TypeError):
        ukf.predict_args(None, None, None, {"u": (0, 0), "v": 1}, 0.005)
    with pytest.raises(ValueError):
        ukf.predict_args(None, None, lambda *a: a, {"u": (0, 0)}, 0.005)
    R = np.diag([0.25, 0.09] * 2)
    lm = [(1.0, 2.0), (3.0, 4.0)]
    Rd, pos = ukf.update_args(None, None, None, {"landmarks": lm}, R, 4)
    assert np.array_equal(Rd, [0.25, 0.09] * 2) and np.array_equal(pos, [1.0, 2.0, 3.0, 4.0])
    Rd, _ = ukf.update_args(2.0, None, None, {"landmarks": lm}, R, 4)    # scalar R: eye * R, this call only
    assert np.array_equal(Rd, [2.0] * 4)
    Rn = R.copy()
    Rn[0, 1] = Rn[1, 0] = 0.01
    with pytest.raises(ValueError, match="diagonal"):
        ukf.update_args(None, None, None, {"landmarks": lm}, Rn, 4)       # non-diagonal R is not dropped
    with pytest.raises(ValueError):
        ukf.update_args(np.eye(3), None, None, {"landmarks": lm}, R, 4)
    with pytest.raises(TypeError):
        ukf.update_args(None, None, None, {}, R, 4)                       # transfer_function needs landmarks
    with pytest.raises(ValueError):
        ukf.update_args(None, None, None, {"landmarks": lm[:1]}, R, 4)
    from lidar_slam_amd import landmarking as lmk
    L = lmk.Landmark(0.5, 3.0, 7, 10.0, 20.0, 50.0, 28.0)
    _, pos = ukf.update_args(None, None, None, {"landmarks": [L, L]}, R, 4)   # Landmark.get_pos()
    assert np.array_equal(pos, [10.0, 20.0, 10.0, 20.0])


@pytest.mark.gpu
def test_system_ukf_keeps_filterpy_state():
    """filterpy keeps sigmas_f from predict: update uses them with the CURRENT x and P, so
    predict -> set x -> update, update twice, and update before any predict (sigmas_f = 0)
    follow filterpy's state handling.  The drop-in and oracle/ukf.py's UKF (the same state
    handling in NumPy) are both held to the 50-digit evaluation of that step on the same
    cached sigma points (oracle/ukf_exact.step(sigmas=...)): x, y, theta at 1e-5.  P at 1e-3
    relative: with x moved by d off the sigma points' mean, P - K S K^T cancels terms scaled
    by the ~1e8 weights, and float64 P errors grow as ~1e-3 |d| (measured on the oracle: 3e-4
    at this d, 3e-3 at ten times it).  The two semantics differ far beyond those bounds (the
    re-drawn sigma points move theta by ~8e-3 here), so the test tells them apart."""
    from oracle import ukf as oukf
    from oracle import ukf_exact as ux
    rng = np.random.default_rng(7)
    lm = [tuple(p) for p in rng.uniform(-3000, 3000, (8, 2))]
    x0 = np.array([1000.0, 800.0, 0.3])
    z = oukf.transfer_function(x0, lm) + rng.normal(0, 0.2, 16)
    Rd = np.array([0.25, 0.09] * 8)
    d = np.array([0.3, -0.2, 0.001])

    def both():
        sysm = systemClass.System([])
        f = oukf.UKF(8)
        sysm.ukf.x, f.x = x0.copy(), x0.copy()
        return sysm.ukf, f

    def update_both(g, f):
        xe, Pe = ux.to_float(*ux.step(g.x, g.P, (0, 0), z, np.array(lm), Rd, predict=False, sigmas=g.sigmas_f))
        xr, Pr = ux.to_float(*ux.step(g.x, g.P, (0, 0), z, np.array(lm), Rd, predict=False))  # re-drawn
        assert ux.component_errors(xr[None], Pr[None], xe[None], Pe[None])["theta_abs"] > 1e-3
        g.update(z, landmarks=lm)
        f.update(z, lm)
        for h in (g, f):
            err = ux.component_errors(h.x[None], h.P[None], xe[None], Pe[None])
            assert max(err["x_rel"], err["y_rel"], err["theta_abs"]) <= 1e-5, (type(h).__module__, err)
            assert err["P_rel"] <= 1e-3, (type(h).__module__, err)

    g, f = both()                                   # predict -> set x -> update
    g.predict(u=[2.0, 2.5])
    f.predict(np.array([2.0, 2.5]))
    assert np.allclose(g.sigmas_f, f.sigmas_f, rtol=1e-9, atol=1e-9)
    f.sigmas_f = g.sigmas_f.copy()                  # the same cached points on both sides
    g.x = f.x = f.x + d
    g.P = f.P = g.P.copy()
    update_both(g, f)
    update_both(g, f)                               # a second update reuses the same sigmas_f
    g, f = both()                                   # update first: filterpy's zero sigmas_f
    assert not np.any(g.sigmas_f)
    g.P = f.P = np.diag([4.0, 4.0, 0.01])
    g.update(z, landmarks=lm)
    f.update(z, lm)
    assert np.array_equal(g.x, x0) and np.array_equal(f.x, x0)   # K = 0: every sigma maps to one point
