"""Generate the golden vectors for the RANSAC/landmark hot path FROM THE REFERENCE.

Run ONLY in the build container, with the interpreter that can import the
reference and its third-party dependency (scikit-image 0.18.3, numpy 1.26.4):

    /opt/conda/bin/python3.9 tests/golden/make_golden.py

It imports ``/root/reference/ransac_functions.py`` and ``landmarking.py``
unmodified (only the Qt-only ``mainWindow`` module is stubbed: its
``PyQt5.QtChart`` import is absent here, and ``ransac_functions.py:5`` only
uses ``time``/``ploting`` from it) and records, per RANSAC call, what the
reference computes.  Outputs are plain ``.npz`` data (no pickles) read by the
tests with ``np.load(allow_pickle=False)``.  Nothing here travels to the GPU
box except the ``.npz`` files.

Files written next to this script:
  mt_choice.npz   legacy MT19937 seeding / raw words / choice(N,2,replace=False)
  batch256.npz    256 scans, lean: per-chunk results + pre-call lists (points regenerated)
  batch.npz       24 independent scans, np.random.seed(s) per scan, fresh
                  landmark list per scan (the batched API's semantics)
  live.npz        one chained run: ONE np.random.seed, ONE landmark list over
                  14 scans (exactly SLAM.py's live semantics, check_ransac loop)
  edge.npz        crafted single ransac calls: early stop, vertical line,
                  duplicates, N=3, N=2 error, thr=0, 2-inlier refit, NaN, T=0
  assoc.npz       crafted landmark lists: skip-after-remove quirk, direct match
  big.npz         C5-shaped calls: 4096 points, 2048 trials
  known.npz       skimage LineModelND known answers (fit.py:48-62, test_fit.py:92-101)
"""
import os
import sys
import time
import types
import warnings

sys.path.insert(0, os.path.dirname(os.path.abspath(__file__)))
import blaspin  # noqa: E402  (pins OPENBLAS_CORETYPE; must precede numpy)
import numpy as np  # noqa: E402

REF = "/root/reference"
HERE = os.path.dirname(os.path.abspath(__file__))
OUT = os.environ.get("LSLAM_GOLDEN_OUT", HERE)  # the dispatch census writes elsewhere
sys.path.insert(0, REF)
sys.path.insert(0, os.path.abspath(os.path.join(HERE, "..", "..")))

_stub = types.ModuleType("mainWindow")
_stub.time = time
_stub.ploting = lambda *a, **k: None
sys.modules["mainWindow"] = _stub

import ransac_functions as rf  # noqa: E402  (reference, unmodified)
import landmarking as lmk  # noqa: E402
from skimage.measure import LineModelND, ransac  # noqa: E402
import skimage  # noqa: E402

from lidar_slam_amd import synth  # noqa: E402

assert skimage.__version__ == "0.18.3", skimage.__version__
warnings.simplefilter("ignore")
THR = rf.THRESHOLD
T = rf.MAX_TRIALS


def _silent(fn, *a, **k):
    import io
    import contextlib
    with contextlib.redirect_stdout(io.StringIO()):
        return fn(*a, **k)


def replay_draws(state, n, ndraw):
    rs = np.random.RandomState()
    rs.set_state(state)
    out = []
    states = []
    for _ in range(ndraw):
        out.append(rs.choice(n, 2, replace=False))
        states.append(rs.get_state())
    return np.asarray(out, dtype=np.int32), states


def same_state(a, b):
    return a[0] == b[0] and np.array_equal(a[1], b[1]) and a[2] == b[2]


def trial_stats(data, draws, ntrial, thr):
    cnt = np.zeros(ntrial, np.int32)
    sm = np.zeros(ntrial, np.float64)
    for t in range(ntrial):
        m = LineModelND()
        m.estimate(data[draws[t]])
        r = np.abs(m.residuals(data))
        cnt[t] = np.sum(r < thr)
        sm[t] = np.sum(r ** 2)
    return cnt, sm


def best_trial(cnt, sm):
    """skimage fit.py:850-869 selection (stop_probability=1, stop_residuals_sum=0)."""
    bc, bs, bt = 0, np.inf, -1
    for t in range(len(cnt)):
        if cnt[t] > bc or (cnt[t] == bc and sm[t] < bs):
            bc, bs, bt = cnt[t], sm[t], t
            if bs <= 0:
                return bt, t
    return bt, len(cnt) - 1


class Recorder:
    """Accumulates per-call records into flat arrays."""

    def __init__(self):
        self.r = {k: [] for k in (
            "draws", "draws_used", "trial_cnt", "trial_sum", "best_trial", "stop_trial",
            "origin", "direction", "a", "b", "tip", "n_inl", "new_landmark",
            "state_before_key", "state_before_pos", "state_after_key", "state_after_pos",
            "landmark_number")}
        self.mask = []
        self.qx, self.qy, self.q_off = [], [], [0]
        self.lm_off = [0]
        self.lm = {k: [] for k in ("id", "life", "a", "b", "pos", "end")}
        self.lm_in_off = [0]
        self.lm_in = {k: [] for k in ("id", "life", "a", "b", "pos", "end")}

    @staticmethod
    def _dump_list(dst, off, lst):
        for L in lst:
            dst["id"].append(L.id)
            dst["life"].append(L.life)
            dst["a"].append(L.a)
            dst["b"].append(L.b)
            dst["pos"].append(np.asarray(L.pos, np.float64))
            dst["end"].append(np.asarray(L.end, np.float64))
        off.append(off[-1] + len(lst))

    def call(self, data, landmark_number, landmarks):
        """One check_ransac iteration (ransac_functions.py:73-78) on `data`."""
        n = data.shape[0]
        st0 = np.random.get_state()
        draws, states = replay_draws(st0, n, T + 1)
        cnt, sm = trial_stats(data, draws, T, THR)
        bt, stop = best_trial(cnt, sm)
        used = stop + 2
        # the mask exactly as skimage computes it inside landmark_extraction
        np.random.set_state(st0)
        model, inl = ransac(data, LineModelND, min_samples=rf.MIN_SAMPLES,
                            residual_threshold=THR, max_trials=T)
        st_a = np.random.get_state()
        assert same_state(st_a, states[used - 1]), "draw accounting mismatch"
        self._dump_list(self.lm_in, self.lm_in_off, landmarks)
        # the reference call itself, from the same RNG state
        np.random.set_state(st0)
        q, fitted, new = _silent(rf.landmark_extraction, [data.tolist()], landmark_number, landmarks)
        st1 = np.random.get_state()
        assert same_state(st1, st_a)
        assert np.array_equal(model.params[0], fitted.pos)
        if new:
            landmarks.append(fitted)  # ransac_functions.py:75-76
        r = self.r
        r["draws"].append(draws)
        r["draws_used"].append(used)
        r["trial_cnt"].append(cnt)
        r["trial_sum"].append(sm)
        r["best_trial"].append(bt)
        r["stop_trial"].append(stop)
        r["origin"].append(np.asarray(model.params[0], np.float64))
        r["direction"].append(np.asarray(model.params[1], np.float64))
        r["a"].append(fitted.a)
        r["b"].append(fitted.b)
        r["tip"].append(np.asarray(fitted.end, np.float64))
        r["n_inl"].append(int(inl.sum()))
        r["new_landmark"].append(bool(new))
        r["state_before_key"].append(st0[1].copy())
        r["state_before_pos"].append(st0[2])
        r["state_after_key"].append(st1[1].copy())
        r["state_after_pos"].append(st1[2])
        r["landmark_number"].append(landmark_number)
        self.mask.append(inl.astype(np.uint8))
        self.qx.extend(p.x() for p in q)
        self.qy.extend(p.y() for p in q)
        self.q_off.append(len(self.qx))
        self._dump_list(self.lm, self.lm_off, landmarks)

    def arrays(self, prefix=""):
        out = {}
        r = self.r
        out["draws"] = np.asarray(r["draws"], np.int32)
        for k in ("draws_used", "best_trial", "stop_trial", "n_inl", "state_before_pos",
                  "state_after_pos", "landmark_number"):
            out[k] = np.asarray(r[k], np.int32)
        out["trial_cnt"] = np.asarray(r["trial_cnt"], np.int32)
        out["trial_sum"] = np.asarray(r["trial_sum"], np.float64)
        for k in ("origin", "direction", "tip"):
            out[k] = np.asarray(r[k], np.float64).reshape(-1, 2)
        out["a"] = np.asarray(r["a"], np.float64)
        out["b"] = np.asarray(r["b"], np.float64)
        out["new_landmark"] = np.asarray(r["new_landmark"], np.uint8)
        out["state_before_key"] = np.asarray(r["state_before_key"], np.uint32)
        out["state_after_key"] = np.asarray(r["state_after_key"], np.uint32)
        out["mask"] = np.concatenate(self.mask).astype(np.uint8)
        out["q_x"] = np.asarray(self.qx, np.float64)
        out["q_y"] = np.asarray(self.qy, np.float64)
        out["q_off"] = np.asarray(self.q_off, np.int32)
        for name, d, off in (("lm", self.lm, self.lm_off), ("lm_in", self.lm_in, self.lm_in_off)):
            out[name + "_off"] = np.asarray(off, np.int32)
            out[name + "_id"] = np.asarray(d["id"], np.int32)
            out[name + "_life"] = np.asarray(d["life"], np.int32)
            out[name + "_a"] = np.asarray(d["a"], np.float64)
            out[name + "_b"] = np.asarray(d["b"], np.float64)
            out[name + "_pos"] = np.asarray(d["pos"], np.float64).reshape(-1, 2)
            out[name + "_end"] = np.asarray(d["end"], np.float64).reshape(-1, 2)
        return {prefix + k: v for k, v in out.items()}


def gen_batch(n_scans=24):
    ids = list(range(n_scans))
    b = synth.make_batch(ids)
    rec = Recorder()
    for s in ids:
        np.random.seed(s)
        landmarks = []
        for c in range(b["scan_chunk_off"][s], b["scan_chunk_off"][s + 1]):
            p0, p1 = b["chunk_pt_off"][c], b["chunk_pt_off"][c + 1]
            rec.call(b["xy"][p0:p1], c - b["scan_chunk_off"][s], landmarks)
    out = rec.arrays()
    out.update(xy=b["xy"], scan_chunk_off=b["scan_chunk_off"], chunk_pt_off=b["chunk_pt_off"],
               seeds=np.asarray(ids, np.uint32))
    blaspin.save_npz(os.path.join(OUT, "batch.npz"), **out)
    print("batch.npz", out["xy"].shape, len(out["a"]), "chunks")


def gen_batch256(n_scans=256):
    """SURVEY §8(c)'s ~256-scan plan, kept lean (~1 MB): the points are NOT stored (synth's
    generator regenerates them bit for bit under numpy 1.26 and 2.x; their sha256 is), nor
    the draws or MT states (batch.npz / mt_choice.npz pin those; here a hash of each scan's
    final state).  Per chunk: mask, per-trial counts, winner, draws used, origin, direction,
    a, b, tip, new-landmark flag, and the pre-call landmark list with every field (the
    association decisions, is_equal at landmarking.py:66-77, are replayed from it)."""
    import hashlib
    ids = list(range(n_scans))
    b = synth.make_batch(ids)
    r = {k: [] for k in ("mask", "trial_cnt", "best_trial", "draws_used", "n_inl", "origin", "direction", "a", "b",
                         "tip", "new_landmark")}
    lin = {k: [] for k in ("id", "life", "a", "b", "pos", "end")}
    lin_off, lout_id, lout_life, lout_off = [0], [], [], [0]
    state_hash = []
    for s in ids:
        np.random.seed(s)
        landmarks = []
        for c in range(b["scan_chunk_off"][s], b["scan_chunk_off"][s + 1]):
            data = b["xy"][b["chunk_pt_off"][c]:b["chunk_pt_off"][c + 1]]
            st0 = np.random.get_state()
            draws, _ = replay_draws(st0, data.shape[0], T + 1)
            cnt, sm = trial_stats(data, draws, T, THR)
            bt, stop = best_trial(cnt, sm)
            np.random.set_state(st0)
            model, inl = ransac(data, LineModelND, min_samples=rf.MIN_SAMPLES, residual_threshold=THR, max_trials=T)
            Recorder._dump_list(lin, lin_off, landmarks)
            np.random.set_state(st0)
            q, fitted, new = _silent(rf.landmark_extraction, [data.tolist()], c - b["scan_chunk_off"][s], landmarks)
            if new:
                landmarks.append(fitted)
            r["mask"].append(inl.astype(np.uint8))
            r["trial_cnt"].append(cnt.astype(np.uint8))
            r["best_trial"].append(bt)
            r["draws_used"].append(stop + 2)
            r["n_inl"].append(int(inl.sum()))
            r["origin"].append(np.asarray(model.params[0], np.float64))
            r["direction"].append(np.asarray(model.params[1], np.float64))
            r["a"].append(fitted.a)
            r["b"].append(fitted.b)
            r["tip"].append(np.asarray(fitted.end, np.float64))
            r["new_landmark"].append(bool(new))
            lout_id.extend(L.id for L in landmarks)
            lout_life.extend(L.life for L in landmarks)
            lout_off.append(len(lout_id))
        st = np.random.get_state()
        state_hash.append(int.from_bytes(hashlib.sha256(st[1].tobytes() + np.int32(st[2]).tobytes()).digest()[:8],
                                         "little"))
    out = dict(
        n_scans=np.int32(n_scans),
        xy_sha256=np.frombuffer(hashlib.sha256(b["xy"].tobytes()).digest(), np.uint8),
        scan_chunk_off=b["scan_chunk_off"], chunk_pt_off=b["chunk_pt_off"], seeds=np.asarray(ids, np.uint32),
        mask=np.concatenate(r["mask"]), trial_cnt=np.asarray(r["trial_cnt"], np.uint8),
        best_trial=np.asarray(r["best_trial"], np.int32), draws_used=np.asarray(r["draws_used"], np.int32),
        n_inl=np.asarray(r["n_inl"], np.int32), origin=np.asarray(r["origin"]), direction=np.asarray(r["direction"]),
        a=np.asarray(r["a"]), b=np.asarray(r["b"]), tip=np.asarray(r["tip"]),
        new_landmark=np.asarray(r["new_landmark"], np.uint8),
        lm_in_off=np.asarray(lin_off, np.int32), lm_in_id=np.asarray(lin["id"], np.int32),
        lm_in_life=np.asarray(lin["life"], np.int32), lm_in_a=np.asarray(lin["a"], np.float64),
        lm_in_b=np.asarray(lin["b"], np.float64), lm_in_pos=np.asarray(lin["pos"], np.float64).reshape(-1, 2),
        lm_in_end=np.asarray(lin["end"], np.float64).reshape(-1, 2),
        lm_out_off=np.asarray(lout_off, np.int32), lm_out_id=np.asarray(lout_id, np.int32),
        lm_out_life=np.asarray(lout_life, np.int32),
        state_after_hash=np.asarray(state_hash, np.uint64))
    blaspin.save_npz(os.path.join(OUT, "batch256.npz"), **out)
    print("batch256.npz", len(out["a"]), "chunks,", os.path.getsize(os.path.join(OUT, "batch256.npz")), "bytes;",
          "matches:", int((out["new_landmark"] == 0).sum()))


def gen_live(n_scans=14, seed=20240611):
    """check_ransac over a chained run: one global RNG stream, one landmark list.
    Scans alternate between a few fixed poses so landmarks get re-observed
    (matches, resets) as well as aged out (removals, skip quirk)."""
    pose_ids = [100, 100, 101, 100, 102, 100, 101, 103, 100, 104, 105, 106, 107, 100]
    b = synth.make_batch(pose_ids[:n_scans])
    np.random.seed(seed)
    rec = Recorder()
    landmarks = []
    number = 0
    for s in range(n_scans):
        for c in range(b["scan_chunk_off"][s], b["scan_chunk_off"][s + 1]):
            p0, p1 = b["chunk_pt_off"][c], b["chunk_pt_off"][c + 1]
            rec.call(b["xy"][p0:p1], number, landmarks)
            number += 1
    out = rec.arrays()
    out.update(xy=b["xy"], scan_chunk_off=b["scan_chunk_off"], chunk_pt_off=b["chunk_pt_off"],
               seed=np.asarray([seed], np.uint32))
    blaspin.save_npz(os.path.join(OUT, "live.npz"), **out)
    print("live.npz", len(out["a"]), "chunks; matches:", int((out["new_landmark"] == 0).sum()),
          "max list", int(np.diff(out["lm_off"]).max()))


def gen_mt_choice():
    seeds = np.array([0, 1, 12345, 2 ** 32 - 1, 20240611], np.uint32)
    ns = np.array([3, 4, 5, 20, 100, 129, 720, 4096], np.int32)
    ndraw = 40
    keys = []
    words = []
    draws = np.zeros((len(seeds), len(ns), ndraw, 2), np.int32)
    after_key = np.zeros((len(seeds), len(ns), 624), np.uint32)
    after_pos = np.zeros((len(seeds), len(ns)), np.int32)
    for i, s in enumerate(seeds):
        rs = np.random.RandomState(int(s))
        st = rs.get_state()
        keys.append(st[1].copy())
        assert st[2] == 624
        words.append(rs.randint(0, 2 ** 32, size=2000, dtype=np.uint64).astype(np.uint32))
        for j, n in enumerate(ns):
            rs = np.random.RandomState(int(s))
            for k in range(ndraw):
                draws[i, j, k] = rs.choice(int(n), 2, replace=False)
            st = rs.get_state()
            after_key[i, j] = st[1]
            after_pos[i, j] = st[2]
    blaspin.save_npz(os.path.join(OUT, "mt_choice.npz"), seeds=seeds, ns=ns,
                        init_key=np.asarray(keys, np.uint32), words=np.asarray(words, np.uint32),
                        draws=draws, after_key=after_key, after_pos=after_pos)
    print("mt_choice.npz")


def _one_call(data, thr, trials, seed):
    """A single skimage ransac call as ransac_functions.py:23-24 makes it,
    recording error type, mask, params, draws used, state after."""
    np.random.seed(seed)
    st0 = np.random.get_state()
    err = 0
    try:
        model, inl = ransac(data, LineModelND, min_samples=2, residual_threshold=thr,
                            max_trials=trials)
    except ValueError:
        err, model, inl = 1, None, None
    st1 = np.random.get_state()
    n = data.shape[0]
    ndraw = 0
    if n > 2:
        _, states = replay_draws(st0, n, trials + 1)
        for k, stk in enumerate(states):
            if same_state(stk, st1):
                ndraw = k + 1
                break
        else:
            raise AssertionError("state not reached")
    else:
        assert same_state(st0, st1)
    if err == 0 and model is None:
        err = 2
    if err == 0:
        a = model.params[1][1] / model.params[1][0]
        b = model.params[0][1] - a * model.params[0][0]
        params = np.array([*model.params[0], *model.params[1], a, b], np.float64)
        mask = inl.astype(np.uint8)
    else:
        params = np.full(6, np.nan)
        mask = np.zeros(n, np.uint8)
    return err, mask, params, ndraw, st1


def gen_edge():
    cases = []
    rng = np.random.default_rng(7)
    xs = np.arange(40, dtype=np.float64) * 25.0
    cases.append(("horizontal_early_stop", np.stack([xs, np.full(40, 5.0)], 1), 20.0, 100))
    cases.append(("vertical_early_stop", np.stack([np.full(40, 7.0), xs], 1), 20.0, 100))
    cases.append(("duplicates", np.tile([[3.0, 4.0]], (12, 1)), 20.0, 100))
    cases.append(("n3", rng.normal(0, 30, (3, 2)), 20.0, 100))
    cases.append(("n2_error", rng.normal(0, 30, (2, 2)), 20.0, 100))
    cases.append(("thr0_no_inliers", rng.normal(0, 300, (10, 2)), 0.0, 100))
    cases.append(("two_inlier_refit", rng.uniform(-1000, 1000, (30, 2)), 1e-9, 100))
    pts = rng.normal(0, 10, (50, 2)) + np.stack([np.linspace(0, 900, 50), np.linspace(0, 300, 50)], 1)
    pts2 = pts.copy()
    pts2[17] = [np.nan, 1.0]
    cases.append(("nan_point", pts2, 20.0, 100))
    cases.append(("t0", pts, 20.0, 0))
    cases.append(("t1", pts, 20.0, 1))
    cases.append(("t250", pts, 20.0, 250))
    cases.append(("thr_tiny_line", pts, 1.0, 100))
    # near-threshold residuals: points at distance ~20 from a horizontal line
    pts3 = np.stack([np.arange(64.0) * 10, np.where(np.arange(64) % 3 == 0, 20.0, 0.0)], 1)
    pts3[::5, 1] = 19.999999999999996
    cases.append(("near_threshold", pts3, 20.0, 100))
    names, offs, xy, thr, trials, seeds = [], [0], [], [], [], []
    err, mask, params, ndraw, keys, poss = [], [], [], [], [], []
    for k, (name, data, th, tr) in enumerate(cases):
        seed = 1000 + k
        e, m, p, nd, st = _one_call(np.ascontiguousarray(data, np.float64), th, tr, seed)
        names.append(name)
        xy.append(data)
        offs.append(offs[-1] + len(data))
        thr.append(th)
        trials.append(tr)
        seeds.append(seed)
        err.append(e)
        mask.append(m)
        params.append(p)
        ndraw.append(nd)
        keys.append(st[1])
        poss.append(st[2])
    blaspin.save_npz(
        os.path.join(OUT, "edge.npz"), names=np.asarray(names), xy=np.concatenate(xy).astype(np.float64),
        off=np.asarray(offs, np.int32), thr=np.asarray(thr), trials=np.asarray(trials, np.int32),
        seeds=np.asarray(seeds, np.uint32), err=np.asarray(err, np.int32),
        mask=np.concatenate(mask), params=np.asarray(params), ndraw=np.asarray(ndraw, np.int32),
        after_key=np.asarray(keys, np.uint32), after_pos=np.asarray(poss, np.int32))
    print("edge.npz", dict(zip(names, err)), dict(zip(names, ndraw)))
    # a chained sequence across an early stop: normal, collinear, normal
    np.random.seed(77)
    seq = [pts, cases[0][1], pts + 3.0]
    rec = Recorder()
    lst = []
    for i, d in enumerate(seq):
        rec.call(np.ascontiguousarray(d), i, lst)
    out = rec.arrays()
    out.update(xy=np.concatenate(seq), chunk_pt_off=np.cumsum([0] + [len(d) for d in seq]).astype(np.int32),
               scan_chunk_off=np.array([0, 3], np.int32), seed=np.array([77], np.uint32))
    blaspin.save_npz(os.path.join(OUT, "edge_chain.npz"), **out)
    print("edge_chain.npz stop trials", out["stop_trial"], "used", out["draws_used"])


def gen_assoc():
    """Crafted landmark lists around one fixed chunk (a clean line).

    Returns, per case, the list before/after and the reference outputs."""
    xs = np.linspace(0.0, 990.0, 100)
    data = np.stack([xs, 0.5 * xs + 100.0], 1) + np.random.default_rng(3).normal(0, 2.0, (100, 2))
    np.random.seed(5)
    st = np.random.get_state()
    model, inl = ransac(data, LineModelND, min_samples=2, residual_threshold=THR, max_trials=T)
    a = model.params[1][1] / model.params[1][0]
    b = model.params[0][1] - a * model.params[0][0]
    pos = model.params[0]
    tipx = data[inl, 0][-1]
    end = np.array([tipx, tipx * a + b])

    def L(id_, da=0.0, db=0.0, life=40, pos_=None, end_=None, far=False):
        p = pos if pos_ is None else pos_
        e = end if end_ is None else end_
        if far:
            p = p + 5000.0
            e = e + 5000.0
        o = lmk.Landmark(a + da, b + db, id_, p[0], p[1], e[0], e[1])
        o.life = life
        return o

    # a matching landmark needs end_i within 100 of pos_new (or pos_i within 100 of end_new)
    match_pos = end.copy()  # pos of an old landmark placed at our tip -> ||pos_i - end_new|| = 0
    cases = {
        "empty": [],
        "direct_match_first": [L(0, pos_=match_pos)],
        "match_after_nonmatches": [L(0, far=True), L(1, far=True, life=3), L(2, pos_=match_pos)],
        "skip_after_remove": [L(0, far=True, life=1), L(1, pos_=match_pos), L(2, far=True)],
        "double_remove": [L(0, far=True, life=1), L(1, far=True, life=1), L(2, far=True, life=1),
                          L(3, far=True, life=5), L(4, pos_=match_pos)],
        "remove_last": [L(0, far=True, life=2), L(1, far=True, life=1)],
        # near (not on) the tolerance edges: the final direction comes from LAPACK
        # dgesdd in the reference, so decisions exactly ON an edge depend on its
        # last bits; these sit 1e-12 away, far beyond that rounding
        "a_tol_edge": [L(0, da=0.1 + 1e-12, pos_=match_pos), L(1, da=0.1 - 1e-12, pos_=match_pos)],
        "b_tol_edge": [L(0, db=10.0 + 1e-9, pos_=match_pos), L(1, db=-10.0 + 1e-9, pos_=match_pos)],
        "life0_in_list": [L(0, far=True, life=0), L(1, far=True), L(2, pos_=match_pos)],
        "no_match_all_decrement": [L(i, far=True, life=40 - i) for i in range(6)],
    }
    names, lin_off, lout_off = [], [0], [0]
    fields = ("id", "life", "a", "b", "pos", "end")
    lin = {k: [] for k in fields}
    lout = {k: [] for k in fields}
    qx, qy, qoff, new = [], [], [0], []
    for name, lst in cases.items():
        Recorder._dump_list(lin, lin_off, lst)
        np.random.set_state(st)
        q, fitted, nw = _silent(rf.landmark_extraction, [data.tolist()], 99, lst)
        if nw:
            lst.append(fitted)
        Recorder._dump_list(lout, lout_off, lst)
        qx.extend(p.x() for p in q)
        qy.extend(p.y() for p in q)
        qoff.append(len(qx))
        new.append(nw)
        names.append(name)
    out = dict(names=np.asarray(names), xy=data, seed=np.array([5], np.uint32),
               q_x=np.asarray(qx), q_y=np.asarray(qy), q_off=np.asarray(qoff, np.int32),
               new_landmark=np.asarray(new, np.uint8),
               fit=np.array([a, b, pos[0], pos[1], end[0], end[1]]))
    for nm, d, off in (("lm_in", lin, lin_off), ("lm_out", lout, lout_off)):
        out[nm + "_off"] = np.asarray(off, np.int32)
        out[nm + "_id"] = np.asarray(d["id"], np.int32)
        out[nm + "_life"] = np.asarray(d["life"], np.int32)
        out[nm + "_a"] = np.asarray(d["a"], np.float64)
        out[nm + "_b"] = np.asarray(d["b"], np.float64)
        out[nm + "_pos"] = np.asarray(d["pos"], np.float64).reshape(-1, 2)
        out[nm + "_end"] = np.asarray(d["end"], np.float64).reshape(-1, 2)
    blaspin.save_npz(os.path.join(OUT, "assoc.npz"), **out)
    print("assoc.npz", dict(zip(names, new)), np.diff(out["lm_out_off"]))


def gen_big(n_calls=2, n_pts=4096, trials=2048):
    xy_all, off, masks, params, ndraw, keys, poss, bests = [], [0], [], [], [], [], [], []
    for k in range(n_calls):
        th, d, _ = synth.scan_polar(500 + k, n_beams=n_pts, cfg=5)
        xy = synth.polar_to_xy_ref(th, d)
        seed = 500 + k
        e, m, p, nd, st = _one_call(xy, 20.0, trials, seed)
        assert e == 0
        xy_all.append(xy)
        off.append(off[-1] + n_pts)
        masks.append(m)
        params.append(p)
        ndraw.append(nd)
        keys.append(st[1])
        poss.append(st[2])
        np.random.seed(seed)
        draws, _ = replay_draws(np.random.get_state(), n_pts, trials + 1)
        cnt, sm = trial_stats(xy, draws, trials, 20.0)
        bt, _ = best_trial(cnt, sm)
        bests.append(bt)
        print("big", k, "inliers", m.sum(), "best", bt, "ties", int((cnt == cnt.max()).sum()))
    blaspin.save_npz(os.path.join(OUT, "big.npz"), xy=np.concatenate(xy_all), off=np.asarray(off, np.int32),
                        seeds=np.array([500 + k for k in range(n_calls)], np.uint32), trials=np.int32(trials),
                        mask=np.concatenate(masks), params=np.asarray(params), ndraw=np.asarray(ndraw, np.int32),
                        after_key=np.asarray(keys, np.uint32), after_pos=np.asarray(poss, np.int32),
                        best_trial=np.asarray(bests, np.int32))


def gen_known():
    x = np.linspace(1, 2, 25)
    y = 1.5 * x + 3
    lm = LineModelND()
    lm.estimate(np.stack([x, y], axis=-1))
    res_model = LineModelND()
    res_model.params = (np.array([0.0, 0.0]), np.array([0.0, 1.0]))
    res_pts = np.array([[0.0, 0.0], [0.0, 1.0], [10.0, 0.0], [-30.0, 5.0]])
    res = res_model.residuals(res_pts)
    blaspin.save_npz(os.path.join(OUT, "known.npz"), doc_xy=np.stack([x, y], -1),
                        doc_origin=lm.params[0], doc_direction=lm.params[1],
                        res_pts=res_pts, res_params=np.array([0.0, 0.0, 0.0, 1.0]), res=res)
    print("known.npz", lm.params, res)


if __name__ == "__main__":
    which = sys.argv[1:] or ["mt", "batch", "batch256", "live", "edge", "assoc", "big", "known"]
    t0 = time.time()
    if "mt" in which:
        gen_mt_choice()
    if "known" in which:
        gen_known()
    if "edge" in which:
        gen_edge()
    if "assoc" in which:
        gen_assoc()
    if "batch" in which:
        gen_batch()
    if "batch256" in which:
        gen_batch256()
    if "live" in which:
        gen_live()
    if "big" in which:
        gen_big()
    print("done in %.1fs" % (time.time() - t0))
