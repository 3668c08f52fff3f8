"""Drop-in for ``ransac_functions.py`` with the hot path on the GPU.

``landmark_extraction(pointsToBeFitted, landmarkNumber, landmarks)`` has the
reference's name, signature, return types and side effects
(ransac_functions.py:15-59):

* takes ``pointsToBeFitted[0]`` and clears the list (``:20-22``);
* runs skimage-semantics RANSAC (``:23-24``: min_samples=2, threshold 20,
  100 trials) on the HIP kernel, drawing hypotheses from - and advancing -
  numpy's GLOBAL legacy RandomState exactly as skimage does (the MT19937 state
  is read with ``np.random.get_state()``, advanced on the device, and written
  back with ``np.random.set_state``);
* computes a, b, the tip and the Landmark (``:25-31``), walks ``landmarks``
  (``:34-54``: life decrements, removals with the skip-after-remove quirk,
  life reset on a match) on the device and applies the walk to the caller's
  Landmark objects in place;
* returns ``(qPointsList, fittedLine, newLandmark)``; the caller appends
  ``fittedLine`` when ``newLandmark`` (``:75-76``) as before.

Error behaviour matches the reference: fewer than 3 points -> ValueError
(fit.py:798-799); no inliers -> RuntimeWarning-free ``warn`` + AttributeError
(``model_robust.params`` on None, ransac_functions.py:25); one final inlier ->
ValueError (fit.py:96-97).

``check_ransac`` and ``ransac_core`` keep the reference's thread/queue
plumbing (:63-120) around this landmark_extraction.
"""
from __future__ import annotations

import ctypes as C
import threading
import time
import warnings

import numpy as np

from . import _lib
from .device import Context
from .landmarking import LIFE, Landmark  # noqa: F401  (re-exported like the reference's `from landmarking import *`)
from .pipeline import LANDMARK_DTYPE, MODEL_DTYPE

THRESHOLD = 20    # ransac_functions.py:9
MAX_TRIALS = 100  # ransac_functions.py:10
MIN_SAMPLES = 2   # ransac_functions.py:11
MIN_POINTS = 100  # ransac_functions.py:12 (unused by the reference too)

VERBOSE = False   # the reference prints "ransacking..." etc. on every call; opt-in here

try:  # the GUI's point type; a minimal stand-in when PyQt5 is absent
    from PyQt5.QtCore import QPointF  # type: ignore
except Exception:  # pragma: no cover - depends on the host
    class QPointF:
        __slots__ = ("_x", "_y")

        def __init__(self, x=0.0, y=0.0):
            self._x, self._y = float(x), float(y)

        def x(self):
            return self._x

        def y(self):
            return self._y

        def __repr__(self):
            return "QPointF(%r, %r)" % (self._x, self._y)


class _Engine:
    """Per-thread device context + reusable buffers for single-chunk calls."""

    def __init__(self, device=0):
        self.ctx = Context(device)
        self.cap_pts = 0
        self.cap_lmk = 0
        self.bufs = {}

    def buf(self, name, nbytes):
        b = self.bufs.get(name)
        if b is None or b.nbytes < nbytes:
            b = self.ctx.empty(max(nbytes, 64), np.uint8)
            self.bufs[name] = b
        return b


_tls = threading.local()
DEVICE = 0


def _engine():
    e = getattr(_tls, "engine", None)
    if e is None:
        e = _Engine(DEVICE)
        _tls.engine = e
    return e


def _upload(e, name, arr):
    arr = np.ascontiguousarray(arr)
    b = e.buf(name, arr.nbytes)
    if arr.nbytes:
        _lib.check(e.ctx._L.lslam_h2d(e.ctx.handle, b.ptr, arr.ctypes.data_as(C.c_void_p), arr.nbytes), "h2d")
    return b


def _download(e, b, dtype, count):
    out = np.empty(count, dtype)
    if out.nbytes:
        _lib.check(e.ctx._L.lslam_d2h(e.ctx.handle, out.ctypes.data_as(C.c_void_p), b.ptr, out.nbytes), "d2h")
    return out


def run_chunk(data, landmarkNumber, landmarks, state=None, threshold=THRESHOLD, max_trials=MAX_TRIALS):
    """One landmark_extraction on the GPU without touching Python objects.

    data: (N,2) fp64.  landmarks: structured array (LANDMARK_DTYPE).
    state: (625,) uint32 legacy MT19937 key+pos (default: numpy's global state).
    Returns dict(mask, model, state, walk_life, lmk_out, lmk_count, y_proj).
    """
    e = _engine()
    data = np.ascontiguousarray(data, np.float64).reshape(-1, 2)
    N = data.shape[0]
    if state is None:
        st = np.random.get_state()
        state = np.concatenate([np.asarray(st[1], np.uint32), np.array([st[2]], np.uint32)])
    L = len(landmarks)
    cap = L + 1
    lm = np.zeros(cap, LANDMARK_DTYPE)
    lm[:L] = landmarks
    b = _lib.ScanBatch()
    b.n_scans, b.n_chunks, b.n_points = 1, 1, N
    b.max_chunk_points, b.max_scan_chunks, b.lmk_capacity = max(N, 1), 1, cap
    b.xy = _upload(e, "xy", data if N else np.zeros((1, 2))).addr
    b.scan_chunk_off = _upload(e, "sco", np.array([0, 1], np.int32)).addr
    b.chunk_pt_off = _upload(e, "cpo", np.array([0, N], np.int32)).addr
    b.mt_state_in = _upload(e, "st_in", np.ascontiguousarray(state, np.uint32)).addr
    b.mt_state_out = e.buf("st_out", 625 * 4).addr
    b.id_base = _upload(e, "idb", np.array([landmarkNumber], np.int32)).addr
    b.landmarks = _upload(e, "lmk", lm).addr
    b.lmk_count = _upload(e, "lmkc", np.array([L], np.int32)).addr
    b.lmk_walk = e.buf("walk", 4 * cap).addr
    b.inlier_mask = e.buf("mask", max(N, 1)).addr
    b.models = e.buf("models", MODEL_DTYPE.itemsize).addr
    b.y_proj = e.buf("yproj", 8 * max(N, 1)).addr
    p = _lib.ransac_params(residual_threshold=float(threshold), max_trials=int(max_trials))
    _lib.check(e.ctx._L.lslam_scan_pipeline(e.ctx.handle, C.byref(b), C.byref(p), None), "lslam_scan_pipeline")
    out = {
        "mask": _download(e, e.bufs["mask"], np.uint8, N).astype(bool),
        "model": _download(e, e.bufs["models"], MODEL_DTYPE, 1)[0],
        "state": _download(e, e.bufs["st_out"], np.uint32, 625),
        "walk_life": _download(e, e.bufs["walk"], np.int32, L),
        "lmk_out": _download(e, e.bufs["lmk"], LANDMARK_DTYPE, cap),
        "lmk_count": int(_download(e, e.bufs["lmkc"], np.int32, 1)[0]),
        "y_proj": _download(e, e.bufs["yproj"], np.float64, N),
    }
    e.ctx.sync()
    return out


def _as_records(landmarks):
    rec = np.zeros(len(landmarks), LANDMARK_DTYPE)
    for i, L in enumerate(landmarks):
        rec[i] = (L.a, L.b, L.pos[0], L.pos[1], L.end[0], L.end[1], L.id, L.life)
    return rec


def landmark_extraction(pointsToBeFitted, landmarkNumber, landmarks):
    """ransac_functions.py:15-59 on the GPU (see module docstring)."""
    data = np.array(pointsToBeFitted[0][:])
    del pointsToBeFitted[:]
    data = np.asarray(data, np.float64)
    if data.ndim != 2 or data.shape[1] != 2:
        raise ValueError("Input data must have shape (N, 2).")
    st = np.random.get_state()
    r = run_chunk(data, landmarkNumber, _as_records(landmarks))
    # the stream advanced exactly as skimage's choice() calls would have
    np.random.set_state((st[0], r["state"][:624].copy(), int(r["state"][624]), st[3], st[4]))
    m = r["model"]
    flags = int(m["flags"])
    if flags & _lib.N_TOO_SMALL:
        raise ValueError("`min_samples` must be in range (0, <number-of-samples>)")
    if flags & _lib.NO_INLIERS:
        warnings.warn("No inliers found. Model not fitted")
        raise AttributeError("'NoneType' object has no attribute 'params'")
    if flags & _lib.EST_FAIL:
        raise ValueError("At least 2 input points needed.")
    a, b = float(m["a"]), float(m["b"])
    fittedLine = Landmark(np.float64(a), np.float64(b), landmarkNumber, np.float64(m["ox"]), np.float64(m["oy"]),
                          np.float64(m["tip_x"]), np.float64(m["tip_y"]))
    if VERBOSE:
        print("ransacking...")
    # apply the device's association walk to the caller's Landmark objects
    walk = r["walk_life"]
    survivors = []
    for i, L in enumerate(list(landmarks)):
        L.life = int(walk[i])
        if L.life == 0:
            if VERBOSE:
                print("Excluded landmark: {}".format(L))
        else:
            survivors.append(L)
    landmarks[:] = survivors
    newLandmark = not (flags & _lib.MATCHED)
    if newLandmark and VERBOSE and len(walk):
        print("New landmark found! Landmarks: {}".format(len(landmarks)))
    mask = r["mask"]
    xBase = data[mask, 0]
    yBase = r["y_proj"][mask]
    qPointsList = [QPointF(xBase[i], yBase[i]) for i in range(xBase.shape[0])]
    return qPointsList, fittedLine, newLandmark


def check_ransac(pairInliers, tempPoints, allPoints, pointsToBeFitted, landmarks, threadEvent):
    """ransac_functions.py:63-93 (worker-thread loop) around the GPU landmark_extraction."""
    inliersList = list()
    landmarkNumber = 0
    while True:
        if pointsToBeFitted != []:
            if pointsToBeFitted[0] != 0:
                tempList, extractedLandmark, newLandmark = landmark_extraction(pointsToBeFitted, landmarkNumber,
                                                                               landmarks)
                inliersList.append(tempList)
                if newLandmark:
                    landmarks.append(extractedLandmark)
                landmarkNumber += 1
            elif inliersList != []:
                pairInliers.append(np.concatenate(inliersList.copy(), axis=0))
                allPoints.append(np.concatenate(tempPoints.copy(), axis=0))
                threadEvent.set()
                del inliersList[:]
                del pointsToBeFitted[:]
                del tempPoints[:]
            else:
                del pointsToBeFitted[:]
        else:
            time.sleep(0)  # yield the GIL (the reference spins)


def ransac_core(rawPoints):
    """ransac_functions.py:97-120: queue drain + worker + GUI threads (GUI = reference's mainWindow)."""
    from mainWindow import ploting  # the reference GUI module, untouched
    pairInliers, pointsToBeFitted, allPoints, tempPoints = [], [], [], []
    landmarks = list()
    threadEvent = threading.Event()
    threading.Thread(target=check_ransac, args=(pairInliers, tempPoints, allPoints, pointsToBeFitted, landmarks,
                                                threadEvent)).start()
    threading.Thread(target=ploting, args=(pairInliers, allPoints, threadEvent)).start()
    try:
        while True:
            time.sleep(0.000005)
            temp = rawPoints.get(True)
            pointsToBeFitted.append(temp)
            if temp != 0:
                tempPoints.append([QPointF(point[0], point[1]) for point in temp])
    except KeyboardInterrupt:
        pass


# ---------------------------------------------------------------------------
# Per-revolution dispatcher: one device launch per
# revolution instead of one landmark_extraction per chunk, no busy spin, and
# QPointF objects made only when the GUI slices a revolution's points.
# ---------------------------------------------------------------------------

class LazyPoints:
    """A revolution's points as float64 arrays; ``p[:]`` / iteration build the
    QPointF list the GUI's QScatterSeries.append/replace take (mainWindow.py:103-109),
    so revolutions the GUI never displays cost no Python objects."""

    __slots__ = ("x", "y")

    def __init__(self, x, y):
        self.x = np.ascontiguousarray(x, np.float64)
        self.y = np.ascontiguousarray(y, np.float64)

    def __len__(self):
        return int(self.x.shape[0])

    def __getitem__(self, k):
        if isinstance(k, slice):
            xs, ys = self.x[k].tolist(), self.y[k].tolist()
            return [QPointF(a, b) for a, b in zip(xs, ys)]
        return QPointF(float(self.x[k]), float(self.y[k]))

    def __iter__(self):
        return iter(self[:])

    def to_numpy(self):
        return np.stack([self.x, self.y], 1)


def run_revolution(chunks, landmarkNumber, landmarks, state=None, threshold=THRESHOLD, max_trials=MAX_TRIALS):
    """All chunks of one revolution in ONE lslam_scan_pipeline call: one "scan"
    whose chunks chain the MT19937 stream and walk one landmark list, exactly
    as check_ransac's sequence of landmark_extraction calls does
    (ransac_functions.py:63-79).  chunks: list of (N_c, 2) arrays.
    landmarks: structured array (LANDMARK_DTYPE).  Returns dict(models, mask,
    y_proj, state, lmk_out, lmk_count, chunk_pt_off)."""
    e = _engine()
    arrs = [np.ascontiguousarray(c, np.float64).reshape(-1, 2) for c in chunks]
    Cn = len(arrs)
    sizes = np.array([a.shape[0] for a in arrs], np.int64)
    cpo = np.concatenate([[0], np.cumsum(sizes)]).astype(np.int32)
    P = int(cpo[-1])
    data = np.concatenate(arrs) if P else np.zeros((1, 2))
    if state is None:
        st = np.random.get_state()
        state = np.concatenate([np.asarray(st[1], np.uint32), np.array([st[2]], np.uint32)])
    L = len(landmarks)
    cap = L + Cn
    lm = np.zeros(max(cap, 1), LANDMARK_DTYPE)
    lm[:L] = landmarks
    b = _lib.ScanBatch()
    b.n_scans, b.n_chunks, b.n_points = 1, Cn, P
    b.max_chunk_points = int(sizes.max()) if Cn else 0
    b.max_scan_chunks, b.lmk_capacity = Cn, max(cap, 1)
    b.xy = _upload(e, "r_xy", data).addr
    b.scan_chunk_off = _upload(e, "r_sco", np.array([0, Cn], np.int32)).addr
    b.chunk_pt_off = _upload(e, "r_cpo", cpo).addr
    b.mt_state_in = _upload(e, "r_st_in", np.ascontiguousarray(state, np.uint32)).addr
    b.mt_state_out = e.buf("r_st_out", 625 * 4).addr
    b.id_base = _upload(e, "r_idb", np.array([landmarkNumber], np.int32)).addr
    b.landmarks = _upload(e, "r_lmk", lm).addr
    b.lmk_count = _upload(e, "r_lmkc", np.array([L], np.int32)).addr
    b.inlier_mask = e.buf("r_mask", max(P, 1)).addr
    b.models = e.buf("r_models", MODEL_DTYPE.itemsize * max(Cn, 1)).addr
    b.y_proj = e.buf("r_yproj", 8 * max(P, 1)).addr
    p = _lib.ransac_params(residual_threshold=float(threshold), max_trials=int(max_trials))
    _lib.check(e.ctx._L.lslam_scan_pipeline(e.ctx.handle, C.byref(b), C.byref(p), None), "lslam_scan_pipeline")
    out = {
        "models": _download(e, e.bufs["r_models"], MODEL_DTYPE, Cn),
        "mask": _download(e, e.bufs["r_mask"], np.uint8, P).astype(bool),
        "y_proj": _download(e, e.bufs["r_yproj"], np.float64, P),
        "state": _download(e, e.bufs["r_st_out"], np.uint32, 625),
        "lmk_out": _download(e, e.bufs["r_lmk"], LANDMARK_DTYPE, max(cap, 1)),
        "lmk_count": int(_download(e, e.bufs["r_lmkc"], np.int32, 1)[0]),
        "chunk_pt_off": cpo,
        "data": data[:P],
    }
    e.ctx.sync()
    return out


_CHUNK_ERRORS = _lib.N_TOO_SMALL | _lib.NO_INLIERS | _lib.EST_FAIL


def process_revolution(chunks, landmarkNumber, landmarks):
    """check_ransac's work for one revolution (ransac_functions.py:66-79) in one
    launch.  Advances numpy's global RNG and updates ``landmarks`` (Landmark
    objects) like the per-chunk calls would; returns (LazyPoints of the
    revolution's projected inliers, new landmarkNumber).

    A chunk the reference would raise on (fewer than 3 points, no inliers, one
    final inlier) makes the revolution replay chunk by chunk through
    landmark_extraction from the saved state, so the exception surfaces at the
    same chunk with the same RNG and list state.
    """
    st = np.random.get_state()
    r = run_revolution(chunks, landmarkNumber, _as_records(landmarks))
    flags = r["models"]["flags"]
    if np.any(flags & _CHUNK_ERRORS):
        inl = []
        for c in chunks:
            q, fitted, new = landmark_extraction([c], landmarkNumber, landmarks)   # raises where the reference does
            inl.append(q)
            if new:
                landmarks.append(fitted)
            landmarkNumber += 1
        pts = [p for q in inl for p in q]
        return LazyPoints([p.x() for p in pts], [p.y() for p in pts]), landmarkNumber
    np.random.set_state((st[0], r["state"][:624].copy(), int(r["state"][624]), st[3], st[4]))
    # the list after the revolution: surviving objects keep their identity (life
    # updated), landmarks created during it become new Landmark objects
    by_id = {L.id: L for L in landmarks}
    rec = r["lmk_out"][:r["lmk_count"]]
    new_list = []
    for k in range(rec.shape[0]):
        e = rec[k]
        L = by_id.get(int(e["id"]))
        if L is None:
            L = Landmark(np.float64(e["a"]), np.float64(e["b"]), int(e["id"]), np.float64(e["pos_x"]),
                         np.float64(e["pos_y"]), np.float64(e["end_x"]), np.float64(e["end_y"]))
        L.life = int(e["life"])
        new_list.append(L)
    landmarks[:] = new_list
    m = r["mask"]
    return LazyPoints(r["data"][m, 0], r["y_proj"][m]), landmarkNumber + len(chunks)


def check_ransac_revolution(pairInliers, tempPoints, allPoints, pointsToBeFitted, landmarks, threadEvent,
                            poll_s=0.0005, stop=None):
    """check_ransac (ransac_functions.py:63-93) as a per-revolution dispatcher.

    Same arguments and outputs: when a revolution's delimiter ``0`` is in
    ``pointsToBeFitted``, its chunks run in one launch (process_revolution),
    ``pairInliers`` gets the revolution's projected inliers and ``allPoints``
    its raw points (both LazyPoints when ``tempPoints`` holds arrays, else the
    reference's concatenated QPointF arrays), and ``threadEvent`` is set.
    Differences: it sleeps ``poll_s`` instead of spinning, and it consumes the
    list up to the delimiter instead of clearing it whole, so chunks that
    arrive meanwhile are not lost (the reference's ``del pointsToBeFitted[:]``
    at :22 drops them).  ``stop``: optional threading.Event to end the loop.
    """
    landmarkNumber = 0
    while stop is None or not stop.is_set():
        try:
            end = next(i for i, c in enumerate(list(pointsToBeFitted)) if isinstance(c, int) and c == 0)
        except StopIteration:
            time.sleep(poll_s)
            continue
        chunks = list(pointsToBeFitted[:end])
        del pointsToBeFitted[:end + 1]
        raw = list(tempPoints[:len(chunks)])
        del tempPoints[:len(chunks)]
        if not chunks:
            continue
        pts, landmarkNumber = process_revolution(chunks, landmarkNumber, landmarks)
        pairInliers.append(pts)
        if raw and isinstance(raw[0], np.ndarray) and raw[0].dtype != object:
            a = np.concatenate([np.asarray(x, np.float64).reshape(-1, 2) for x in raw])
            allPoints.append(LazyPoints(a[:, 0], a[:, 1]))
        else:
            allPoints.append(np.concatenate(raw, axis=0) if raw else np.zeros(0, object))
        threadEvent.set()


def ransac_core_revolution(rawPoints):
    """ransac_core with the per-revolution dispatcher: raw chunks are kept as
    arrays (no QPointF per point on arrival, ransac_functions.py:114) and the
    GUI receives LazyPoints."""
    from mainWindow import ploting  # the reference GUI module, untouched
    pairInliers, pointsToBeFitted, allPoints, tempPoints = [], [], [], []
    landmarks = list()
    threadEvent = threading.Event()
    threading.Thread(target=check_ransac_revolution,
                     args=(pairInliers, tempPoints, allPoints, pointsToBeFitted, landmarks, threadEvent)).start()
    threading.Thread(target=ploting, args=(pairInliers, allPoints, threadEvent)).start()
    try:
        while True:
            temp = rawPoints.get(True)
            if temp is None:  # functions.scanning's end-of-stream marker
                break
            if temp != 0:
                tempPoints.append(np.asarray(temp, np.float64).reshape(-1, 2))
            pointsToBeFitted.append(temp)
    except KeyboardInterrupt:
        pass
