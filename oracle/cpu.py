"""ORACLE — TEST INFRASTRUCTURE ONLY.  ctypes binding of oracle/ransac_oracle.c.

Build with ``make -C oracle`` (``__graft_entry__.build()`` does it).  See the C
file's header for the reference file:line each function restates.
"""
from __future__ import annotations

import ctypes as C
import os
import subprocess

import numpy as np

_HERE = os.path.dirname(os.path.abspath(__file__))
_SO = os.path.join(_HERE, "build", "liboracle.so")

FLAG_VALID, FLAG_N_TOO_SMALL, FLAG_NO_INLIERS, FLAG_EST_FAIL = 1, 2, 4, 8
FLAG_EARLY_STOP, FLAG_VERTICAL, FLAG_NEW_LANDMARK, FLAG_MATCHED = 16, 32, 64, 128


class ChunkModel(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("ox", "oy", "ux", "uy", "a", "b", "tip_x", "tip_y",
                                          "proj_a", "proj_b")] + \
               [(n, C.c_int32) for n in ("n_inliers", "best_trial", "n_draws", "flags",
                                         "match_index", "landmark_id", "n_points", "reserved")]


class Landmark(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("a", "b", "px", "py", "ex", "ey")] + \
               [("id", C.c_int32), ("life", C.c_int32)]


_lib = None


def lib():
    global _lib
    if _lib is None:
        if not os.path.exists(_SO):
            subprocess.check_call(["make", "-C", _HERE, "-s"])
        L = C.CDLL(_SO)
        P = C.POINTER
        L.or_mt_seed.argtypes = [C.c_uint32, P(C.c_uint32), P(C.c_int32)]
        L.or_mt_next.argtypes = [P(C.c_uint32), P(C.c_int32)]
        L.or_mt_next.restype = C.c_uint32
        L.or_choice2.argtypes = [P(C.c_uint32), P(C.c_int32), C.c_int32, P(C.c_int32), P(C.c_int32)]
        L.or_ecut.argtypes = [C.c_double]
        L.or_ecut.restype = C.c_double
        L.or_ransac.argtypes = [P(C.c_double), C.c_int32, C.c_double, C.c_int32, P(C.c_uint32),
                                P(C.c_int32), P(C.c_int32), P(C.c_uint8), P(ChunkModel), P(C.c_int32),
                                P(C.c_int32), P(C.c_double)]
        L.or_ransac_chained.argtypes = [P(C.c_double), C.c_int32, C.c_double, C.c_int32, P(C.c_uint32),
                                        P(C.c_int32), P(C.c_uint8), P(ChunkModel), P(C.c_int32),
                                        P(C.c_int32), P(C.c_double)]
        L.or_landmark_extraction.argtypes = [P(C.c_double), C.c_int32, C.c_int32, C.c_double, C.c_int32,
                                             P(C.c_uint32), P(C.c_int32), P(Landmark), P(C.c_int32),
                                             C.c_int32, P(C.c_uint8), P(C.c_double), P(ChunkModel)]
        L.or_is_equal.argtypes = [P(Landmark), P(Landmark)]
        L.or_associate.argtypes = [P(Landmark), P(C.c_int32), C.c_int32, P(Landmark), P(C.c_int32),
                                   P(C.c_double), P(C.c_double)]
        L.or_associate.restype = C.c_int32
        L.or_set_tolerances.argtypes = [C.c_double, C.c_double, C.c_double]
        _lib = L
    return _lib


def _p(a, t):
    return a.ctypes.data_as(C.POINTER(t))


class MTState:
    """numpy legacy RandomState MT19937 state (key[624], pos)."""

    def __init__(self, key=None, pos=624, seed=None):
        self.key = np.zeros(624, np.uint32) if key is None else np.array(key, np.uint32)
        self.pos = C.c_int32(int(pos))
        if seed is not None:
            lib().or_mt_seed(C.c_uint32(int(seed) & 0xFFFFFFFF), _p(self.key, C.c_uint32), C.byref(self.pos))

    @classmethod
    def from_numpy(cls, st):
        return cls(st[1], st[2])

    def next32(self):
        return lib().or_mt_next(_p(self.key, C.c_uint32), C.byref(self.pos))

    def choice2(self, n):
        perm = np.zeros(n, np.int32)
        out = np.zeros(2, np.int32)
        lib().or_choice2(_p(self.key, C.c_uint32), C.byref(self.pos), int(n), _p(perm, C.c_int32),
                         _p(out, C.c_int32))
        return out

    def copy(self):
        return MTState(self.key.copy(), self.pos.value)


def ecut(thr):
    return lib().or_ecut(float(thr))


def model_dict(m):
    return {f: getattr(m, f) for f, _ in ChunkModel._fields_}


def ransac(xy, thr=20.0, trials=100, state=None, hyp=None, chained=True, want_trials=False):
    """One skimage-semantics ransac call.  Returns (mask, model dict, extra)."""
    xy = np.ascontiguousarray(xy, np.float64)
    n = xy.shape[0]
    mask = np.zeros(max(n, 1), np.uint8)
    m = ChunkModel()
    draws = np.zeros((trials + 1) * 2, np.int32)
    cnt = np.zeros(max(trials, 1), np.int32)
    sm = np.zeros(max(trials, 1), np.float64)
    st = state if state is not None else MTState(seed=0)
    L = lib()
    if hyp is not None:
        h = np.ascontiguousarray(hyp, np.int32).reshape(-1)
        rc = L.or_ransac(_p(xy, C.c_double), n, float(thr), int(trials), _p(st.key, C.c_uint32),
                         C.byref(st.pos), _p(h, C.c_int32), _p(mask, C.c_uint8), C.byref(m),
                         _p(draws, C.c_int32), _p(cnt, C.c_int32), _p(sm, C.c_double))
    elif chained:
        rc = L.or_ransac_chained(_p(xy, C.c_double), n, float(thr), int(trials), _p(st.key, C.c_uint32),
                                 C.byref(st.pos), _p(mask, C.c_uint8), C.byref(m), _p(draws, C.c_int32),
                                 _p(cnt, C.c_int32), _p(sm, C.c_double))
    else:
        rc = L.or_ransac(_p(xy, C.c_double), n, float(thr), int(trials), _p(st.key, C.c_uint32),
                         C.byref(st.pos), None, _p(mask, C.c_uint8), C.byref(m), _p(draws, C.c_int32),
                         _p(cnt, C.c_int32), _p(sm, C.c_double))
    if rc != 0:
        raise ValueError("oracle ransac rc=%d" % rc)
    extra = {"draws": draws.reshape(-1, 2), "state": st}
    if want_trials:
        extra["cnt"] = cnt[:trials]
        extra["sum"] = sm[:trials]
    return mask[:n], model_dict(m), extra


def landmarks_to_array(lst, cap):
    arr = (Landmark * max(cap, 1))()
    for i, L in enumerate(lst):
        arr[i].a, arr[i].b = L["a"], L["b"]
        arr[i].px, arr[i].py = L["pos"]
        arr[i].ex, arr[i].ey = L["end"]
        arr[i].id, arr[i].life = L["id"], L["life"]
    return arr


def array_to_landmarks(arr, count):
    return [{"a": arr[i].a, "b": arr[i].b, "pos": (arr[i].px, arr[i].py), "end": (arr[i].ex, arr[i].ey),
             "id": arr[i].id, "life": arr[i].life} for i in range(count)]


def landmark_extraction(xy, landmark_number, landmarks, state, thr=20.0, trials=100, cap=None):
    """ransac_functions.py:15-59 (+ check_ransac's append) on one chunk.
    `landmarks` is a list of dicts {a,b,pos,end,id,life}; returns
    (mask, yproj, model, new_landmarks_list)."""
    xy = np.ascontiguousarray(xy, np.float64)
    n = xy.shape[0]
    cap = cap or (len(landmarks) + 1)
    arr = landmarks_to_array(landmarks, cap)
    count = C.c_int32(len(landmarks))
    mask = np.zeros(max(n, 1), np.uint8)
    yproj = np.zeros(max(n, 1), np.float64)
    m = ChunkModel()
    rc = lib().or_landmark_extraction(_p(xy, C.c_double), n, int(landmark_number), float(thr), int(trials),
                                      _p(state.key, C.c_uint32), C.byref(state.pos), arr, C.byref(count),
                                      cap, _p(mask, C.c_uint8), _p(yproj, C.c_double), C.byref(m))
    if rc == -2:
        # no match and the list was full (the library's LSLAM_CAPACITY): the chunk's landmark is
        # dropped, its inliers projected on its own line (or_associate left proj_a/b = a, b)
        m.flags |= 64 | 256
        m.match_index = -1
        yproj[:n] = np.where(mask[:n] != 0, m.proj_a * xy[:, 0] + m.proj_b, 0.0)
    elif rc != 0:
        raise RuntimeError("oracle landmark_extraction rc=%d" % rc)
    return mask[:n], yproj[:n], model_dict(m), array_to_landmarks(arr, count.value)


def set_tolerances(tol_a=0.1, tol_b=10.0, tol_dist=100.0):
    """landmarking.py:4-6 constants used by the association walk (defaults = the reference's)."""
    lib().or_set_tolerances(float(tol_a), float(tol_b), float(tol_dist))


def associate(landmarks, F, cap):
    """ransac_functions.py:34-54 walk + check_ransac's append for an already
    fitted line F = {a, b, pos, end, id}.  Returns (match index or -1 / -2 if
    the list was full, matched landmark dict or None, new list)."""
    arr = landmarks_to_array(landmarks, cap)
    f = landmarks_to_array([dict(F, life=0)], 1)
    count = C.c_int32(len(landmarks))
    nf = C.c_int32(0)
    pa, pb = C.c_double(0), C.c_double(0)
    m = lib().or_associate(arr, C.byref(count), int(cap), f, C.byref(nf), C.byref(pa), C.byref(pb))
    matched = dict(landmarks[m]) if m >= 0 else None
    return m, matched, array_to_landmarks(arr, count.value)


def run_batch(xy, scan_chunk_off, chunk_pt_off, seeds, thr=20.0, trials=100, landmarks_in=None):
    """Batched semantics: per scan np.random.seed(seed[s]) chained over its
    chunks, per-scan landmark list (default empty), landmark ids = chunk index
    within the scan.  Returns (mask[P], models list, per-scan landmark lists)."""
    xy = np.ascontiguousarray(xy, np.float64)
    P = xy.shape[0]
    mask = np.zeros(P, np.uint8)
    yproj = np.zeros(P, np.float64)
    models, lists = [], []
    for s in range(len(scan_chunk_off) - 1):
        st = MTState(seed=int(seeds[s]))
        lst = list(landmarks_in[s]) if landmarks_in is not None else []
        for k, c in enumerate(range(scan_chunk_off[s], scan_chunk_off[s + 1])):
            p0, p1 = chunk_pt_off[c], chunk_pt_off[c + 1]
            m, y, mod, lst = landmark_extraction(xy[p0:p1], k, lst, st, thr, trials,
                                                 cap=len(lst) + 1)
            mask[p0:p1] = m
            yproj[p0:p1] = y
            models.append(mod)
        lists.append(lst)
    return mask, yproj, models, lists
