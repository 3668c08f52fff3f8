"""ctypes binding of the HIP library ``liblidarslam.so`` (C ABI: include/lidarslam.h).

The library is built in-tree (``python -m lidar_slam_amd.build`` or
``__graft_entry__.build()``).  There is NO CPU fallback: if the shared object
is missing or cannot be loaded, every entry point raises ``HIPLibraryError``.
"""
from __future__ import annotations

import ctypes as C
import os
import re

_HERE = os.path.dirname(os.path.abspath(__file__))
LIB_PATH = os.environ.get("LSLAM_LIB") or os.path.join(_HERE, "liblidarslam.so")  # override: experiments

# ---- constants mirrored from include/lidarslam.h ----
ABI_VERSION = 4  # include/lidarslam.h LSLAM_ABI_VERSION (struct layouts below)
LSLAM_OK = 0
LSLAM_ERR_ARG = -1
LSLAM_ERR_HIP = -2
LSLAM_ERR_NOMEM = -3
LSLAM_ERR_CAPACITY = -4
LSLAM_ERR_UNSUPPORTED = -5

VALID, N_TOO_SMALL, NO_INLIERS, EST_FAIL = 1, 2, 4, 8
EARLY_STOP, VERTICAL, NEW_LANDMARK, MATCHED = 16, 32, 64, 128
CAPACITY, CHUNK_BOUND = 256, 512

HYP_MT19937, HYP_PHILOX, HYP_EXPLICIT = 0, 1, 2
UKF_PREDICT, UKF_UPDATE, UKF_LMK_FROM_RANSAC, UKF_MAP, UKF_SIGMAS_IN = 1, 2, 4, 8, 16
K_POLAR, K_HYP, K_PIPELINE, K_LANDMARK, K_UKF, K_RNG, K_CONSENSUS = 0, 1, 2, 3, 4, 5, 6
K_EXPRESS, K_EXPRESS_SCATTER = 7, 8


class HIPLibraryError(RuntimeError):
    """The HIP library is missing, failed to load, or returned an error."""


class ChunkModel(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("ox", "oy", "ux", "uy", "a", "b", "tip_x", "tip_y",
                                          "proj_a", "proj_b")] + \
               [(n, C.c_int32) for n in ("n_inliers", "best_trial", "n_draws", "flags",
                                         "match_index", "landmark_id", "n_points", "reserved")]


class LandmarkRec(C.Structure):
    _fields_ = [(n, C.c_double) for n in ("a", "b", "pos_x", "pos_y", "end_x", "end_y")] + \
               [("id", C.c_int32), ("life", C.c_int32)]


class RansacParams(C.Structure):
    _fields_ = [("residual_threshold", C.c_double), ("max_trials", C.c_int32), ("min_samples", C.c_int32),
                ("hyp_source", C.c_int32), ("life", C.c_int32), ("tol_a", C.c_double), ("tol_b", C.c_double),
                ("tol_dist", C.c_double), ("philox_seed", C.c_uint64)]


class UkfParams(C.Structure):
    _fields_ = [("n_landmarks", C.c_int32), ("flags", C.c_int32), ("dt", C.c_double),
                ("wheel_radius", C.c_double), ("wheel_base", C.c_double), ("alpha", C.c_double),
                ("beta", C.c_double), ("kappa", C.c_double), ("Q", C.c_double * 9)]


_VP = C.c_void_p


class ScanBatch(C.Structure):
    _fields_ = [("n_scans", C.c_int32), ("n_chunks", C.c_int32), ("n_points", C.c_int64),
                ("max_chunk_points", C.c_int32), ("max_scan_chunks", C.c_int32), ("lmk_capacity", C.c_int32),
                ("reserved", C.c_int32)] + \
               [(n, _VP) for n in ("xy", "scan_chunk_off", "chunk_pt_off", "seeds", "mt_state_in", "mt_state_out",
                                   "hyp", "id_base", "landmarks", "lmk_count", "lmk_walk", "inlier_mask", "models", "y_proj",
                                   "draws_out", "trial_cnt_out", "ukf_x", "ukf_P", "ukf_u", "ukf_z", "ukf_lmk",
                                   "ukf_R_diag", "theta_deg", "dist_mm", "ukf_sigmas")]


class ExpressMeasures(C.Structure):
    _fields_ = [(n, _VP) for n in ("angle_deg", "dist_mm", "new_scan", "valid", "xy", "pkt_valid")]


class ExpressRevs(C.Structure):
    _fields_ = [(n, _VP) for n in ("xy", "scan_chunk_off", "chunk_pt_off", "counts")] + \
               [("cap_points", C.c_int64), ("cap_scans", C.c_int32), ("cap_chunks", C.c_int32)]


assert C.sizeof(ChunkModel) == 112
assert C.sizeof(LandmarkRec) == 56

EXPORTS = [
    "lslam_version", "lslam_status_string", "lslam_last_error", "lslam_device_count", "lslam_ctx_create",
    "lslam_ctx_destroy", "lslam_sync", "lslam_malloc", "lslam_free", "lslam_host_alloc", "lslam_host_free",
    "lslam_h2d", "lslam_d2h", "lslam_d2d", "lslam_memset", "lslam_host_register", "lslam_host_unregister",
    "lslam_ctx_stream", "lslam_abi_sizes", "lslam_set_timing", "lslam_set_timing_mask", "lslam_timing",
    "lslam_timing_reset", "lslam_set_steps_budget",
    "lslam_ransac_params_default", "lslam_ukf_params_default", "lslam_inlier_cutoff", "lslam_ukf_weights",
    "lslam_mt_seed_state", "lslam_polar_to_xy", "lslam_hyp_mt19937", "lslam_ransac", "lslam_landmarks",
    "lslam_ukf_step", "lslam_ukf_trace", "lslam_scan_pipeline", "lslam_express_decode", "lslam_express_scans",
]

_lib = None
_err = None


def load():
    """Load and type the library (raises HIPLibraryError if unavailable)."""
    global _lib, _err
    if _lib is not None:
        return _lib
    if _err is not None:
        raise _err
    if not os.path.exists(LIB_PATH):
        _err = HIPLibraryError("HIP library %s is not built; run `python -m lidar_slam_amd.build` "
                               "(there is no CPU fallback)" % LIB_PATH)
        raise _err
    try:
        L = C.CDLL(LIB_PATH)
    except OSError as e:  # pragma: no cover
        _err = HIPLibraryError("cannot load %s: %s" % (LIB_PATH, e))
        raise _err
    P = C.POINTER
    i32, i64, u32, dbl, sz = C.c_int32, C.c_int64, C.c_uint32, C.c_double, C.c_size_t
    sig = {
        "lslam_version": ([], C.c_char_p),
        "lslam_status_string": ([C.c_int], C.c_char_p),
        "lslam_last_error": ([], C.c_char_p),
        "lslam_device_count": ([P(C.c_int)], C.c_int),
        "lslam_ctx_create": ([C.c_int, P(_VP)], C.c_int),
        "lslam_ctx_destroy": ([_VP], C.c_int),
        "lslam_sync": ([_VP], C.c_int),
        "lslam_malloc": ([_VP, sz, P(_VP)], C.c_int),
        "lslam_free": ([_VP, _VP], C.c_int),
        "lslam_host_alloc": ([sz, P(_VP)], C.c_int),
        "lslam_host_free": ([_VP], C.c_int),
        "lslam_h2d": ([_VP, _VP, _VP, sz], C.c_int),
        "lslam_d2h": ([_VP, _VP, _VP, sz], C.c_int),
        "lslam_d2d": ([_VP, _VP, _VP, sz], C.c_int),
        "lslam_memset": ([_VP, _VP, C.c_int, sz], C.c_int),
        "lslam_host_register": ([_VP, sz], C.c_int),
        "lslam_host_unregister": ([_VP], C.c_int),
        "lslam_ctx_stream": ([_VP, P(_VP)], C.c_int),
        "lslam_abi_sizes": ([P(i64), C.c_int], C.c_int),
        "lslam_set_timing": ([_VP, C.c_int], C.c_int),
        "lslam_set_timing_mask": ([_VP, u32], C.c_int),
        "lslam_timing": ([_VP, C.c_int, P(dbl), P(i64)], C.c_int),
        "lslam_timing_reset": ([_VP], C.c_int),
        "lslam_set_steps_budget": ([_VP, i64], C.c_int),
        "lslam_ransac_params_default": ([P(RansacParams)], C.c_int),
        "lslam_ukf_params_default": ([P(UkfParams), i32], C.c_int),
        "lslam_inlier_cutoff": ([dbl], dbl),
        "lslam_ukf_weights": ([P(UkfParams), P(dbl), P(dbl), P(dbl)], C.c_int),
        "lslam_mt_seed_state": ([u32, P(u32)], C.c_int),
        "lslam_polar_to_xy": ([_VP, _VP, _VP, _VP, i64], C.c_int),
        "lslam_hyp_mt19937": ([_VP, P(ScanBatch), i32], C.c_int),
        "lslam_ransac": ([_VP, P(ScanBatch), P(RansacParams)], C.c_int),
        "lslam_landmarks": ([_VP, P(ScanBatch), P(RansacParams)], C.c_int),
        "lslam_ukf_step": ([_VP, P(ScanBatch), P(UkfParams)], C.c_int),
        "lslam_ukf_trace": ([_VP, P(ScanBatch), P(UkfParams), _VP], C.c_int),
        "lslam_scan_pipeline": ([_VP, P(ScanBatch), P(RansacParams), P(UkfParams)], C.c_int),
        "lslam_express_decode": ([_VP, _VP, i64, P(ExpressMeasures)], C.c_int),
        "lslam_express_scans": ([_VP, _VP, i64, i32, P(ExpressRevs)], C.c_int),
    }
    try:
        for name, (args, res) in sig.items():
            f = getattr(L, name)
            f.argtypes = args
            f.restype = res
    except AttributeError as e:
        _err = HIPLibraryError("%s lacks %s: a stale build? rebuild with `python -m lidar_slam_amd.build`"
                               % (LIB_PATH, e))
        raise _err
    _check_abi(L)
    _lib = L
    return L


def _check_abi(L):
    """The library must be the ABI these ctypes layouts describe: a stale .so (e.g. via LSLAM_LIB)
    would silently ignore appended struct fields."""
    global _err
    ver = L.lslam_version().decode(errors="replace")
    m = re.search(r"\(abi (\d+), src ([0-9a-f]{16}),", ver)
    if not m or int(m.group(1)) != ABI_VERSION:
        _err = HIPLibraryError("%s reports %r; this binding needs ABI %d (rebuild the library)"
                               % (LIB_PATH, ver, ABI_VERSION))
        raise _err
    _check_source(m.group(2))
    got = (C.c_int64 * 7)()
    L.lslam_abi_sizes(got, 7)
    want = [C.sizeof(t) for t in (ChunkModel, LandmarkRec, RansacParams, UkfParams, ScanBatch, ExpressMeasures,
                                  ExpressRevs)]
    if list(got) != want:
        _err = HIPLibraryError("struct sizes differ between %s %s and the ctypes layouts %s"
                               % (LIB_PATH, list(got), want))
        raise _err


def _check_source(lib_hash, want=None):
    """The library must be built from the sources next to it: a stale .so (built from other
    sources, e.g. an A/B leftover) raises.  ``LSLAM_ALLOW_STALE=1`` skips the check (A/B runs of
    deliberately different builds via LSLAM_LIB)."""
    global _err
    if os.environ.get("LSLAM_ALLOW_STALE") == "1":
        return
    if want is None:
        from . import build
        want = build.source_hash()
    if lib_hash != want:
        _err = HIPLibraryError("%s was built from other sources (src %s, the tree's is %s): rebuild with "
                               "`python -m lidar_slam_amd.build`" % (LIB_PATH, lib_hash, want))
        raise _err


def check(status, what=""):
    if status != LSLAM_OK:
        L = load()
        msg = L.lslam_last_error().decode(errors="replace")
        st = L.lslam_status_string(status).decode()
        if status == LSLAM_ERR_ARG:
            raise ValueError("%s: %s (%s)" % (what, st, msg))
        raise HIPLibraryError("%s: %s (%s)" % (what, st, msg))
    return status


def ransac_params(**kw):
    p = RansacParams()
    load().lslam_ransac_params_default(C.byref(p))
    for k, v in kw.items():
        setattr(p, k, v)
    return p


def ukf_params(n_landmarks, **kw):
    p = UkfParams()
    load().lslam_ukf_params_default(C.byref(p), int(n_landmarks))
    for k, v in kw.items():
        if k == "Q":
            for i, q in enumerate(list(v)):
                p.Q[i] = float(q)
        else:
            setattr(p, k, v)
    return p
