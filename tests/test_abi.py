"""CPU-side checks of the C ABI: the library loads, exports every symbol that
include/lidarslam.h declares, struct layouts match, and the pure-host helpers
agree with the oracle.  No device calls (no GPU in the build container)."""
import ctypes as C
import os
import re

import numpy as np
import pytest

from lidar_slam_amd import _lib
from lidar_slam_amd import pipeline as pl
from oracle import cpu as orc
from oracle import ukf as oukf

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))


def _header_functions():
    txt = open(os.path.join(ROOT, "include", "lidarslam.h")).read()
    return sorted(set(re.findall(r"\b(lslam_[a-z0-9_]+)\s*\(", txt)))


def test_header_symbols_exported():
    L = _lib.load()
    declared = _header_functions()
    assert len(declared) >= 25
    for name in declared:
        assert hasattr(L, name), name
    assert sorted(_lib.EXPORTS) == declared


def test_struct_layouts():
    assert C.sizeof(_lib.ChunkModel) == 112 == pl.MODEL_DTYPE.itemsize
    assert C.sizeof(_lib.LandmarkRec) == 56 == pl.LANDMARK_DTYPE.itemsize
    assert C.sizeof(_lib.RansacParams) == 56
    for f, _ in _lib.ChunkModel._fields_:
        assert getattr(_lib.ChunkModel, f).offset == pl.MODEL_DTYPE.fields[f][1]


def test_library_built_from_these_sources():
    from lidar_slam_amd import build
    L = _lib.load()
    assert ("src %s," % build.source_hash()).encode() in L.lslam_version()
    assert build.embedded_hash() == build.source_hash()


def test_stale_library_raises(monkeypatch):
    """A library whose embedded source hash differs from the tree's is refused (no silent A/B leftovers)."""
    from lidar_slam_amd import build
    monkeypatch.delenv("LSLAM_ALLOW_STALE", raising=False)
    monkeypatch.setattr(_lib, "_err", None)
    with pytest.raises(_lib.HIPLibraryError, match="built from other sources"):
        _lib._check_source("0123456789abcdef", want=build.source_hash())
    with pytest.raises(_lib.HIPLibraryError, match="built from other sources"):
        _lib._check_source("0123456789abcdef")
    _lib._check_source(build.source_hash())
    monkeypatch.setenv("LSLAM_ALLOW_STALE", "1")
    _lib._check_source("0123456789abcdef")


def test_version_and_defaults():
    L = _lib.load()
    assert b"gfx950" in L.lslam_version()
    assert b"(abi %d," % _lib.ABI_VERSION in L.lslam_version()
    p = _lib.ransac_params()
    assert (p.residual_threshold, p.max_trials, p.min_samples, p.life) == (20.0, 100, 2, 40)
    assert (p.tol_a, p.tol_b, p.tol_dist) == (0.1, 10.0, 100.0)
    u = _lib.ukf_params(8)
    assert u.dt == 0.005 and u.alpha == 1e-4 and u.beta == 2 and u.kappa == 0
    assert list(u.Q) == [0.001, 0, 0, 0, 0.001, 0, 0, 0, 0.001]


def test_cutoff_matches_oracle():
    for thr in (20.0, 1.0, 0.5, 1e-9, 77.7, 0.0):
        assert pl.inlier_cutoff(thr) == orc.ecut(thr)
    assert pl.inlier_cutoff(20.0) == 399.99999999999994


def test_seed_state_matches_numpy():
    for seed in (0, 1, 12345, 2 ** 32 - 1):
        st = pl.mt_seed_state(seed)
        ref = np.random.RandomState(seed).get_state()
        assert np.array_equal(st[:624], ref[1]) and st[624] == ref[2]


def test_ukf_weights_match_filterpy_restatement():
    Wm, Wc, lpn = pl.ukf_weights(_lib.ukf_params(20))
    pts = oukf.MerweScaledSigmaPoints(3, 1e-4, 2.0, 0.0)
    assert np.array_equal(Wm, pts.Wm) and np.array_equal(Wc, pts.Wc)
    assert lpn == (1e-4 ** 2 * 3 - 3) + 3


def test_no_device_is_loud_not_silent():
    """Without a GPU, creating a context must raise, never fall back to CPU."""
    from lidar_slam_amd.device import Context
    if Context.device_count() > 0:
        pytest.skip("a GPU is present")
    with pytest.raises((_lib.HIPLibraryError, ValueError)):
        Context(0)
