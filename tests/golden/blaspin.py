"""Pin and record the BLAS dispatch the golden generators run under.

Import this module BEFORE numpy in every generator that runs the reference:

    import blaspin  # noqa: F401  (sets OPENBLAS_CORETYPE, must precede numpy)
    import numpy as np

Why: the reference's float outputs go through OpenBLAS (``dgemv_t`` behind
``(data - origin) @ direction`` and ``ddot`` behind ``np.linalg.norm``,
skimage ``fit.py:89,130-131``; LAPACK ``dgesdd`` at ``fit.py:94``, called from
``/root/reference/ransac_functions.py:23``).  numpy 1.26.4's bundled OpenBLAS
0.3.23 is a DYNAMIC_ARCH build: it picks a kernel set per host CPU at load
time, and the kernels round differently (the SkylakeX/Haswell ``dgemv_t``
uses FMA, the generic Prescott kernel does not).  The fixtures were made
under the SkylakeX kernels, so every generator forces that core
(``OPENBLAS_CORETYPE``, read by OpenBLAS when numpy loads it) and writes the
core OpenBLAS actually selected, the CPU model and the library versions into
each ``.npz`` as ``meta_*`` string arrays.  ``LSLAM_GOLDEN_CORETYPE``
overrides the pin for the dispatch census (``tests/golden/census_dispatch.py``).

``save_npz`` writes deterministic archives (fixed zip timestamps, sorted
members), so regenerating a fixture under the same pin is byte-identical.
"""
import ctypes
import os
import sys
import zipfile

PINNED_CORE = "SkylakeX"

if "numpy" in sys.modules:
    raise RuntimeError("blaspin must be imported before numpy (OPENBLAS_CORETYPE is read at load time)")
os.environ["OPENBLAS_CORETYPE"] = os.environ.get("LSLAM_GOLDEN_CORETYPE", PINNED_CORE)
os.environ["OPENBLAS_NUM_THREADS"] = "1"

import numpy as np  # noqa: E402


def _openblas():
    with open("/proc/self/maps") as f:
        libs = sorted({ln.split()[-1] for ln in f if "openblas" in ln.lower() and ln.rstrip().endswith(".so")})
    for path in libs:
        lib = ctypes.CDLL(path)
        for prefix in ("", "scipy_"):
            for suffix in ("64_", ""):
                fn = getattr(lib, prefix + "openblas_get_corename" + suffix, None)
                if fn is not None:
                    fn.restype = ctypes.c_char_p
                    cfg = getattr(lib, prefix + "openblas_get_config" + suffix)
                    cfg.restype = ctypes.c_char_p
                    return fn().decode(), cfg().decode()
    return "none", "none"


def cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return "unknown"


def meta():
    """The dispatch and environment a fixture was generated under, as npz-safe string arrays."""
    np.dot(np.ones(4), np.ones(4))  # make sure the BLAS is loaded
    core, config = _openblas()
    want = os.environ["OPENBLAS_CORETYPE"]
    if core.lower() != want.lower():
        raise RuntimeError("OpenBLAS selected core %r, not the pinned %r" % (core, want))
    m = {"meta_blas_core": core, "meta_blas_config": config, "meta_cpu_model": cpu_model(),
         "meta_numpy": np.__version__, "meta_python": sys.version.split()[0]}
    try:
        import skimage
        m["meta_skimage"] = skimage.__version__
    except ImportError:
        pass
    return {k: np.asarray(v) for k, v in m.items()}


def save_npz(path, **arrays):
    """np.savez_compressed with the dispatch metadata added, and byte-reproducible output."""
    arrays = dict(arrays)
    arrays.update(meta())
    with zipfile.ZipFile(path, "w", zipfile.ZIP_DEFLATED) as zf:
        for name in sorted(arrays):
            info = zipfile.ZipInfo(name + ".npy", date_time=(1980, 1, 1, 0, 0, 0))
            info.compress_type = zipfile.ZIP_DEFLATED
            info.external_attr = 0o644 << 16
            with zf.open(info, "w", force_zip64=True) as fh:
                np.lib.format.write_array(fh, np.asanyarray(arrays[name]), allow_pickle=False)
