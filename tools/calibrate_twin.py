"""Calibrate bench.py's CPU baseline: the NumPy twin (oracle/numpy_twin.py) against the
reference's own CPU path on the same scans, one core.

The reference cannot travel to the GPU box, so bench.py times the twin there; this
script, run ONLY in the build container with the interpreter that can import the
reference (scikit-image 0.18.3), measures how the twin's rate relates to the
reference's:

    /opt/conda/bin/python3.9 tools/calibrate_twin.py [--scans 256]

Reference path timed: ransac_functions.py:15-59 ``landmark_extraction`` imported
unmodified (only the Qt-only ``mainWindow`` module is stubbed), driven as
check_ransac does (ransac_functions.py:73-78: each chunk arrives as a Python list,
np.random.seed(scan) per scan, the new landmark appended).  Its prints go to a
buffer.  Twin timed: ``numpy_twin.process_scan`` on the same chunks and seeds.  The
twin's masks are checked equal to the reference's.  Writes profiles/r02_calibration.json.
"""
import argparse
import contextlib
import io
import json
import os
import platform
import sys
import time
import types

os.environ["OPENBLAS_NUM_THREADS"] = "1"
os.environ["OMP_NUM_THREADS"] = "1"
sys.path.insert(0, os.path.join(os.path.dirname(os.path.abspath(__file__)), "..", "tests", "golden"))
import blaspin  # noqa: E402  (pins OPENBLAS_CORETYPE = SkylakeX; must precede numpy)
import numpy as np  # noqa: E402

HERE = os.path.dirname(os.path.abspath(__file__))
ROOT = os.path.dirname(HERE)
sys.path.insert(0, "/root/reference")
sys.path.insert(0, ROOT)
_stub = types.ModuleType("mainWindow")
_stub.time = time
_stub.ploting = lambda *a, **k: None
sys.modules["mainWindow"] = _stub

import ransac_functions as rf  # noqa: E402  (the reference, unmodified)

from lidar_slam_amd import synth  # noqa: E402
from oracle import numpy_twin as tw  # noqa: E402


def cpu_model():
    with open("/proc/cpuinfo") as f:
        for line in f:
            if line.startswith("model name"):
                return line.split(":", 1)[1].strip()
    return platform.processor()


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=256)
    ap.add_argument("--out", default=os.path.join(ROOT, "profiles", "r02_calibration.json"))
    args = ap.parse_args()
    ids = list(range(args.scans))
    b = synth.make_batch(ids)
    sco, cpo, xy = b["scan_chunk_off"], b["chunk_pt_off"], b["xy"]
    chunks = [[xy[cpo[c]:cpo[c + 1]].tolist() for c in range(sco[s], sco[s + 1])] for s in ids]
    # warm both paths
    np.random.seed(0)
    with contextlib.redirect_stdout(io.StringIO()):
        rf.landmark_extraction([list(chunks[0][0])], 0, [])
    tw.process_scan(xy[cpo[0]:cpo[sco[1]]], cpo[0:sco[1] + 1] - cpo[0], 0)

    ref_masks = []
    sink = io.StringIO()
    t0 = time.perf_counter()
    with contextlib.redirect_stdout(sink):
        for s in ids:
            np.random.seed(s)
            landmarks = []
            for k, pts in enumerate(chunks[s]):
                batch = [pts]
                q, fitted, new = rf.landmark_extraction(batch, k, landmarks)
                if new:
                    landmarks.append(fitted)
                ref_masks.append(len(q))
    t_ref = time.perf_counter() - t0

    twin_counts = []
    t0 = time.perf_counter()
    for s in ids:
        c0, c1 = sco[s], sco[s + 1]
        masks, _ = tw.process_scan(xy[cpo[c0]:cpo[c1]], cpo[c0:c1 + 1] - cpo[c0], s)
        twin_counts.extend(int(np.sum(m)) for m in masks)
    t_twin = time.perf_counter() - t0
    assert twin_counts == ref_masks, "the twin's inlier counts differ from the reference's"

    out = {
        "scans": args.scans, "points_per_scan": 720, "chunks_per_scan": 8,
        "reference_s": round(t_ref, 3), "reference_scans_per_s": round(args.scans / t_ref, 2),
        "twin_s": round(t_twin, 3), "twin_scans_per_s": round(args.scans / t_twin, 2),
        "twin_over_reference": round(t_ref / t_twin, 3),
        "cores": 1, "cpu_model": cpu_model(), "host_cpus": os.cpu_count(),
        "python": platform.python_version(), "numpy": np.__version__,
        "blas_core": str(blaspin.meta()["meta_blas_core"]),
        "note": "reference = ransac_functions.landmark_extraction (skimage 0.18.3 ransac) per chunk as check_ransac "
                "drives it; twin = oracle/numpy_twin.process_scan; same scans and seeds, inlier counts equal",
    }
    with open(args.out, "w") as f:
        json.dump(out, f, indent=1)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
