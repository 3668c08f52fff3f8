"""Diagnostic: phase cycles of select_kernel (large chunks) on C5, from the
stamps build (python -m lidar_slam_amd.build --stamps).  Shares matter, not
absolute cycles (stamps serialise the wave).

python tools/selectstamps.py [scans]
"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "lidar_slam_amd", "liblidarslam_stamps.so")
L = _lib.load()
L.lslam_debug_set_stamps.argtypes = [C.c_void_p]
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 1024
ctx = Context(0)
b, _ = make_workload(list(range(S)), 4096, 20)
sco = np.arange(S + 1, dtype=np.int32)
cpo = (np.arange(S + 1) * 4096).astype(np.int32)
dbg = ctx.empty((S, 16), np.uint64)
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
p = pl.ScanPipeline(ctx, b["xy"], sco, cpo, hyp="philox", max_trials=2048)
p.run()
acc = dbg.download().astype(np.float64)
names = ["load_box", "counts_max_tied", "tie_sums", "candidates", "finish_fit", "finish_chunk"]
tot = acc[:, 8:14].sum(1).mean()
out = {"scans": S, "cycles_total": round(float(tot), 0),
       "shares": {n: round(float(acc[:, 8 + k].mean() / tot), 3) for k, n in enumerate(names)},
       "ntied_mean": float(acc[:, 14].mean()), "n_inliers_mean": float(acc[:, 15].mean())}
print(json.dumps(out))
