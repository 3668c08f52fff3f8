"""Diagnostic: per-phase cycle shares of the MT19937 parse (s_memtime stamps).

Uses the separate diagnostic build lidar_slam_amd/liblidarslam_stamps.so
(hipcc ... -DLSLAM_STAMPS); the product library has no stamps.  Read the
SHARES, not the absolute time (stamps serialise the wave)."""
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

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ctx = Context(0)
b, _ = make_workload(list(range(S)), 720, 20)
dbg = ctx.empty((S, 8), np.uint64)
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
pl.hyp_mt19937(ctx, b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.arange(S))
acc = dbg.download().astype(np.float64)
names = ["twist", "load+temper", "fixed-point", "scatter+advance", "resolve"]
tot = acc[:, :5].sum(1)
out = {n: round(float(np.mean(acc[:, k])), 0) for k, n in enumerate(names)}
out["total_cycles_per_scan"] = round(float(tot.mean()), 0)
out["shares"] = {n: round(float(np.mean(acc[:, k]) / tot.mean()), 3) for k, n in enumerate(names)}
print(json.dumps(out))
