"""Diagnostic: per-phase cycle shares of chunk_kernel (s_memtime stamps), C3 workload.

Uses the diagnostic build lidar_slam_amd/liblidarslam_stamps.so (python -m
lidar_slam_amd.build --stamps).  Phases: 0 owning scan + draws, 6 point staging,
1 bounding box + cutoffs, 2 count pass, 3 ties + selection, 4 winner mask + refit,
5 line record + mask/y_proj stores.  Read the SHARES (stamps serialise the wave).
python tools/chunkstamps.py [scans] [philox|mt19937]"""
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "lidar_slam_amd", "liblidarslam_stamps.so")
L = _lib.load()
import ctypes as C  # noqa: E402
L.lslam_debug_set_stamps.argtypes = [C.c_void_p]
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
hyp = sys.argv[2] if len(sys.argv) > 2 else "philox"
ctx = Context(0)
b, _ = make_workload(list(range(S)), 720, 20)
nc = int(b["scan_chunk_off"][-1])
dbg = ctx.empty((max(nc, S), 16), np.uint64)
p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.arange(S), hyp=hyp)
p.run_ransac_only()
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
p.run_ransac_only()
ctx.sync()
L.lslam_debug_set_stamps(None)
d = dbg.download()[:nc]
names = {0: "scan+draws", 6: "stage", 1: "bbox+cutoffs", 2: "count", 3: "ties+select", 4: "mask+refit", 5: "record+stores"}
tot = d[:, list(names)].sum()
out = {"chunks": nc, "hyp": hyp, "cycles_per_chunk": round(float(tot) / nc, 1)}
for k, n in names.items():
    out[n] = round(float(d[:, k].sum()) / tot, 4)
print(json.dumps(out))
