"""Diagnostic: per-phase cycles of the post pass (association + y_proj over fitted models, s_memtime
stamps in post_assoc_reg, the register-list pass C3 takes, and post_assoc_fast), C3 workload, alone and in the pipeline beside the next call's producer.

Uses the diagnostic build lidar_slam_amd/liblidarslam_stamps.so (python -m lidar_slam_amd.build
--stamps).  Phases per scan: 1 records + offsets in, 2 association walk over the chunks, 3 records
out, 4 y_proj, 7 the whole post wave (list in/out included);
within the walk (associate): 12 is_equal + ballots, 9 the serial walk, 10 compaction, 11 append.  Read the SHARES (stamps serialise
the wave).   python tools/poststamps.py [scans] [calls]"""
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
from lidar_slam_amd.device import Context  # noqa: E402
from lidar_slam_amd.pipeline import ScanPipeline  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
calls = int(sys.argv[2]) if len(sys.argv) > 2 else 6
ctx = Context(0)
b, ukf = make_workload(list(range(S)), 720, 20)
nc = int(b["scan_chunk_off"][-1])
pipe = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.arange(S, dtype=np.uint32),
                    lmk_capacity=64, want_yproj=True, ukf=ukf)
dbg = ctx.empty((nc + S, 16), np.uint64)
names = {1: "records_in", 2: "walk", 12: "is_equal", 9: "walk_loop", 10: "compaction", 11: "append",
         3: "records_out", 4: "y_proj", 7: "post_wave"}


def summary(d, n):
    post = d[nc:nc + S].astype(np.float64) / n
    out = {nm: round(float(post[:, k].mean()), 1) for k, nm in names.items()}
    tot = post[:, 7].mean() or post[:, [1, 2, 3, 4]].sum(1).mean()
    out["shares"] = {nm: round(float(post[:, k].mean() / tot), 3) for k, nm in names.items() if k != 7}
    t0 = d[nc:nc + S, 8].astype(np.int64)
    out["start_spread_cycles"] = int(t0.max() - t0.min())
    return out


pipe.run()
res = {}
# alone: the post pass of the last call, nothing beside it
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
pipe.run_landmarks_only()
ctx.sync()
L.lslam_debug_set_stamps(None)
res["alone"] = summary(dbg.download(), 1)
# in the pipeline: calls back to back (each post beside the next call's producer, the last alone)
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
for _ in range(calls):
    pipe.run(sync=False)
ctx.sync()
L.lslam_debug_set_stamps(None)
res["pipeline_mean_per_call"] = summary(dbg.download(), calls)
print(json.dumps(res))
