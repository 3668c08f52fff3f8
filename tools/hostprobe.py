"""Host-side duration of each lslam_scan_pipeline call (sync=False) on C3: a
call that blocks for about a step's length means the host, not the GPU, paces
the stream of calls.

python tools/hostprobe.py [--no-timing]   (--no-timing: only the pass without HIP-event timers,
                                          e.g. under rocprofv3 --kernel-trace for a timeline)
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

ctx = Context(0)
ids = list(range(4096))
b, ukf = make_workload(ids, 720, 20)
p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                    ukf=ukf)
for timing in ((False,) if "--no-timing" in sys.argv else (False, True)):
    ctx.set_timing(timing)
    for _ in range(3):
        p.run(sync=False)
    ctx.sync()
    t0 = time.perf_counter()
    d = []
    for _ in range(20):
        t = time.perf_counter()
        p.run(sync=False)
        d.append((time.perf_counter() - t) * 1e3)
    t1 = time.perf_counter()
    ctx.sync()
    t2 = time.perf_counter()
    print("timing=%d host ms per call: %s | enqueue total %.3f ms, drain %.3f ms, step %.4f ms" % (
        timing, " ".join("%.3f" % x for x in d), (t1 - t0) * 1e3, (t2 - t1) * 1e3, (t2 - t0) / 20 * 1e3), flush=True)
