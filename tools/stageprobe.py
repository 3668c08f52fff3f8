"""C3 step time with parts of the pipeline switched off (parity mode): which stage sets the step?

python tools/stageprobe.py
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
variants = {
    "full (assoc+ukf)": dict(lmk_capacity=32, ukf=ukf),
    "assoc only": dict(lmk_capacity=32),
    "ukf only": dict(ukf=ukf),
    "ransac only": dict(),
}
for name, kw in variants.items():
    p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), **kw)
    fn = p.run if kw else p.run_ransac_only
    for _ in range(3):
        fn(sync=False)
    ctx.sync()
    t = time.perf_counter()
    for _ in range(20):
        fn(sync=False)
    ctx.sync()
    print("%-18s %.4f ms" % (name, (time.perf_counter() - t) / 20 * 1e3), flush=True)
