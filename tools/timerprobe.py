"""Step time of the C3 pipeline with HIP-event timing off, on for every kernel,
and on for one kernel id at a time (timing events between kernels of the two
streams change how they overlap).

python tools/timerprobe.py
"""
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_workload  # noqa: E402
from lidar_slam_amd import _lib  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

ctx = Context(0)
ids = list(range(4096))
b, ukf = make_workload(ids, 720, 20)
p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                    ukf=ukf)


def run(kernels, on):
    ctx.set_timing(on, kernels)
    ctx.timing_reset()
    for _ in range(3):
        p.run(sync=False)
    ctx.sync()
    t = time.perf_counter()
    for _ in range(20):
        p.run(sync=False)
    ctx.sync()
    dt = (time.perf_counter() - t) / 20 * 1e3
    ctx.set_timing(False)
    return dt


for rep in range(2):
    row = {"off": run(None, False), "all": run(None, True)}
    for name, k in (("pipeline", _lib.K_PIPELINE), ("rng", _lib.K_RNG), ("consensus", _lib.K_CONSENSUS)):
        row[name] = run([k], True)
    print(" ".join("%s %.4f" % kv for kv in row.items()), flush=True)
