"""Post-pass cost split on C3 (4096 scans): association walk + y_proj
(lslam_landmarks) and the UKF step (lslam_ukf_step) timed alone with HIP events.

python tools/postprobe.py
"""
import json
import os
import sys

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from bench import make_workload  # noqa: E402
from lidar_slam_amd import _lib  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

ctx = Context(0)
ids = list(range(4096))
b, ukf = make_workload(ids, 720, 20)
out = {}
for yp in (True, False):
    p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                        ukf=ukf, hyp="philox", want_yproj=yp)
    p.run()
    for name, fn, k in (("assoc" + ("_yproj" if yp else ""), p.run_landmarks_only, _lib.K_LANDMARK),
                        ("ukf", p.run_ukf_only, _lib.K_UKF)):
        ctx.set_timing(True)
        ctx.timing_reset()
        for _ in range(10):
            p.reset_state()
            fn(sync=False)
        ctx.sync()
        ms, n = ctx.timing(k)
        ctx.set_timing(False)
        out[name + "_ms"] = round(ms / n, 4)
print(json.dumps(out))

# fused post pass = pipeline (philox: chunk + post) - ransac only (chunk)
p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                    ukf=ukf, hyp="philox")
res = {}
for name, fn in (("pipeline", p.run), ("ransac", p.run_ransac_only)):
    fn()
    ctx.set_timing(True, [_lib.K_PIPELINE])
    ctx.timing_reset()
    for _ in range(10):
        fn(sync=False)
    ctx.sync()
    ms, n = ctx.timing(_lib.K_PIPELINE)
    ctx.set_timing(False)
    res[name] = ms / n
print(json.dumps({"philox_pipeline_ms": round(res["pipeline"], 4), "philox_ransac_ms": round(res["ransac"], 4),
                  "fused_post_ms": round(res["pipeline"] - res["ransac"], 4)}))
