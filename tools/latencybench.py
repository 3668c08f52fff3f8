"""Latency of the drop-in entry points (live use: one sensor, one revolution at a time).

python tools/latencybench.py [--revs 50]

landmark_extraction per 100-point chunk (ransac_functions.py:15 drop-in, numpy's
global RNG in and out), process_revolution per 720-point revolution (8 chunks,
one pipeline call), and LandmarkMap.step for one robot.  Host wall-clock per
call, median over the runs after a warmup.
"""
import argparse
import json
import os
import sys
import time

import numpy as np

sys.path.insert(0, os.path.dirname(os.path.dirname(os.path.abspath(__file__))))
from lidar_slam_amd import ransac_functions as rf  # noqa: E402
from lidar_slam_amd import synth  # noqa: E402


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--revs", type=int, default=50)
    args = ap.parse_args()
    b = synth.make_batch(list(range(args.revs)))
    sco, cpo, xy = b["scan_chunk_off"], b["chunk_pt_off"], b["xy"]
    revs = [[xy[cpo[c]:cpo[c + 1]].tolist() for c in range(sco[s], sco[s + 1])] for s in range(args.revs)]
    out = {}
    # per chunk
    np.random.seed(1)
    lm, num, t = [], 0, []
    for r in revs:
        for ch in r:
            t0 = time.perf_counter()
            q, fitted, new = rf.landmark_extraction([ch], num, lm)
            t.append(time.perf_counter() - t0)
            if new:
                lm.append(fitted)
            num += 1
    out["landmark_extraction_ms"] = round(1e3 * float(np.median(t[8:])), 3)
    # per revolution
    np.random.seed(1)
    lm, num, t = [], 0, []
    for r in revs:
        t0 = time.perf_counter()
        pts, num = rf.process_revolution(r, num, lm)
        t.append(time.perf_counter() - t0)
    out["process_revolution_ms"] = round(1e3 * float(np.median(t[2:])), 3)
    # map step, one robot
    from lidar_slam_amd.device import Context
    from lidar_slam_amd.slam import LandmarkMap
    ctx = Context(0)
    poses = synth.trajectory([0], args.revs)
    m = LandmarkMap(ctx, 1, lmk_capacity=256, x0=poses[0], P0=np.diag([25.0, 25.0, 1e-4]), R_diag=[25.0, 1e-4] * 8)
    t = []
    for k in range(args.revs):
        rev = synth.revolutions_at(poses[k + 1], k, [0])
        t0 = time.perf_counter()
        m.step(rev["xy"], rev["scan_chunk_off"], rev["chunk_pt_off"], u=[[2.0, 2.5]])
        t.append(time.perf_counter() - t0)
    out["map_step_1robot_ms"] = round(1e3 * float(np.median(t[2:])), 3)
    print(json.dumps(out))


if __name__ == "__main__":
    main()
