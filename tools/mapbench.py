"""Landmark-map mode throughput (LSLAM_UKF_MAP, lidar_slam_amd/slam.py).

python tools/mapbench.py [--robots 4096] [--steps 20] [--warmup 3] [--unique 8] [--hyp mt19937]

R robots drive the trajectories of synth.trajectory; every step is one
720-point revolution per robot (7x100 + 20 chunks): RANSAC with the chained
MT19937 stream, world-frame association against the robot's persistent map,
UKF predict + update with the matched chunks, all in one lslam_scan_pipeline
launch.  Inputs of `unique` consecutive steps are staged in HBM first and
cycled (the map and the filter state keep evolving); the timed region is K
asynchronous steps bracketed by device syncs.
"""
from __future__ import annotations

import argparse
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--robots", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    ap.add_argument("--unique", type=int, default=8)
    ap.add_argument("--hyp", default="mt19937")
    ap.add_argument("--reference-tolerances", action="store_true",
                    help="landmarking.py:4-6 tolerances (almost no re-identification)")
    args = ap.parse_args()
    from lidar_slam_amd import _lib, synth
    from lidar_slam_amd.device import Context
    from lidar_slam_amd.slam import LandmarkMap

    R = args.robots
    robots = list(range(R))
    t0 = time.perf_counter()
    poses = synth.trajectory(robots, args.unique)
    revs = [synth.revolutions_at(poses[k + 1], k, robots) for k in range(args.unique)]
    gen_s = time.perf_counter() - t0
    ctx = Context(0)
    tol = {} if args.reference_tolerances else dict(tol_b=100.0, tol_dist=1000.0)
    rng = np.random.default_rng(9)
    x0 = poses[0] + rng.normal(0, [3.0, 3.0, 0.01], (R, 3))
    lm = LandmarkMap(ctx, R, lmk_capacity=256, seeds=robots, x0=x0, P0=np.diag([25.0, 25.0, 1e-4]),
                     R_diag=[25.0, 1e-4] * 8, hyp=args.hyp, **tol)
    staged = [lm.upload(r["xy"], r["scan_chunk_off"], r["chunk_pt_off"]) for r in revs]
    lm.step(staged[0], u=np.tile([2.0, 2.5], (R, 1)))
    for k in range(1, args.warmup):
        lm.step(staged[k % args.unique], sync=False)
    ctx.sync()
    t0 = time.perf_counter()
    for k in range(args.steps):
        lm.step(staged[(args.warmup + k) % args.unique], sync=False)
    ctx.sync()
    dt = time.perf_counter() - t0
    res = lm.results()
    flags = res["models"]["flags"]
    out = {"metric": "map-mode scans/s (RANSAC + world-frame association + UKF with map measurements)",
           "value": round(R * args.steps / dt, 1), "unit": "scans/s", "ms_per_step": round(1e3 * dt / args.steps, 4),
           "robots": R, "steps": args.steps, "warmup": args.warmup, "unique_inputs": args.unique, "hyp": args.hyp,
           "tolerances": "reference" if args.reference_tolerances else "tol_b=100, tol_dist=1000",
           "matched_frac_last_step": round(float(np.mean((flags & _lib.MATCHED) != 0)), 4),
           "mean_map_size": round(float(np.mean(res["lmk_count"])), 2),
           "input_gen_s": round(gen_s, 1)}
    print(json.dumps(out))


if __name__ == "__main__":
    main()
