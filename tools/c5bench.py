"""C5 (BASELINE configs[4]) dense-return stress: 4096-point scans, each ONE
RANSAC call of 2048 hypotheses, plus the UKF with L = 200 landmarks (dim_z 400).

python tools/c5bench.py [--scans 1024] [--reps 3] [--hyp both|mt19937|philox]

Prints one JSON object per hypothesis source: ms per pipeline call, scans/s,
the consensus kernel's ms and FP64 rate (12 flop per point-hypothesis
evaluation) against the 78.6 TF/s vector peak, and the parity
producer's ms (mt19937).
"""
import argparse
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_workload  # noqa: E402
from lidar_slam_amd import _lib  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

FP64_PEAK = 78.6e12


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=1024)
    ap.add_argument("--points", type=int, default=4096)
    ap.add_argument("--trials", type=int, default=2048)
    ap.add_argument("--landmarks", type=int, default=200)
    ap.add_argument("--reps", type=int, default=3)
    ap.add_argument("--hyp", default="both")
    ap.add_argument("--budget-gib", type=float, default=0.0,
                    help="producer steps scratch per slot (0: the library default, 2 GiB)")
    args = ap.parse_args()
    ctx = Context(0)
    ctx.set_steps_budget(int(args.budget_gib * (1 << 30)))
    S, Np, T = args.scans, args.points, args.trials
    ids = list(range(S))
    b, ukf = make_workload(ids, Np, args.landmarks)
    sco = np.arange(S + 1, dtype=np.int32)            # one chunk per scan
    cpo = (np.arange(S + 1) * Np).astype(np.int32)
    hyps = ("mt19937", "philox") if args.hyp == "both" else (args.hyp,)
    for hyp in hyps:
        p = pl.ScanPipeline(ctx, b["xy"], sco, cpo, seeds=np.array(ids), hyp=hyp, max_trials=T,
                            lmk_capacity=8, ukf=ukf)
        p.run()
        ctx.set_timing(True)
        ctx.timing_reset()
        for _ in range(args.reps):
            p.run(sync=False)
        ctx.sync()
        res = {"config": "C5", "hyp": hyp, "scans": S, "points": Np, "trials": T, "landmarks": args.landmarks}
        ms, n = ctx.timing(_lib.K_PIPELINE)
        res["pipeline_ms"] = ms / max(n, 1)
        res["scans_per_s"] = S / res["pipeline_ms"] * 1e3
        for name, k in (("consensus", _lib.K_CONSENSUS), ("rng", _lib.K_RNG)):
            m2, n2 = ctx.timing(k)
            if n2:
                res[name + "_ms"] = m2 / args.reps  # per call (the producer may run in epochs)
                res[name + "_launches_per_call"] = n2 / args.reps
        if hyp == "mt19937":  # two slots of min(budget, all steps) bytes (u16 steps)
            full = (T + 1) * S * Np * 2
            budget = args.budget_gib * (1 << 30) if args.budget_gib > 0 else 2 << 30
            per_draw = S * Np * 2
            slot = full if full <= budget else max(1, int(budget // per_draw)) * per_draw
            res["steps_scratch_gb"] = 2 * slot / 1e9
        ctx.set_timing(False)
        if "consensus_ms" in res:
            flops = 12.0 * Np * T * S
            res["consensus_tflops"] = flops / res["consensus_ms"] / 1e9
            res["consensus_frac_fp64"] = res["consensus_tflops"] * 1e12 / FP64_PEAK
        print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}), flush=True)


if __name__ == "__main__":
    main()
