"""Per-phase kernel timings on the C3 workload (HIP events on the lib stream).

python tools/microbench.py [--scans 4096] [--reps 10]
Prints one JSON object: ms per launch for the fused pipeline (mt19937 /
philox, with and without UKF), RANSAC-only, the MT19937 draw generator alone,
and the UKF alone.
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


BREAKDOWN = {}


def timed(ctx, fn, kid, reps, tag=None):
    fn()
    ctx.sync()
    ctx.set_timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        fn()
    ctx.sync()
    ms, n = ctx.timing(kid)
    if tag:
        for name, k in (("rng", _lib.K_RNG), ("consensus", _lib.K_CONSENSUS)):
            m2, n2 = ctx.timing(k)
            if n2:
                BREAKDOWN["%s_%s_ms" % (tag, name)] = m2 / n2
    ctx.set_timing(False)
    return ms / max(n, 1)


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=10)
    ap.add_argument("--beams", type=int, default=720)
    args = ap.parse_args()
    ctx = Context(0)
    ids = list(range(args.scans))
    b, ukf = make_workload(ids, args.beams, 20)
    res = {"scans": args.scans}
    for hyp in ("mt19937", "philox"):
        for with_ukf in (True, False):
            p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), hyp=hyp,
                                lmk_capacity=32, ukf=ukf if with_ukf else None)
            tag = "pipeline_%s%s" % (hyp, "_ukf" if with_ukf else "")
            res[tag + "_ms"] = timed(ctx, lambda: p.run(sync=False), _lib.K_PIPELINE, args.reps, tag)
        p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), hyp=hyp)
        res["ransac_only_%s_ms" % hyp] = timed(ctx, lambda: p.run_ransac_only(sync=False), _lib.K_PIPELINE, args.reps)
    p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), ukf=ukf)
    res["ukf_only_ms"] = timed(ctx, lambda: p.run_ukf_only(sync=False), _lib.K_UKF, args.reps)
    # draws alone
    import ctypes as C
    keep = []

    def d(a):
        x = ctx.to_device(a)
        keep.append(x)
        return x.addr

    bb = _lib.ScanBatch()
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    bb.n_scans, bb.n_chunks, bb.n_points = len(ids), int(sco[-1]), int(cpo[-1])
    bb.max_chunk_points, bb.max_scan_chunks = int(np.diff(cpo).max()), int(np.diff(sco).max())
    bb.scan_chunk_off, bb.chunk_pt_off, bb.seeds = d(sco), d(cpo), d(np.array(ids, np.uint32))
    dr = ctx.empty((int(sco[-1]), 101, 2), np.int32)
    bb.draws_out = dr.addr
    res["mt19937_draws_only_ms"] = timed(
        ctx, lambda: _lib.check(_lib.load().lslam_hyp_mt19937(ctx.handle, C.byref(bb), 100)), _lib.K_HYP, args.reps)
    res.update(BREAKDOWN)
    print(json.dumps({k: (round(v, 4) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
