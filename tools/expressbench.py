"""Express-scan codec throughput (HIP events on the lib stream).

python tools/expressbench.py [--revs 4096] [--reps 20]

A synthetic stream of ~22.5 packets per revolution (720 measures, the C3 scan
size), resident in HBM.  Prints one JSON object:
  * scans_*: lslam_express_scans (flags, ranks, revolution CSR, decode + A1 +
    scatter), whole call and the scatter kernel alone;
  * decode_*: lslam_express_decode with every measure-level output.
Algorithmic bytes: scans = packets read once (84 B) + xy written (16 B per kept
measure) + the CSR; decode = 84 B in + 32 x 34 B out per packet.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from lidar_slam_amd import _lib, synth  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402
from lidar_slam_amd.express import ExpressRevolutions  # noqa: E402

HBM_PEAK_GBS = 8000.0


def timed(ctx, fn, kids, reps):
    fn()
    ctx.sync()
    ctx.set_timing(True)
    ctx.timing_reset()
    for _ in range(reps):
        fn()
    ctx.sync()
    out = {}
    for k in kids:
        ms, n = ctx.timing(k)
        out[k] = ms / max(n, 1)
    ctx.set_timing(False)
    return out


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--revs", type=int, default=4096)
    ap.add_argument("--reps", type=int, default=20)
    args = ap.parse_args()
    ctx = Context(0)
    M = int(args.revs * 22.5) + 1
    pk = synth.express_packets(M, seed=1, scan_id=1)
    rv = ExpressRevolutions(ctx, M)
    rv.upload(pk)
    t = timed(ctx, lambda: rv.launch(skip=0), (_lib.K_EXPRESS, _lib.K_EXPRESS_SCATTER), args.reps)
    rv.fetch()
    res = {"packets": M, "revolutions": rv.n_scans, "points": rv.n_points, "chunks": rv.n_chunks}
    b_scans = 84 * M + 16 * rv.n_points + 4 * (rv.n_scans + rv.n_chunks + 2)
    b_scatter = 84 * M + 16 * rv.n_points
    res["scans_ms"] = t[_lib.K_EXPRESS]
    res["scans_scatter_ms"] = t[_lib.K_EXPRESS_SCATTER]
    res["scans_GBps"] = b_scans / t[_lib.K_EXPRESS] / 1e6
    res["scatter_GBps"] = b_scatter / t[_lib.K_EXPRESS_SCATTER] / 1e6
    res["scans_revs_per_s"] = rv.n_scans / t[_lib.K_EXPRESS] * 1e3
    # measure-level decode, every output
    n = (M - 1) * 32
    outs = {k: ctx.empty(n * w, np.uint8) for k, w in (("angle_deg", 8), ("dist_mm", 8), ("new_scan", 1),
                                                        ("valid", 1), ("xy", 16))}
    outs["pkt_valid"] = ctx.empty(M, np.uint8)
    m = _lib.ExpressMeasures()
    for k, a in outs.items():
        setattr(m, k, a.addr)
    L = _lib.load()
    t2 = timed(ctx, lambda: _lib.check(L.lslam_express_decode(ctx.handle, rv.d_packets.addr, M, C.byref(m))),
               (_lib.K_EXPRESS,), args.reps)
    b_dec = 84 * M + 34 * n + M
    res["decode_ms"] = t2[_lib.K_EXPRESS]
    res["decode_GBps"] = b_dec / t2[_lib.K_EXPRESS] / 1e6
    for k in ("scans_GBps", "scatter_GBps", "decode_GBps"):
        res[k.replace("GBps", "frac")] = res[k] / HBM_PEAK_GBS
    print(json.dumps({k: (round(v, 5) if isinstance(v, float) else v) for k, v in res.items()}))


if __name__ == "__main__":
    main()
