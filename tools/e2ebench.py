"""End-to-end C3 rate with the PCIe copies inside the timed loop (the
kernel-only rate is bench.py's `value`; this is the host-buffer rate beside it).

python tools/e2ebench.py [--scans 4096] [--steps 20]

Per step, on the context's stream: (a) xy: pinned host xy (16 B/point) -> HBM,
the pipeline, then mask + chunk models + y_proj back to pinned host memory;
(b) packets: the raw RPLidar express stream (84 B per 32 measures) -> HBM,
packets -> revolutions on the device, the pipeline, the same outputs back.
"""
import argparse
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)

from bench import make_workload  # noqa: E402
from lidar_slam_amd import _lib, synth  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402
from lidar_slam_amd.express import ExpressRevolutions  # noqa: E402
from lidar_slam_amd.pipeline import ScanPipeline  # noqa: E402


def pinned(nbytes):
    p = C.c_void_p()
    _lib.check(_lib.load().lslam_host_alloc(int(nbytes), C.byref(p)), "lslam_host_alloc")
    return p


def run_loop(ctx, pipe, h2d, outs, steps, warmup):
    L = _lib.load()

    def step():
        for dst, src, n in h2d:
            _lib.check(L.lslam_h2d(ctx.handle, dst, src, n), "h2d")
        for pre in getattr(pipe, "pre", []):
            pre()
        pipe.run(sync=False)
        for dst, src, n in outs:
            _lib.check(L.lslam_d2h(ctx.handle, dst, src, n), "d2h")

    for _ in range(warmup):
        step()
    ctx.sync()
    t = time.perf_counter()
    for _ in range(steps):
        step()
    ctx.sync()
    return (time.perf_counter() - t) / steps


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--scans", type=int, default=4096)
    ap.add_argument("--steps", type=int, default=20)
    ap.add_argument("--warmup", type=int, default=3)
    args = ap.parse_args()
    ctx = Context(0)
    S = args.scans
    ids = list(range(S))
    b, ukf = make_workload(ids, 720, 20)
    res = {"scans": S}
    # (a) xy in, outputs out
    pipe = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids), lmk_capacity=32,
                        ukf=ukf)
    P, Cn = pipe.P, pipe.C
    hx = pinned(P * 16)
    C.memmove(hx, b["xy"].ctypes.data, P * 16)
    ho = [pinned(n) for n in (P, Cn * 112, P * 8)]
    outs = [(ho[0], pipe.mask.ptr, P), (ho[1], pipe.models.ptr, Cn * 112), (ho[2], pipe.yproj.ptr, P * 8)]
    dt = run_loop(ctx, pipe, [(C.c_void_p(pipe.batch.xy), hx, P * 16)], outs, args.steps, args.warmup)
    in_b, out_b = P * 16, P + Cn * 112 + P * 8
    res["xy"] = {"ms_per_step": round(dt * 1e3, 4), "scans_per_s": round(S / dt, 1), "h2d_bytes": in_b,
                 "d2h_bytes": out_b}
    # (b) express packets in: 22.5 packets per revolution of 720 measures
    M = int(S * 22.5) + 2
    pk = synth.express_packets(M, seed=5)
    rv = ExpressRevolutions(ctx, M)
    rv.run(pk)
    n = rv.n_scans
    pipe2 = ScanPipeline(ctx, rv.xy, rv.scan_chunk_off, rv.chunk_pt_off, seeds=np.arange(n), lmk_capacity=32)
    hp = pinned(pk.nbytes)
    C.memmove(hp, pk.ctypes.data, pk.nbytes)
    P2, C2 = pipe2.P, pipe2.C
    ho2 = [pinned(x) for x in (P2, C2 * 112, P2 * 8)]
    outs2 = [(ho2[0], pipe2.mask.ptr, P2), (ho2[1], pipe2.models.ptr, C2 * 112), (ho2[2], pipe2.yproj.ptr, P2 * 8)]

    def express_kernels():
        _lib.check(_lib.load().lslam_express_scans(ctx.handle, rv.d_packets.addr, M, 0, C.byref(rv.out)),
                   "lslam_express_scans")

    pipe2.pre = [express_kernels]
    dt2 = run_loop(ctx, pipe2, [(rv.d_packets.ptr, hp, pk.nbytes)], outs2, args.steps, args.warmup)
    res["packets"] = {"ms_per_step": round(dt2 * 1e3, 4), "scans_per_s": round(n / dt2, 1), "revolutions": n,
                      "h2d_bytes": int(pk.nbytes), "d2h_bytes": P2 + C2 * 112 + P2 * 8,
                      "note": "association, no UKF (the packet stream carries no odometry)"}
    print(json.dumps(res))


if __name__ == "__main__":
    main()
