"""Diagnostic: wave census of the C3 pipeline (diagnostic build liblidarslam_census.so).

Every wave of the producer (parsers, helpers) and of the consumer kernels (resolve,
consensus, fix-up, post pass, UKF) writes {kernel, call, HW_ID, XCC_ID, entry and exit
s_memrealtime} (WaveCensus in csrc/lidarslam.hip).  For each kernel of the census calls
this prints when its waves became resident (start offsets from the dispatch's first
wave), how long they lived, how many were resident at once, and how the parsers were
placed (parsers per SIMD, late workgroups).  The s_memrealtime clock is 100 MHz.

  python tools/census.py [--steps K] [--warmup W] [--scans S] [--out gpurun_out/census.npz]
LSLAM_MT_SPECULATE=0 applies as usual.
"""
import argparse
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import _lib  # noqa: E402

NAMES = {1: "rng_parser", 2: "rng_helper", 3: "resolve", 4: "chunk", 5: "fixup", 6: "post", 7: "ukf"}


def decode(rec):
    kid = (rec[:, 0] & 0xff).astype(np.int64)
    call = ((rec[:, 0] >> 8) & 0xffff).astype(np.int64)
    hw = ((rec[:, 0] >> 24) & 0xffffffff).astype(np.int64)
    xcc = ((rec[:, 0] >> 56) & 0xff).astype(np.int64)
    simd = (hw >> 4) & 3
    cu = (hw >> 8) & 15
    sh = (hw >> 12) & 1
    se = (hw >> 13) & 7
    queue = (hw >> 24) & 7
    simd_key = (((xcc * 8 + se) * 2 + sh) * 16 + cu) * 4 + simd
    return dict(kid=kid, call=call, simd_key=simd_key, cu_key=simd_key // 4, queue=queue,
                t0=rec[:, 1].astype(np.int64), t1=rec[:, 2].astype(np.int64))


def resident(t0, t1):
    ev = np.concatenate([np.stack([t0, np.ones_like(t0)], 1), np.stack([t1, -np.ones_like(t1)], 1)])
    ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
    return int(np.cumsum(ev[:, 1]).max())


def summarise(d, origin):
    out = {}
    for call in np.unique(d["call"]):
        for kid in np.unique(d["kid"]):
            m = (d["call"] == call) & (d["kid"] == kid)
            if not m.any():
                continue
            t0, t1 = d["t0"][m], d["t1"][m]
            life = (t1 - t0) / 100.0
            st = (t0 - t0.min()) / 100.0
            e = dict(waves=int(m.sum()), start_us=round((t0.min() - origin) / 100.0, 1),
                     end_us=round((t1.max() - origin) / 100.0, 1), span_us=round((t1.max() - t0.min()) / 100.0, 1),
                     life_p50_p90_max=[round(float(np.percentile(life, q)), 1) for q in (50, 90)] + [round(float(life.max()), 1)],
                     start_off_p50_p90_max=[round(float(np.percentile(st, q)), 1) for q in (50, 90)] + [round(float(st.max()), 1)],
                     max_resident=resident(t0, t1), queues=sorted(set(int(q) for q in d["queue"][m])))
            sk = d["simd_key"][m]
            _, per = np.unique(sk, return_counts=True)
            e["simds_used"] = int(len(per))
            e["waves_per_simd_max"] = int(per.max())
            out["call%d/%s" % (call, NAMES.get(int(kid), kid))] = e
    return out


def parser_placement(d):
    """per call: parsers per SIMD histogram, and the start-time spread of the producer's waves"""
    res = {}
    for call in np.unique(d["call"]):
        m = (d["call"] == call) & (d["kid"] == 1)
        if not m.any():
            continue
        sk = d["simd_key"][m]
        _, per = np.unique(sk, return_counts=True)
        hist = np.bincount(per)
        t0 = d["t0"][m]
        life = (d["t1"][m] - t0) / 100.0
        late = (t0 - t0.min()) / 100.0
        # parsers per SIMD vs their lifetime
        load = dict(zip(*np.unique(sk, return_counts=True)))
        ld = np.array([load[k] for k in sk])
        res["call%d" % call] = dict(
            parsers_per_simd_hist={int(i): int(v) for i, v in enumerate(hist) if v},
            late_start_us_p50_p99_max=[round(float(np.percentile(late, 50)), 1),
                                       round(float(np.percentile(late, 99)), 1), round(float(late.max()), 1)],
            n_late_over_20us=int((late > 20).sum()),
            life_by_simd_load={int(L): [int((ld == L).sum()), round(float(np.median(life[ld == L])), 1),
                                        round(float(life[ld == L].max()), 1)] for L in np.unique(ld)})
    return res


def main():
    ap = argparse.ArgumentParser()
    ap.add_argument("--steps", type=int, default=4)
    ap.add_argument("--warmup", type=int, default=4)
    ap.add_argument("--scans", type=int, default=4096)
    ap.add_argument("--out", default=os.path.join(ROOT, "gpurun_out", "census.npz"))
    ap.add_argument("--lib", default="census", choices=["census", "stamps"],
                    help="liblidarslam_census.so (wave census only: production timing) or _stamps.so")
    args = ap.parse_args()
    _lib.LIB_PATH = os.path.join(ROOT, "lidar_slam_amd", "liblidarslam_%s.so" % args.lib)
    L = _lib.load()
    L.lslam_debug_set_census.argtypes = [C.c_void_p, C.c_void_p, C.c_uint]
    L.lslam_debug_set_census.restype = C.c_int
    from bench import make_workload
    from lidar_slam_amd.device import Context
    from lidar_slam_amd.pipeline import ScanPipeline

    ctx = Context(0)
    S = args.scans
    ids = list(range(S))
    b, ukf = make_workload(ids, 720, 20)
    pipe = ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.array(ids, np.uint32),
                        max_trials=100, lmk_capacity=64, want_yproj=True, ukf=ukf)
    for _ in range(args.warmup):
        pipe.run(sync=False)
    ctx.sync()
    cap = 256 * 1024 * (args.steps + 1)
    buf = ctx.empty((cap, 3), np.uint64)
    cnt = ctx.empty((256,), np.uint32)
    cnt.fill_zero()
    if L.lslam_debug_set_census(C.c_void_p(buf.addr), C.c_void_p(cnt.addr), cap) != 0:
        raise SystemExit("census not supported by this build")
    for _ in range(args.steps):
        pipe.run(sync=False)
    ctx.sync()
    L.lslam_debug_set_census(None, None, 0)
    per = cap // 256
    counts = cnt.download().astype(np.int64)
    n = int(counts.sum())
    if (counts > per).any():
        raise SystemExit("census buckets overflowed: raise the capacity")
    allrec = buf.download().reshape(256, per, 3)
    rec = np.concatenate([allrec[b, :counts[b]] for b in range(256)])
    d = decode(rec)
    origin = int(d["t0"].min())
    os.makedirs(os.path.dirname(args.out), exist_ok=True)
    np.savez_compressed(args.out, rec=rec)
    out = dict(records=n, capacity=cap, env={k: v for k, v in os.environ.items() if k.startswith("LSLAM_")},
               kernels=summarise(d, origin), parsers=parser_placement(d))
    print(json.dumps(out, indent=1))


if __name__ == "__main__":
    main()
