"""Experiment: does the consensus + post pass of step k hide under the MT
producer of step k+1 when they run on two streams?  (Two contexts: ctx1 runs
lslam_hyp_mt19937 into a double-buffered draw array, ctx2 runs the explicit-
hypothesis pipeline on the previous step's draws; both synced per step.)"""
import ctypes as C
import json
import os
import sys
import time

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from bench import make_workload  # noqa: E402
from lidar_slam_amd import _lib  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402
from lidar_slam_amd.pipeline import ScanPipeline  # noqa: E402

S = 4096
ctx1, ctx2 = Context(0), Context(0)
ids = list(range(S))
b, ukf = make_workload(ids, 720, 20)
sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
Cn = int(sco[-1])
keep = []


def d(a):
    x = ctx1.to_device(a)
    keep.append(x)
    return x.addr


hb = _lib.ScanBatch()
hb.n_scans, hb.n_chunks, hb.n_points = S, Cn, int(cpo[-1])
hb.max_chunk_points, hb.max_scan_chunks = int(np.diff(cpo).max()), int(np.diff(sco).max())
hb.scan_chunk_off, hb.chunk_pt_off, hb.seeds = d(sco), d(cpo), d(np.array(ids, np.uint32))
bufs = [ctx1.empty((Cn, 101, 2), np.int32) for _ in range(2)]
dummy = np.zeros((Cn, 101, 2), np.int32)
dummy[..., 1] = 1
pipes = []
for k in range(2):
    p = ScanPipeline(ctx2, b["xy"], sco, cpo, hyp="explicit", hyp_draws=dummy, lmk_capacity=32, ukf=ukf)
    p.batch.hyp = bufs[k].addr
    pipes.append(p)
L = _lib.load()


def rng(k):
    hb.draws_out = bufs[k % 2].addr
    _lib.check(L.lslam_hyp_mt19937(ctx1.handle, C.byref(hb), 100))


def cons(k):
    pipes[k % 2].run(sync=False)


res = {}
for mode in ("serial", "overlap"):
    for rep in range(2):
        rng(0)
        ctx1.sync()
        t0 = time.perf_counter()
        K = 20
        for k in range(K):
            if mode == "serial":
                rng(k + 1)
                ctx1.sync()
                cons(k)
                ctx2.sync()
            else:
                rng(k + 1)
                cons(k)
                ctx1.sync()
                ctx2.sync()
        dt = (time.perf_counter() - t0) / K * 1e3
    res[mode + "_ms_per_step"] = round(dt, 4)
print(json.dumps(res))
