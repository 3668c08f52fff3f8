"""Time the parity-stream producer alone (lslam_hyp_mt19937) over batch sizes.

python tools/drawsbench.py [S ...]
"""
import ctypes as C, json, os, sys
import numpy as np
sys.path.insert(0, os.getcwd())
from bench import make_workload
from lidar_slam_amd import _lib
from lidar_slam_amd.device import Context
ctx = Context(0)
out = {}
SIZES = [int(x) for x in sys.argv[1:]] or [256, 1024, 2048, 4096, 8192]
for S in SIZES:
    ids = list(range(S))
    b, _ = make_workload(ids, 720, 20)
    keep = []
    def d(a):
        x = ctx.to_device(a); keep.append(x); return x.addr
    bb = _lib.ScanBatch()
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
    bb.n_scans, bb.n_chunks, bb.n_points = len(ids), int(sco[-1]), int(cpo[-1])
    bb.max_chunk_points, bb.max_scan_chunks = int(np.diff(cpo).max()), int(np.diff(sco).max())
    bb.scan_chunk_off, bb.chunk_pt_off, bb.seeds = d(sco), d(cpo), d(np.array(ids, np.uint32))
    dr = ctx.empty((int(sco[-1]), 101, 2), np.int32)
    bb.draws_out = dr.addr
    L = _lib.load()
    fn = lambda: _lib.check(L.lslam_hyp_mt19937(ctx.handle, C.byref(bb), 100))
    fn(); ctx.sync()
    ctx.set_timing(True); ctx.timing_reset()
    for _ in range(5): fn()
    ctx.sync()
    ms, n = ctx.timing(_lib.K_HYP)
    rms, rn = ctx.timing(_lib.K_RNG)
    ctx.set_timing(False)
    out[S] = {"hyp_ms": round(ms / n, 4), "rng_ms": round(rms / max(rn, 1), 4)}
print(json.dumps(out))
