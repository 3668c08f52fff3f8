"""Diagnostic: per-phase cycle shares of the MT19937 parser wave (s_memtime stamps).

Uses the separate diagnostic build lidar_slam_amd/liblidarslam_stamps.so
(python -m lidar_slam_amd.build --stamps); the product library has no stamps.  Read the
SHARES, not the absolute time (stamps serialise the wave).
    python tools/stamps.py [scans] [c5]   (c5: 4096-point one-chunk scans, 2048 trials: mask mode)"""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.path.join(ROOT, "lidar_slam_amd", "liblidarslam_stamps.so")
L = _lib.load()
L.lslam_debug_set_stamps.argtypes = [C.c_void_p]
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
C5 = len(sys.argv) > 2 and sys.argv[2] == "c5"  # C5: one 4096-point chunk per scan, 2048 trials (mask mode, epochs)
ctx = Context(0)
if C5:
    sco = np.arange(S + 1, dtype=np.int32)
    cpo = (np.arange(S + 1) * 4096).astype(np.int32)
else:
    b, _ = make_workload(list(range(S)), 720, 20)
    sco, cpo = b["scan_chunk_off"], b["chunk_pt_off"]
dbg = ctx.empty((S, 16), np.uint64)
dbg.fill_zero()
L.lslam_debug_set_stamps(dbg.ptr)
pl.hyp_mt19937(ctx, sco, cpo, seeds=np.arange(S), max_trials=2048 if C5 else 100)
acc = dbg.download().astype(np.float64)
names = ["block_wait", "unused", "fixed_point", "rest", "start_time", "windows", "fp_iterations",
         "parser_total"]
out = {n: round(float(np.mean(acc[:, k])), 1) for k, n in enumerate(names) if n not in ("start_time", "rest")}
tot = acc[:, 7].mean()
out["shares"] = {n: round(float(np.mean(acc[:, k]) / tot), 3) for k, n in enumerate(names[:3])}
out["cycles_per_window"] = round(float(tot / acc[:, 5].mean()), 1)
out["iterations_per_window"] = round(float(acc[:, 6].mean() / acc[:, 5].mean()), 2)
raw = dbg.download()
st = raw[:, 4].astype(np.int64)
en = raw[:, 3].astype(np.int64)
base = st.min()
st, en = st - base, en - base
ev = np.concatenate([np.stack([st, np.ones_like(st)], 1), np.stack([en, -np.ones_like(en)], 1)])
ev = ev[np.lexsort((ev[:, 1], ev[:, 0]))]
out["max_resident_parsers"] = int(np.cumsum(ev[:, 1]).max())
out["start_p50_p99_us"] = [float(np.percentile(st, 50)) / 100, float(np.percentile(st, 99)) / 100]
out["span_us"] = float(en.max()) / 100
hw = raw[:, 8:14].astype(np.int64)
key = ((hw[:, 3] * 8 + hw[:, 2]) * 2 + hw[:, 5]) * 16 + hw[:, 1]  # xcc, se, sh, cu
cus = {}
for k_, ps, hs in zip(key, hw[:, 0], hw[:, 4]):
    c_ = cus.setdefault(int(k_), [[0] * 4, [0] * 4])
    c_[0][ps] += 1
    c_[1][hs] += 1
out["n_cus_seen"] = len(cus)
out["parsers_per_simd_max"] = int(max(max(v[0]) for v in cus.values()))
out["parser_simd_hist_total"] = [int(sum(v[0][q] for v in cus.values())) for q in range(4)]
out["helper_simd_hist_total"] = [int(sum(v[1][q] for v in cus.values())) for q in range(4)]
slow = np.argsort(-(en - st))[:64]
out["slowest_parser_simd_load"] = float(np.mean([cus[int(key[i])][0][hw[i, 0]] for i in slow]))
out["median_parser_simd_load"] = float(np.median([cus[int(key[i])][0][hw[i, 0]] for i in range(S)]))
dur = (en - st) / 100.0
load = np.array([cus[int(key[i])][0][hw[i, 0]] for i in range(S)])
out["parser_us_by_simd_load"] = {int(L_): [int((load == L_).sum()), round(float(np.median(dur[load == L_])), 1),
                                           round(float(dur[load == L_].max()), 1)] for L_ in np.unique(load)}
# age order inside a SIMD: rank of the parser's start time among its SIMD's parsers
rank = np.zeros(S, np.int64)
groups = {}
for i in range(S):
    groups.setdefault((int(key[i]), int(hw[i, 0])), []).append(i)
for g_ in groups.values():
    for r_, i in enumerate(sorted(g_, key=lambda t: st[t])):
        rank[i] = r_
out["parser_us_by_age_rank"] = {int(r_): round(float(np.median(dur[rank == r_])), 1) for r_ in np.unique(rank)}
out["parser_us_p50_max"] = [float(np.percentile(en - st, 50)) / 100, float((en - st).max()) / 100]
print(json.dumps(out))
