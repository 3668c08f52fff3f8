"""Diagnostic: the producer's table-mode window cut into segments (s_memtime stamps).

Uses the diagnostic build lidar_slam_amd/variants/lib_wstamps.so
(python tools/build_variants.py wstamps=-DLSLAM_STAMPS,-DLSLAM_WSTAMPS); the product
library has no stamps.  Runs the MT19937 producer alone (lslam_hyp_mt19937) on the C3
scans and prints, per window inside a run (tbl_window<false>, K = 99 and K = 19), the mean
cycles of each segment with the stamp's own cost (an empty segment) subtracted:
  temper      the next window's word load issued + temper of this window's words
  table       reject-table row read (LDS) + the two funnel shifts
  unchecked   the first evaluation + 2 evaluations without a test
  checked     the checked loop: one evaluation, VALU->SALU compare and branch per turn
  store       the accepted lanes' store, accepted count, step / position bookkeeping
Stamps serialise the wave (s_memtime + s_waitcnt): read the segments as a latency
breakdown of one window, not as the production time."""
import ctypes as C
import json
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("LSLAM_ALLOW_STALE", "1")
from lidar_slam_amd import _lib  # noqa: E402

_lib.LIB_PATH = os.environ.get("LSLAM_LIB") or os.path.join(ROOT, "lidar_slam_amd", "variants", "lib_wstamps.so")
L = _lib.load()
L.lslam_debug_set_stamps.argtypes = [C.c_void_p]
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

S = int(sys.argv[1]) if len(sys.argv) > 1 else 4096
ctx = Context(0)
b, _ = make_workload(list(range(S)), 720, 20)
dbg = ctx.empty((S, 16), np.uint64)
out = {}
for rep in range(3):
    dbg.fill_zero()
    L.lslam_debug_set_stamps(dbg.ptr)
    pl.hyp_mt19937(ctx, b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.arange(S))
w = dbg.download()[:, 8:16].astype(np.float64)
nwin = w[:, 5].sum()
cal = w[:, 7].sum() / nwin
names = ["temper", "table", "unchecked", "checked", "store"]
seg = {n: round(w[:, k].sum() / nwin - cal, 1) for k, n in enumerate(names)}
out["cycles_per_window"] = seg
out["window_total_minus_stamps"] = round(sum(seg.values()), 1)
out["stamp_cost"] = round(cal, 1)
out["windows_per_scan"] = round(nwin / S, 1)
out["checked_turns_per_window"] = round(w[:, 6].sum() / nwin, 3)
out["unchecked_evals"] = 3
out["shares"] = {n: round(v / max(sum(seg.values()), 1e-9), 3) for n, v in seg.items()}
out["parser_total_cycles_per_scan"] = round(float(dbg.download()[:, 7].astype(np.float64).mean()), 1)
print(json.dumps(out))
