"""Diagnostic driver for tools/chunkphase.sh: the C3 consensus (Philox hypotheses, chunk_kernel
only: lslam_ransac) twice on 4096 scans with the library named by LSLAM_LIB.  Run under
rocprofv3 --pmc with the LSLAM_CHUNK_EXIT variants; the per-launch SQ counters then hold the
instructions of the phases before the exit."""
import os
import sys

import numpy as np

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
os.environ.setdefault("LSLAM_ALLOW_STALE", "1")
from bench import make_workload  # noqa: E402
from lidar_slam_amd import pipeline as pl  # noqa: E402
from lidar_slam_amd.device import Context  # noqa: E402

S = 4096
ctx = Context(0)
b, _ = make_workload(list(range(S)), 720, 20)
p = pl.ScanPipeline(ctx, b["xy"], b["scan_chunk_off"], b["chunk_pt_off"], seeds=np.arange(S), hyp="philox")
for _ in range(2):
    p.run_ransac_only()
print("chunks", int(b["scan_chunk_off"][-1]))
