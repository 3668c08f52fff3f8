"""One-rank RCCL communicator smoke test on device 0 (init, broadcast): does RCCL come up in
this process beside the library's HIP context.   python tools/rccl_probe.py"""
import os, sys, time
sys.path.insert(0, os.getcwd())
import numpy as np
from lidar_slam_amd.device import Context
from lidar_slam_amd import collective
ctx = Context(0)
t = time.time()
try:
    comm = collective.Comm(ctx, 1, 0, collective.unique_id())
    print("init ok %.1fs" % (time.time() - t), flush=True)
    a = ctx.to_device(np.arange(100, dtype=np.uint8)); comm.broadcast(a, 100, 0); ctx.sync()
    print("bcast ok", a.download()[:5], flush=True)
except Exception as e:
    print("FAIL %.1fs" % (time.time() - t), e, flush=True)
