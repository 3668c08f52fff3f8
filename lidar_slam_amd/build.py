"""Build the HIP library in-tree for gfx950: ``python -m lidar_slam_amd.build``.

hipcc cross-compiles without a GPU.  -ffp-contract=off is required (the
reference's rounding has FMAs only where the kernels write __builtin_fma).
"""
from __future__ import annotations

import os
import subprocess
import sys

HERE = os.path.dirname(os.path.abspath(__file__))
SRC = os.path.join(HERE, "csrc", "lidarslam.hip")
OUT = os.path.join(HERE, "liblidarslam.so")
HIPCC = os.environ.get("HIPCC", "/opt/rocm/bin/hipcc")
FLAGS = ["--offload-arch=gfx950", "-O3", "-std=c++17", "-ffp-contract=off", "-fno-fast-math", "-fno-strict-aliasing", "-fPIC", "-shared",
         "-Wall", "-Wno-unused-function", "-Wno-unused-variable"]


def _deps():
    files = [SRC, os.path.join(HERE, "..", "include", "lidarslam.h")]
    d = os.path.join(HERE, "csrc")
    files += [os.path.join(d, f) for f in os.listdir(d) if f.endswith(".h")]
    return files


def up_to_date():
    if not os.path.exists(OUT):
        return False
    t = os.path.getmtime(OUT)
    return all(os.path.getmtime(f) <= t for f in _deps())


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + ["-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_stamps():
    """Diagnostic build with s_memtime phase stamps (tools/stamps.py)."""
    out = os.path.join(HERE, "liblidarslam_stamps.so")
    subprocess.check_call([HIPCC] + FLAGS + ["-DLSLAM_STAMPS", "-o", out, SRC])
    return out


if __name__ == "__main__":
    if "--stamps" in sys.argv:
        build_stamps()
    else:
        build(force="--force" in sys.argv)
