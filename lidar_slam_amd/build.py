"""Build the HIP library in-tree for gfx950: ``python -m lidar_slam_amd.build``.

hipcc cross-compiles without a GPU.  -ffp-contract=off is required (the
reference's rounding has FMAs only where the kernels write __builtin_fma).
"""
from __future__ import annotations

import hashlib
import os
import re
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


def source_hash():
    """16 hex digits of sha256 over the library's sources (csrc/*.hip, csrc/*.h,
    include/lidarslam.h), by file name then content.  Embedded in lslam_version() so that
    the loader can refuse a library built from other sources."""
    h = hashlib.sha256()
    for f in sorted(_deps(), key=os.path.basename):
        h.update(os.path.basename(f).encode() + b"\0")
        with open(f, "rb") as fh:
            h.update(fh.read())
    return h.hexdigest()[:16]


def embedded_hash(path=OUT):
    """The source hash a built library carries (None if absent or unreadable)."""
    try:
        with open(path, "rb") as f:
            m = re.search(rb"\(abi \d+, src ([0-9a-f]{16}),", f.read())
    except OSError:
        return None
    return m.group(1).decode() if m else None


def up_to_date():
    return os.path.exists(OUT) and embedded_hash(OUT) == source_hash()


def _hash_flag():
    return ['-DLSLAM_SRC_HASH="%s"' % source_hash()]


def build(force=False, verbose=True):
    if not force and up_to_date():
        return OUT
    cmd = [HIPCC] + FLAGS + _hash_flag() + ["-o", OUT + ".tmp", SRC]
    if verbose:
        print(" ".join(cmd), flush=True)
    subprocess.check_call(cmd)
    os.replace(OUT + ".tmp", OUT)
    return OUT


def build_stamps():
    """Diagnostic build with s_memtime phase stamps (tools/stamps.py)."""
    out = os.path.join(HERE, "liblidarslam_stamps.so")
    subprocess.check_call([HIPCC] + FLAGS + _hash_flag() + ["-DLSLAM_STAMPS", "-o", out, SRC])
    return out


def build_census():
    """Diagnostic build with only the wave census (tools/census.py): production timing."""
    out = os.path.join(HERE, "liblidarslam_census.so")
    subprocess.check_call([HIPCC] + FLAGS + _hash_flag() + ["-DLSLAM_CENSUS", "-o", out, SRC])
    return out


if __name__ == "__main__":
    if "--stamps" in sys.argv:
        build_stamps()
    elif "--census" in sys.argv:
        build_census()
    else:
        build(force="--force" in sys.argv)
