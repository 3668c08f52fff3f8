"""Build the HIP library of another git revision as an A/B arm.

    python tools/build_rev.py REV NAME   -> lidar_slam_amd/variants/lib_NAME.so

The revision's csrc/ and include/ are exported to a temporary tree (git archive) and compiled
with the product flags; load the result with LSLAM_LIB=... LSLAM_ALLOW_STALE=1 (its source hash
is the revision's commit id, not the tree's).  ABI and struct layouts must match the working tree's
Python side: use it for kernel-only changes."""
import os
import shutil
import subprocess
import sys
import tempfile

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import build as b  # noqa: E402


def main(rev, name):
    tmp = tempfile.mkdtemp(prefix="lslam_rev_")
    try:
        arc = subprocess.check_output(["git", "archive", rev, "lidar_slam_amd/csrc", "include"], cwd=ROOT)
        subprocess.run(["tar", "-x", "-C", tmp], input=arc, check=True)
        out = os.path.join(ROOT, "lidar_slam_amd", "variants", "lib_%s.so" % name)
        os.makedirs(os.path.dirname(out), exist_ok=True)
        sha = subprocess.check_output(["git", "rev-parse", rev], cwd=ROOT, text=True).strip()[:16]
        subprocess.check_call([b.HIPCC] + b.FLAGS + ['-DLSLAM_SRC_HASH="%s"' % sha] +
                              ["-o", out, os.path.join(tmp, "lidar_slam_amd", "csrc", "lidarslam.hip")])
        print(out)
    finally:
        shutil.rmtree(tmp)


if __name__ == "__main__":
    main(sys.argv[1], sys.argv[2])
