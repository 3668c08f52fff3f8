"""Build A/B variants of the HIP library with extra preprocessor defines (diagnostics and
experiments only; the product build is lidar_slam_amd/build.py).

    python tools/build_variants.py NAME=-DFOO,-DBAR=3 OTHER=-DBAZ ...

writes lidar_slam_amd/variants/lib_NAME.so (built from the same sources, so it carries the
tree's source hash; load it with LSLAM_LIB=... LSLAM_ALLOW_STALE=1)."""
import os
import subprocess
import sys
from concurrent.futures import ThreadPoolExecutor

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
sys.path.insert(0, ROOT)
from lidar_slam_amd import build as b  # noqa: E402

OUT = os.path.join(ROOT, "lidar_slam_amd", "variants")


def one(spec):
    name, _, defs = spec.partition("=")
    out = os.path.join(OUT, "lib_%s.so" % name)
    cmd = [b.HIPCC] + b.FLAGS + b._hash_flag() + [d for d in defs.split(",") if d] + ["-o", out, b.SRC]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with ThreadPoolExecutor(max_workers=4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
