"""Build A/B variants of the HIP library with extra preprocessor defines (diagnostics and
experiments only; the product build is lidar_slam_amd/build.py).

    python tools/build_variants.py NAME=-DFOO,-DBAR=3 OTHER=-DBAZ ...
    python tools/build_variants.py mfma=patch:mfma_consensus.patch

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


PATCHES = os.path.join(ROOT, "tools", "variants")


def one(spec):
    """NAME=-DFOO,-DBAR builds with defines; NAME=patch:FILE applies tools/variants/FILE (a measured
    experiment kept out of the shipped sources) to a copy of the tree and builds that."""
    name, _, defs = spec.partition("=")
    out = os.path.join(OUT, "lib_%s.so" % name)
    if defs.startswith("patch:"):
        import shutil
        import tempfile
        tmp = tempfile.mkdtemp(prefix="lslam_variant_")
        for d in ("lidar_slam_amd/csrc", "include"):
            shutil.copytree(os.path.join(ROOT, d), os.path.join(tmp, d))
        subprocess.check_call(["git", "apply", os.path.join(PATCHES, defs[6:])], cwd=tmp)
        src = os.path.join(tmp, "lidar_slam_amd", "csrc", "lidarslam.hip")
        subprocess.check_call([b.HIPCC] + b.FLAGS + ["-mllvm", "-amdgpu-mfma-vgpr-form"] + b._hash_flag() +
                              ["-o", out, src])
        shutil.rmtree(tmp)
        return out
    cmd = [b.HIPCC] + b.FLAGS + b._hash_flag() + [d for d in defs.split(",") if d] + ["-o", out, b.SRC]
    subprocess.check_call(cmd)
    return out


if __name__ == "__main__":
    os.makedirs(OUT, exist_ok=True)
    with ThreadPoolExecutor(max_workers=4) as ex:
        for o in ex.map(one, sys.argv[1:]):
            print(o)
