"""Register budgets of the pipeline kernels that share the SIMDs with the producer (CPU test: needs
hipcc's llvm-readelf, no GPU).  Beside the producer's four 30-VGPR parser waves per SIMD, the
consensus keeps three waves per SIMD only at <= 128 VGPRs (allocation granule 8, 512 per SIMD
lane): a 132-VGPR build left it two and the C3 step 3.4 % slower (profiles/r06_ab_priorities_slot.txt, r06g;
DESIGN.md §8).  The producer's parsers must stay at <= 32 so that four fit
with the consumers, the seeding and cut kernels must not spill."""
import os
import re
import shutil
import subprocess

import pytest

LLVM = "/opt/rocm/lib/llvm/bin"

pytestmark = pytest.mark.skipif(not os.path.exists(os.path.join(LLVM, "llvm-readelf")),
                                reason="needs llvm-readelf")


@pytest.fixture(scope="module")
def notes(tmp_path_factory):
    from lidar_slam_amd import build
    lib = build.build(verbose=False)
    d = tmp_path_factory.mktemp("lib")
    so = str(d / "lib.so")
    shutil.copy(lib, so)
    subprocess.check_call([os.path.join(LLVM, "llvm-objdump"), "--offloading", so], cwd=str(d),
                          stdout=subprocess.DEVNULL, stderr=subprocess.DEVNULL)
    co = [f for f in os.listdir(str(d)) if "gfx950" in f]
    assert co, "no gfx950 code object in the library"
    text = subprocess.check_output([os.path.join(LLVM, "llvm-readelf"), "--notes", str(d / co[0])], text=True)
    out = {}
    name = None
    for ln in text.splitlines():
        m = re.match(r"\s+\.name:\s+(\S+)", ln)
        if m:
            name = m.group(1)
            continue
        m = re.match(r"\s+\.(vgpr_count|vgpr_spill_count|sgpr_spill_count):\s+(\d+)", ln)
        if m and name:
            out.setdefault(name, {})[m.group(1)] = int(m.group(2))
    return out


@pytest.mark.parametrize("symbol", ["_Z12chunk_kernelILi0EEv5KArgs", "_Z12chunk_kernelILi1EEv5KArgs",
                                    "_Z12chunk_kernelILi2EEv5KArgs"])
def test_consensus_fits_three_waves_beside_the_parsers(notes, symbol):
    k = notes[symbol]
    assert k["vgpr_count"] <= 128, k
    assert k.get("vgpr_spill_count", 0) == 0, k


@pytest.mark.parametrize("symbol", ["_Z10rng_kernelIhEv5KArgs", "_Z10rng_kernelItEv5KArgs"])
def test_parser_waves_stay_small(notes, symbol):
    k = notes[symbol]
    assert k["vgpr_count"] <= 32, k
    assert k.get("vgpr_spill_count", 0) == 0 and k.get("sgpr_spill_count", 0) == 0, k


@pytest.mark.parametrize("symbol", ["_Z11seed_kernelPKjiPj", "_Z15cut_lane_kernel5KArgsP8ChunkCut",
                                    "_Z19resolve_reg8_kernel5KArgsi"])
def test_side_kernels_do_not_spill(notes, symbol):
    k = notes[symbol]
    assert k.get("vgpr_spill_count", 0) == 0 and k.get("sgpr_spill_count", 0) == 0, k
