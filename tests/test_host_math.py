"""Host-side helpers of the library (lidar_slam_amd/csrc/lslam_host_math.h), compiled with g++ on
the CPU.  sqrt_le_bound(t) replaces the association's two square roots per landmark test
(landmarking.py:57-72: sqrt(e) <= TOL_DIST) by e <= bound: the bound must be exactly the last
e whose correctly rounded square root is <= t."""
import os
import shutil
import subprocess

import pytest

ROOT = os.path.dirname(os.path.dirname(os.path.abspath(__file__)))
HDR = os.path.join(ROOT, "lidar_slam_amd", "csrc", "lslam_host_math.h")

PROG = r"""
#include "lslam_host_math.h"
#include <cstdio>
#include <cstdlib>
#include <random>
int main() {
    std::mt19937_64 g(7);
    std::uniform_real_distribution<double> u(-3.0, 3.0);
    double ts[] = {0.0, -0.0, 1e-300, 1e-160, 0.5, 1.0, 2.0, 3.0, 20.0, 100.0, 1000.0, 1e150, 1e154, 1e200, 1.7e308};
    int bad = 0, n = 0;
    auto check = [&](double t) {
        const double b = sqrt_le_bound(t);
        n++;
        if (t < 0.0 || std::isnan(t)) { bad += !(b < 0.0); return; }
        if (!(std::sqrt(b) <= t)) bad++;
        const double nb = std::nextafter(b, HUGE_VAL);
        if (std::isfinite(nb) && std::sqrt(nb) <= t) bad++;
    };
    for (double t : ts) check(t);
    for (int i = 0; i < 200000; i++) check(std::ldexp(1.0 + std::fabs(u(g)), (int)(g() % 200) - 100));
    check(-1.0); check(NAN);
    if (!(sqrt_le_bound(HUGE_VAL) == HUGE_VAL)) bad++;
    std::printf("%d %d\n", n, bad);
    return bad != 0;
}
"""


@pytest.mark.skipif(shutil.which("g++") is None, reason="needs g++")
def test_sqrt_le_bound(tmp_path):
    src = tmp_path / "t.cpp"
    src.write_text(PROG)
    exe = tmp_path / "t"
    subprocess.check_call(["g++", "-O2", "-std=c++17", "-ffp-contract=off", "-I", os.path.dirname(HDR), str(src),
                           "-o", str(exe)])
    out = subprocess.run([str(exe)], capture_output=True, text=True)
    n, bad = map(int, out.stdout.split())
    assert n > 200000 and bad == 0, out.stdout
