"""The rounding bound behind the consensus kernels' cheap inlier test
(lidarslam.hip: chunk_consensus, count_kernel).

Both evaluate the cross product of a point with a hypothesis' unit direction as
two fmas, r = fl(x*uy - fl(y*ux + k)) with k = fl(ox*uy - fl(oy*ux)), and
decide r^2 against the cutoff outside a band of width
2^-42 (E2 + ecut + R (sqrt(ecut) + 1)).  That band rests on
|r - r_true| <= 4 u R + u |r_true| (u = 2^-53, R = max|x| + max|y| over the
chunk's box, which holds o), where r_true = (x - ox) uy - (y - oy) ux exactly.
This checks the bound with the fmas emulated exactly (Fraction arithmetic,
correctly rounded back to double), on random and adversarial chunks:
coordinates up to the 5 m range of the sensor model, directions near the
axes, points on and near the line.  CPU only.
"""
import math
import random
from fractions import Fraction as F

U = 2.0 ** -53


def fma(a, b, c):
    return float(F(a) * F(b) + F(c))


def mul(a, b):
    return float(F(a) * F(b))


def kernel_r(x, y, ox, oy, ux, uy):
    k = fma(ox, uy, -mul(oy, ux))
    return fma(x, uy, -fma(y, ux, k))


def check_chunk(pts, o, u):
    ox, oy = o
    ux, uy = u
    xs = [p[0] for p in pts] + [ox]
    ys = [p[1] for p in pts] + [oy]
    R = max(abs(min(xs)), abs(max(xs))) + max(abs(min(ys)), abs(max(ys)))
    worst = 0.0
    for x, y in pts:
        r = kernel_r(x, y, ox, oy, ux, uy)
        rt = (F(x) - F(ox)) * F(uy) - (F(y) - F(oy)) * F(ux)
        err = abs(F(r) - rt)
        bound = F(4 * U) * F(R) + F(U) * abs(rt)
        assert err <= bound, (x, y, o, u, float(err), float(bound))
        worst = max(worst, float(err / bound) if bound else 0.0)
    return worst


def unit(theta):
    ux, uy = math.cos(theta), math.sin(theta)
    n = math.sqrt(ux * ux + uy * uy)
    return ux / n, uy / n


def test_random_chunks_within_bound():
    rng = random.Random(7)
    worst = 0.0
    for _ in range(300):
        scale = rng.choice([1.0, 100.0, 5000.0])
        o = (rng.uniform(-scale, scale), rng.uniform(-scale, scale))
        u = unit(rng.uniform(-math.pi, math.pi))
        pts = []
        for _ in range(40):
            t = rng.uniform(-scale, scale)
            d = rng.choice([0.0, rng.uniform(-30, 30), rng.uniform(-1e-9, 1e-9), 20.0])
            pts.append((o[0] + t * u[0] - d * u[1], o[1] + t * u[1] + d * u[0]))
        worst = max(worst, check_chunk(pts, o, u))
    assert worst <= 1.0


def test_axis_aligned_and_near_axis_directions():
    rng = random.Random(11)
    for theta in (0.0, math.pi / 2, math.pi, -math.pi / 2, 1e-12, math.pi / 2 - 1e-12, 1e-300):
        u = unit(theta)
        o = (rng.uniform(-5000, 5000), rng.uniform(-5000, 5000))
        pts = [(o[0] + rng.uniform(-5000, 5000), o[1] + rng.uniform(-25, 25)) for _ in range(60)]
        pts += [(o[0] + rng.uniform(-25, 25), o[1] + rng.uniform(-5000, 5000)) for _ in range(60)]
        check_chunk(pts, o, u)


def test_points_at_the_threshold_distance():
    # points exactly 20 mm off the line (the band the cutoffs bracket), far from the origin
    rng = random.Random(3)
    for _ in range(100):
        o = (rng.uniform(-5000, 5000), rng.uniform(-5000, 5000))
        u = unit(rng.uniform(-math.pi, math.pi))
        pts = []
        for _ in range(20):
            t = rng.uniform(-4000, 4000)
            s = rng.choice([-20.0, 20.0])
            pts.append((o[0] + t * u[0] - s * u[1], o[1] + t * u[1] + s * u[0]))
        check_chunk(pts, o, u)
