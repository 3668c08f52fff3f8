// Host-side numeric helpers of the library (plain C++, also compiled by tests/test_host_math.py).
#pragma once
#include <cmath>

// The largest v with RN(sqrt(v)) <= t (IEEE sqrt, as cr_sqrt on the device): sqrt is monotone, so
// {v >= 0 : RN(sqrt(v)) <= t} = [0, bound], and the association's distance tests
// (landmarking.py:57-72, sqrt(e) <= TOL_DIST) become e <= bound without a square root.
// t < 0 or NaN: no v (bound -1); t = +inf: every v but NaN.
static inline double sqrt_le_bound(double t) {
    if (std::isnan(t) || t < 0.0) return -1.0;
    if (std::isinf(t)) return HUGE_VAL;
    double v = t * t;
    while (v > 0.0 && std::sqrt(v) > t) v = std::nextafter(v, 0.0);
    while (std::sqrt(std::nextafter(v, HUGE_VAL)) <= t) v = std::nextafter(v, HUGE_VAL);
    return v;
}
