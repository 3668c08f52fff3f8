// lslam_wave.h — wave64 primitives for gfx950 (CDNA4).
//
// Every kernel in this library runs ONE 64-lane wave per workgroup and one
// scan per wave, so "wave-uniform" and "workgroup-uniform" coincide and
// __syncthreads() is a single-wave LDS ordering point.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>

#define LSLAM_WAVE 64

namespace lslam {

__device__ __forceinline__ int lane_id() { return (int)threadIdx.x; }

__device__ __forceinline__ uint64_t ballot(bool p) { return (uint64_t)__ballot(p); }

// number of set bits of m strictly below this lane
__device__ __forceinline__ uint32_t mbcnt(uint64_t m) {
    return __builtin_amdgcn_mbcnt_hi((uint32_t)(m >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)m, 0u));
}

__device__ __forceinline__ int uni(int v) { return __builtin_amdgcn_readfirstlane(v); }
__device__ __forceinline__ uint32_t uniu(uint32_t v) { return (uint32_t)__builtin_amdgcn_readfirstlane((int)v); }
__device__ __forceinline__ double unid(double v) {
    int64_t b = __double_as_longlong(v);
    int lo = __builtin_amdgcn_readfirstlane((int)(uint32_t)b);
    int hi = __builtin_amdgcn_readfirstlane((int)(uint32_t)(b >> 32));
    return __longlong_as_double((int64_t)(((uint64_t)(uint32_t)hi << 32) | (uint32_t)lo));
}

__device__ __forceinline__ int wave_max(int v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v = max(v, __shfl_xor(v, o));
    return v;
}

__device__ __forceinline__ double wave_sum(double v) {
#pragma unroll
    for (int o = 32; o > 0; o >>= 1) v += __shfl_xor(v, o);
    return v;
}

__device__ __forceinline__ int popc64(uint64_t m) { return __popcll(m); }
// index of the lowest set bit (m != 0)
__device__ __forceinline__ int ffs64(uint64_t m) { return __ffsll((unsigned long long)m) - 1; }
// index of the highest set bit (m != 0)
__device__ __forceinline__ int fls64(uint64_t m) { return 63 - __clzll((long long)m); }

// Correctly rounded sqrt.  The hardware/LLVM sequence is accurate to <= 1 ulp;
// one Tuckerman step makes it exact (x is a multiple of ulp(y)^2, so the
// products y*y(+-) are never within ulp^2/4 of a representable x).
__device__ __forceinline__ double cr_sqrt(double x) {
    double y = __builtin_sqrt(x);
    if (!(x > 0.0) || !(x < __builtin_inf())) return y;
    double yu = __longlong_as_double(__double_as_longlong(y) + 1);
    double yd = __longlong_as_double(__double_as_longlong(y) - 1);
    if (__builtin_fma(y, yu, -x) < 0.0) return yu;
    if (__builtin_fma(yd, y, -x) >= 0.0) return yd;
    return y;
}

}  // namespace lslam
