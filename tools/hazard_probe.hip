// Hazard probe (test infrastructure, not product): the table window's fixed-point evaluation
// (lslam_rng_pipe.h tbl_window) and the resolve's tracker steps (lidarslam.hip rr_group_sdwa)
// written in plain HIP, so that the compiler's own gfx950 hazard recognizer places the wait
// states.  tests/test_isa_hazards.py compiles this file to assembly,
// reads the wait states the compiler put between (a) v_lshlrev_b64 and the first VALU reading
// its result and (b) a v_cmp writing an SGPR pair and the v_mbcnt reading it as a lane mask,
// and checks that the hand-scheduled asm block in the built library's rng_kernel has at least
// as many at every such pair; likewise (c) a v_cmp mask -> the v_cndmask reading it and (d) a
// VALU write of a VGPR -> an SDWA instruction reading it, against resolve_reg8_kernel.  The chain is fully dependent and unrolled, so the scheduler has
// nothing independent to fill them with: the compiler's s_nops are exactly its requirement.
#include <hip/hip_runtime.h>
#include <stdint.h>

__global__ void hazard_probe(const uint64_t *Min, uint64_t *out) {
    const uint32_t lane = threadIdx.x & 63u;
    const uint64_t M = Min[threadIdx.x];
    uint64_t R = __ballot((int)(M >> 63));
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t s = __builtin_amdgcn_mbcnt_hi((uint32_t)(R >> 32), __builtin_amdgcn_mbcnt_lo((uint32_t)R, 63u - lane));
        uint32_t hi = (uint32_t)((M << s) >> 32);
        asm("" : "+v"(hi));
        R = __ballot((int32_t)hi < 0);
    }
    out[threadIdx.x] = R;
}

// (c), (d): c = (byte k of w == c) ? k + 2 : c for two trackers; the compiler emits SDWA byte
// compares into VCC and v_cndmask_b32 selects, the trackers' chains dependent throughout.
__global__ void hazard_probe_sel(const uint32_t *J, uint32_t *out) {
    uint32_t c0 = J[threadIdx.x], c1 = J[64 + threadIdx.x];
    const uint32_t w = J[128 + threadIdx.x];
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const uint32_t j = (w >> (8 * i)) & 0xffu;
        c0 = (j == c0) ? (uint32_t)(i + 2) : c0;
        c1 = (j == c1) ? (uint32_t)(i + 2) : c1;
        asm("" : "+v"(c0), "+v"(c1));
    }
    out[threadIdx.x] = c0 + c1;
}

// (e), (f): the consensus count step (lidarslam.hip count_one / count_four) as one dependent
// chain: r = fma(x, uy, -fma(y, ux, k)), lo += |hi(r)| < c, each step's first FMA reading the
// previous step's r.  The compiler's s_nops give (e) a v_fma_f64 -> the first VALU reading its
// result (none needed) and (f) a v_cmp mask -> the v_addc reading it as the carry-in, against
// chunk_kernel's hand-scheduled count_four blocks.
__global__ void hazard_probe_count(const double *X, const float *C, int *out, double *outS) {
    double ux = X[threadIdx.x], uy = X[64 + threadIdx.x], k = X[128 + threadIdx.x];
    double x[4], y[4];
    for (int i = 0; i < 4; i++) {
        x[i] = X[192 + 64 * i + threadIdx.x];
        y[i] = X[448 + 64 * i + threadIdx.x];
    }
    float c = C[threadIdx.x];
    // every operand loaded before the chain starts (no s_waitcnt inside it)
    asm volatile("s_waitcnt vmcnt(0)" : "+v"(ux), "+v"(uy), "+v"(k), "+v"(c));
    for (int i = 0; i < 4; i++) asm volatile("" : "+v"(x[i]), "+v"(y[i]));
    int lo = 0;
    double S = 0.0;
#pragma unroll
    for (int i = 0; i < 4; i++) {
        const double r = __builtin_fma(x[i], uy, -__builtin_fma(y[i], ux, k));
        S = __builtin_fma(r, r, S);
        const float h = __uint_as_float((uint32_t)(__double_as_longlong(r) >> 32));
        lo += __builtin_fabsf(h) < c ? 1 : 0;
        asm("" : "+v"(lo), "+v"(S));
        k = r;  // the next step's first FMA reads this one's result
    }
    out[threadIdx.x] = lo;
    outS[threadIdx.x] = S;
}
