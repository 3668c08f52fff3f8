// Micro-benchmark: do a wave's s_nop / s_sleep / SALU / VALU instructions take issue slots from
// the other waves of its SIMD?  (diagnostic, not product; VERDICT r04 "the s_nop question")
//
// One workgroup of 16 waves per CU (a large LDS request keeps it alone on the CU), so wave w
// runs on SIMD w % 4.  Waves 0..11 are VICTIMS (3 per SIMD): 8 independent v_xor_b32 chains,
// ITER iterations, timed with s_memtime.  Waves 12..15 (1 per SIMD) are OTHERS and run one role
// until the victims of their workgroup are done (an LDS flag polled every 64 instructions):
//   0 idle (exit at once)          1 s_nop 0 x64        2 s_nop 7 x64
//   3 s_add_u32 x64                4 v_xor_b32 x64 (8 chains)
//   5 the table window's evaluation: (mbcnt lo, mbcnt hi, lshl_b64, s_nop 0, cmp into vcc, s_nop 1) x16
//   6 the same evaluation without the s_nops (hazards ignored: the values are never used)
//   7 s_sleep 1
// Reported: victim cycles per v_xor per SIMD (3 victims share a SIMD), median over all victims.
// If s_nop took issue slots like SALU does, roles 1/2 would slow the victims like role 3.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_issue tools/ubench_issue.hip
#include <hip/hip_runtime.h>
#include <algorithm>
#include <cstdint>
#include <cstdio>
#include <vector>

#define ITER 2048
#define NW 16
#define NVICT 12

__global__ __launch_bounds__(1024) void kern(uint64_t *out, int role, uint32_t seed) {
    extern __shared__ uint32_t lds[];
    const int w = __builtin_amdgcn_readfirstlane(threadIdx.x / 64);
    if (threadIdx.x == 0) lds[0] = 0;
    __syncthreads();
    if (w < NVICT) {
        uint32_t a[8], b = seed * (threadIdx.x + 1);
        for (int k = 0; k < 8; k++) a[k] = b + k;
        const uint64_t t0 = __builtin_amdgcn_s_memtime();
        for (int it = 0; it < ITER; it++) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[k]) : "v"(b));
        }
        const uint64_t t1 = __builtin_amdgcn_s_memtime();
        uint32_t acc = 0;
        for (int k = 0; k < 8; k++) acc ^= a[k];
        if (threadIdx.x % 64 == 0) {
            out[blockIdx.x * NVICT + w] = t1 - t0;
            atomicAdd(&lds[0], 1u);
        }
        if (acc == 0x5a5a5a5au) out[0] = acc;
        return;
    }
    if (role == 0) return;
    // the other wave issues first whenever it is ready (waves of a SIMD issue by priority, then
    // age: at equal priority the older victims would take every slot and starve it)
    __builtin_amdgcn_s_setprio(3);
    uint32_t iters = 0;
    uint32_t a[8], b = seed * (threadIdx.x + 3);
    for (int k = 0; k < 8; k++) a[k] = b + k;
    uint32_t q = __builtin_amdgcn_readfirstlane(b), s = 0;
    volatile uint32_t *flag = lds;
    for (;;) {
        if (role == 1) {
#pragma unroll
            for (int k = 0; k < 64; k++) asm volatile("s_nop 0");
        } else if (role == 2) {
#pragma unroll
            for (int k = 0; k < 64; k++) asm volatile("s_nop 7");
        } else if (role == 3) {
#pragma unroll
            for (int k = 0; k < 64; k++) asm volatile("s_add_u32 %0, %0, 3" : "+s"(q)::"scc");
        } else if (role == 4) {
#pragma unroll
            for (int k = 0; k < 8; k++)
#pragma unroll
                for (int u = 0; u < 8; u++) asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[u]) : "v"(b));
        } else if (role == 5) {
            asm volatile(
                ".rept 16\n\t"
                "v_mbcnt_lo_u32_b32 v26, vcc_lo, v27\n\tv_mbcnt_hi_u32_b32 v26, vcc_hi, v26\n\t"
                "v_lshlrev_b64 v[28:29], v26, v[28:29]\n\ts_nop 0\n\tv_cmp_gt_i32_e32 vcc, 0, v29\n\ts_nop 1\n\t"
                ".endr" ::: "vcc", "v26", "v27", "v28", "v29");
        } else if (role == 6) {
            asm volatile(
                ".rept 16\n\t"
                "v_mbcnt_lo_u32_b32 v26, vcc_lo, v27\n\tv_mbcnt_hi_u32_b32 v26, vcc_hi, v26\n\t"
                "v_lshlrev_b64 v[28:29], v26, v[28:29]\n\tv_cmp_gt_i32_e32 vcc, 0, v29\n\t"
                ".endr" ::: "vcc", "v26", "v27", "v28", "v29");
        } else {
            asm volatile("s_sleep 1");
        }
        iters++;
        if (__builtin_amdgcn_readfirstlane(*flag) >= NVICT) break;
    }
    if ((threadIdx.x & 63) == 0) out[(size_t)gridDim.x * NVICT + blockIdx.x * 4 + (w - NVICT)] = iters;
    uint32_t acc = q ^ s;
    for (int k = 0; k < 8; k++) acc ^= a[k];
    if (acc == 0x5a5a5a5au) out[1] = acc;
}

int main() {
    int n_cu = 0;
    (void)hipDeviceGetAttribute(&n_cu, hipDeviceAttributeMultiprocessorCount, 0);
    const int nwg = n_cu > 0 ? n_cu : 256;
    uint64_t *d;
    (void)hipMalloc(&d, sizeof(uint64_t) * nwg * (NVICT + 4));
    std::vector<uint64_t> h(nwg * (NVICT + 4));
    const size_t lds = 96 * 1024;  // one workgroup per CU
    (void)hipFuncSetAttribute((const void *)kern, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    static const char *names[8] = {"idle", "s_nop 0", "s_nop 7", "s_add_u32", "v_xor_b32",
                                   "eval with s_nops", "eval without s_nops", "s_sleep 1"};
    printf("{\"unit\": \"victim cycles per v_xor_b32 per SIMD (3 victim waves + 1 other wave per SIMD)\", \"cus\": %d", nwg);
    for (int role = 0; role < 8; role++) {
        kern<<<nwg, 64 * NW, lds>>>(d, role, 7);  // warm-up
        kern<<<nwg, 64 * NW, lds>>>(d, role, 11);
        (void)hipDeviceSynchronize();
        (void)hipMemset(d, 0, sizeof(uint64_t) * nwg * (NVICT + 4));
        kern<<<nwg, 64 * NW, lds>>>(d, role, 11);
        (void)hipDeviceSynchronize();
        (void)hipMemcpy(h.data(), d, sizeof(uint64_t) * nwg * (NVICT + 4), hipMemcpyDeviceToHost);
        std::vector<double> c(h.begin(), h.begin() + nwg * NVICT);
        std::vector<double> o(h.begin() + nwg * NVICT, h.end());
        std::sort(o.begin(), o.end());
        std::sort(c.begin(), c.end());
        const double med = c[c.size() / 2];
        // 3 victims per SIMD, 8 v_xor per iteration each
        printf(",\n \"%s\": {\"victim\": %.3f, \"other_iters_median\": %.0f}", names[role], med / (ITER * 8.0 * 3.0), o[o.size() / 2]);
    }
    printf("\n}\n");
    (void)hipFree(d);
    return 0;
}
