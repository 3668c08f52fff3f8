// Issue-rate microbenchmark: waves per SIMD x instruction type -> cycles per
// wave-instruction per SIMD.  hipcc --offload-arch=gfx950 -O3 issue.hip -o issue
#include <hip/hip_runtime.h>
#include <stdio.h>
#include <stdint.h>

template <int KIND>
__global__ __launch_bounds__(256) void k(uint32_t *out, int iters) {
    uint32_t a0 = threadIdx.x, a1 = a0 + 1, a2 = a0 + 2, a3 = a0 + 3, a4 = a0 + 4, a5 = a0 + 5, a6 = a0 + 6, a7 = a0 + 7;
    uint32_t s0 = blockIdx.x, s1 = s0 + 1, s2 = s0 + 2, s3 = s0 + 3;
    for (int it = 0; it < iters; it++) {
        if (KIND == 0) {  // 8 independent VALU chains, 8 instrs per loop body x 8 unroll
#pragma unroll
            for (int u = 0; u < 8; u++) {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(a2));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a2) : "v"(a3));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a3) : "v"(a4));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a4) : "v"(a5));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a5) : "v"(a6));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a6) : "v"(a7));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a7) : "v"(a0));
            }
        } else if (KIND == 1) {  // SALU independent
#pragma unroll
            for (int u = 0; u < 16; u++) {
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(s2));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s2) : "s"(s3));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s3) : "s"(s0));
            }
        } else if (KIND == 2) {  // mixed: 1 VALU + 1 SALU alternating
#pragma unroll
            for (int u = 0; u < 16; u++) {
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s0) : "s"(s1));
                asm volatile("v_add_u32 %0, %0, %1" : "+v"(a1) : "v"(a2));
                asm volatile("s_add_u32 %0, %0, %1" : "+s"(s1) : "s"(s2));
            }
        } else if (KIND == 3) {  // dependent VALU chain
#pragma unroll
            for (int u = 0; u < 64; u++) asm volatile("v_add_u32 %0, %0, %1" : "+v"(a0) : "v"(a1));
        } else if (KIND == 4) {  // VALU writes SGPR (v_cmp) -> SALU compare chain, like a ballot loop
#pragma unroll
            for (int u = 0; u < 16; u++) {
                uint64_t m;
                asm volatile("v_cmp_gt_u32 %0, %1, %2" : "=s"(m) : "v"(a0), "v"(a1));
                asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0" : "+v"(a0) : "s"((uint32_t)m));
            }
        }
    }
    out[blockIdx.x * blockDim.x + threadIdx.x] = a0 + a1 + a2 + a3 + a4 + a5 + a6 + a7 + s0 + s1 + s2 + s3;
}

int main() {
    uint32_t *out;
    hipMalloc(&out, 256 * 4096 * 4);
    hipEvent_t e0, e1;
    hipEventCreate(&e0);
    hipEventCreate(&e1);
    const int iters = 2000;
    const char *names[] = {"valu_indep", "salu_indep", "valu+salu", "valu_dep", "vcmp->mbcnt"};
    const int per_iter[] = {64, 64, 64, 64, 32};
    for (int kind = 0; kind < 5; kind++) {
        for (int wps = 1; wps <= 8; wps *= 2) {
            // 256 CUs x 4 SIMDs: blocks of 256 threads = 4 waves (one per SIMD); wps blocks per CU
            const int blocks = 256 * wps;
            auto launch = [&]() {
                switch (kind) {
                    case 0: hipLaunchKernelGGL(k<0>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 1: hipLaunchKernelGGL(k<1>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 2: hipLaunchKernelGGL(k<2>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 3: hipLaunchKernelGGL(k<3>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                    case 4: hipLaunchKernelGGL(k<4>, dim3(blocks), dim3(256), 0, 0, out, iters); break;
                }
            };
            launch();
            hipDeviceSynchronize();
            hipEventRecord(e0);
            launch();
            hipEventRecord(e1);
            hipEventSynchronize(e1);
            float ms;
            hipEventElapsedTime(&ms, e0, e1);
            const double instr_per_simd = (double)wps * iters * per_iter[kind];
            printf("%-12s waves/SIMD=%d  %.3f ms  cycles/instr/SIMD @2.4GHz = %.2f\n", names[kind], wps, ms,
                   ms * 1e-3 * 2.4e9 / instr_per_simd);
        }
    }
    return 0;
}
