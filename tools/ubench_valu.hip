// Micro-benchmark: issue cost of the producer's VALU forms on gfx950 (diagnostic, not product).
// For each instruction form, every wave runs ITER iterations of 8 independent chains (throughput)
// or 1 chain (dependent latency); cycles from s_memtime around the loop, per wave-instruction.
// Grid: 256 workgroups of 64 * W threads (W waves per CU spread over its 4 SIMDs).
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_valu tools/ubench_valu.hip
// Run:   tools/ubench_valu     (prints one JSON object)
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdint>
#include <vector>
#include <algorithm>

#define ITER 256

enum Op { XOR32 = 0, MBCNT, LSHL64, CMP64, CMP32, BITOP3, ALIGNBIT, EVAL64, EVAL32, FMA64, XOR64E, CMPE32, CMPE64ND, MAD24, SADD, MIX, NOPS };
static const char *names[NOPS] = {"v_xor_b32", "v_mbcnt_lo+hi (pair)", "v_lshlrev_b64", "v_cmp_gt_i64_e64",
                                  "v_cmp_gt_i32_e64", "v_bitop3_b32", "v_alignbit_b32",
                                  "eval: mbcnt x2 + lshl_b64 + cmp_i64 (dependent)",
                                  "eval: mbcnt x2 + lshl_b64 + cmp_i32 hi (dependent)", "v_fma_f64", "v_xor_b32_e64 (VOP3 encoding)", "v_cmp_gt_i32_e32 (vcc, no consumer)", "v_cmp_gt_i32_e64 (sgpr, no consumer)", "v_mad_u32_u24", "s_add_u32 (SALU; per_simd_Nw = per SIMD share, x4 for per CU)", "mix: 8 v_xor_b32 + 8 s_add_u32 per iteration (per_simd: cycles per xor+s_add pair)"};

template <int OP, bool DEP>
__global__ void kern(uint64_t *out, uint32_t seed) {
    uint32_t a[8], b[8];
    uint64_t m[8];
    double f[8];
    for (int k = 0; k < 8; k++) {
        a[k] = seed * (threadIdx.x + 1) + k;
        b[k] = a[k] ^ 0x9e3779b9u;
        m[k] = ((uint64_t)a[k] << 32) | b[k];
        f[k] = (double)a[k];
    }
    uint64_t s0 = 0x12345, s1 = 0x6789a;
    const uint64_t t0 = __builtin_amdgcn_s_memtime();
    for (int it = 0; it < ITER; it++) {
        if (OP == XOR32) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_xor_b32 %0, %1, %0" : "+v"(a[k]) : "v"(DEP ? a[k] : b[k]));
        } else if (OP == MBCNT) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %0\n\tv_mbcnt_hi_u32_b32 %0, %2, %0"
                             : "+v"(a[k]) : "s"((uint32_t)s0), "s"((uint32_t)s1));
        } else if (OP == LSHL64) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_lshlrev_b64 %0, %1, %0" : "+v"(m[k]) : "v"(b[k]));
        } else if (OP == CMP64) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                uint64_t r;
                asm volatile("v_cmp_gt_i64_e64 %0, 0, %1" : "=s"(r) : "v"(m[k]));
                s0 ^= r;
            }
        } else if (OP == CMP32) {
#pragma unroll
            for (int k = 0; k < 8; k++) {
                uint64_t r;
                asm volatile("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(r) : "v"(a[k]));
                s0 ^= r;
            }
        } else if (OP == BITOP3) {
#pragma unroll
            for (int k = 0; k < 8; k++)
                asm volatile("v_bitop3_b32 %0, %0, %1, %2 bitop3:0x6a" : "+v"(a[k]) : "s"((uint32_t)s0), "v"(b[k]));
        } else if (OP == ALIGNBIT) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_alignbit_b32 %0, %1, %0, %2" : "+v"(a[k]) : "v"(b[k]), "v"(b[k]));
        } else if (OP == EVAL64 || OP == EVAL32) {
            // one fixed-point evaluation per chain: s = mbcnt(R, base); R = ballot(bit 63 of M << s)
            // (the chain runs through the SGPR mask, as in tbl_window)
            const int nch = DEP ? 1 : 4;
            uint64_t R[4] = {s0, s1, s0 ^ s1, s0 + s1};
#pragma unroll
            for (int k = 0; k < nch; k++) {
                uint32_t s;
                uint64_t sh;
                asm volatile("v_mbcnt_lo_u32_b32 %0, %1, %2\n\tv_mbcnt_hi_u32_b32 %0, %3, %0"
                             : "=&v"(s) : "s"((uint32_t)R[k]), "v"(b[k]), "s"((uint32_t)(R[k] >> 32)));
                asm volatile("v_lshlrev_b64 %0, %1, %2" : "=v"(sh) : "v"(s), "v"(m[k]));
                if (OP == EVAL64)
                    asm volatile("v_cmp_gt_i64_e64 %0, 0, %1" : "=s"(R[k]) : "v"(sh));
                else
                    asm volatile("v_cmp_gt_i32_e64 %0, 0, %1" : "=s"(R[k]) : "v"((uint32_t)(sh >> 32)));
            }
            s0 = R[0] ^ R[1] ^ R[2] ^ R[3];
        } else if (OP == XOR64E) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_xor_b32_e64 %0, %1, %0" : "+v"(a[k]) : "v"(b[k]));
        } else if (OP == CMPE32) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_cmp_gt_i32_e32 vcc, 0, %0" ::"v"(a[k]) : "vcc");
        } else if (OP == CMPE64ND) {
            uint64_t r0, r1, r2, r3;
#pragma unroll
            for (int k = 0; k < 2; k++)
                asm volatile("v_cmp_gt_i32_e64 %0, 0, %4\n\tv_cmp_gt_i32_e64 %1, 0, %5\n\tv_cmp_gt_i32_e64 %2, 0, %6\n\tv_cmp_gt_i32_e64 %3, 0, %7"
                             : "=s"(r0), "=s"(r1), "=s"(r2), "=s"(r3) : "v"(a[4 * k]), "v"(a[4 * k + 1]), "v"(a[4 * k + 2]), "v"(a[4 * k + 3]));
        } else if (OP == MAD24) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_mad_u32_u24 %0, %1, 28, %0" : "+v"(a[k]) : "v"(b[k]));
        } else if (OP == SADD) {
            uint32_t q0 = (uint32_t)s0, q1 = (uint32_t)s1, q2 = q0 ^ 5u, q3 = q1 ^ 7u, q4 = q0 + 3u, q5 = q1 + 9u,
                     q6 = q0 * 3u, q7 = q1 * 5u;
            asm volatile(
                "s_add_u32 %0, %0, 3\n\ts_add_u32 %1, %1, 5\n\ts_add_u32 %2, %2, 7\n\ts_add_u32 %3, %3, 9\n\t"
                "s_add_u32 %4, %4, 3\n\ts_add_u32 %5, %5, 5\n\ts_add_u32 %6, %6, 7\n\ts_add_u32 %7, %7, 9"
                : "+s"(q0), "+s"(q1), "+s"(q2), "+s"(q3), "+s"(q4), "+s"(q5), "+s"(q6), "+s"(q7)::"scc");
            s0 = (uint64_t)(q0 ^ q1 ^ q2 ^ q3) << 32 | (q4 ^ q5 ^ q6 ^ q7);
        } else if (OP == MIX) {
            uint32_t q0 = (uint32_t)s0, q1 = (uint32_t)s1, q2 = q0 ^ 5u, q3 = q1 ^ 7u, q4 = q0 + 3u, q5 = q1 + 9u,
                     q6 = q0 * 3u, q7 = q1 * 5u;
            asm volatile(
                "s_add_u32 %0, %0, 3\n\tv_xor_b32 %8, %16, %8\n\ts_add_u32 %1, %1, 5\n\tv_xor_b32 %9, %16, %9\n\t"
                "s_add_u32 %2, %2, 7\n\tv_xor_b32 %10, %16, %10\n\ts_add_u32 %3, %3, 9\n\tv_xor_b32 %11, %16, %11\n\t"
                "s_add_u32 %4, %4, 3\n\tv_xor_b32 %12, %16, %12\n\ts_add_u32 %5, %5, 5\n\tv_xor_b32 %13, %16, %13\n\t"
                "s_add_u32 %6, %6, 7\n\tv_xor_b32 %14, %16, %14\n\ts_add_u32 %7, %7, 9\n\tv_xor_b32 %15, %16, %15"
                : "+s"(q0), "+s"(q1), "+s"(q2), "+s"(q3), "+s"(q4), "+s"(q5), "+s"(q6), "+s"(q7),
                  "+v"(a[0]), "+v"(a[1]), "+v"(a[2]), "+v"(a[3]), "+v"(a[4]), "+v"(a[5]), "+v"(a[6]), "+v"(a[7])
                : "v"(b[0])
                : "scc");
            s0 = (uint64_t)(q0 ^ q1 ^ q2 ^ q3) << 32 | (q4 ^ q5 ^ q6 ^ q7);
        } else if (OP == FMA64) {
#pragma unroll
            for (int k = 0; k < 8; k++) asm volatile("v_fma_f64 %0, %0, %1, %1" : "+v"(f[k]) : "v"(DEP ? f[k] : 1.0));
        }
    }
    const uint64_t t1 = __builtin_amdgcn_s_memtime();
    uint64_t acc = s0 ^ s1;
    for (int k = 0; k < 8; k++) acc += a[k] + m[k] + (uint64_t)f[k];
    if (threadIdx.x % 64 == 0) out[2 * (blockIdx.x * (blockDim.x / 64) + threadIdx.x / 64)] = t1 - t0;
    if (acc == 0x5a5a5a5a5a5aull) out[1] = acc;  // keeps the chains live
}

template <int OP, bool DEP>
static double run(int W, uint64_t *d_out, std::vector<uint64_t> &h) {
    const int nwg = 256;
    const int nwaves = nwg * W;
    hipMemset(d_out, 0, sizeof(uint64_t) * 2 * nwaves);
    kern<OP, DEP><<<nwg, 64 * W>>>(d_out, 7);  // warm-up
    kern<OP, DEP><<<nwg, 64 * W>>>(d_out, 11);
    hipDeviceSynchronize();
    hipMemcpy(h.data(), d_out, sizeof(uint64_t) * 2 * nwaves, hipMemcpyDeviceToHost);
    std::vector<double> c;
    for (int w = 0; w < nwaves; w++) c.push_back((double)h[2 * w]);
    std::sort(c.begin(), c.end());
    const double med = c[c.size() / 2];
    // wave-instructions per wave in the loop
    double per = 8.0;
    if (OP == MBCNT) per = 16.0;
    if (OP == SADD) per = 77.0 / 4.0;
    if (OP == MIX) per = 8.0;  // pairs (plus ~11 combining SALU per iteration, see SADD)  // SALU instructions per iteration in the compiled loop (4 iterations: 77)
    if (OP == EVAL64 || OP == EVAL32) per = (DEP ? 1.0 : 4.0) * 4.0;
    // cycles per wave-instruction per SIMD (W/4 waves per SIMD share it)
    return med / (ITER * per) / (W >= 4 ? W / 4.0 : 1.0);
}

template <int OP>
static void one(uint64_t *d, std::vector<uint64_t> &h, bool first) {
    printf("%s  \"%s\": {\"dep_1wave\": %.2f, \"thr_1wave\": %.2f, \"thr_per_simd_4w\": %.2f, \"thr_per_simd_8w\": %.2f, \"thr_per_simd_16w\": %.2f}\n",
           first ? "" : ",", names[OP], run<OP, true>(1, d, h), run<OP, false>(1, d, h), run<OP, false>(4, d, h),
           run<OP, false>(8, d, h), run<OP, false>(16, d, h));
}

int main() {
    uint64_t *d;
    std::vector<uint64_t> h(2 * 256 * 16);
    hipMalloc(&d, sizeof(uint64_t) * 2 * 256 * 16);
    printf("{\"unit\": \"cycles (s_memtime) per wave-instruction; 1wave = one wave per CU, per_simd_Nw = N waves per CU (N/4 per SIMD), per SIMD\",\n");
    one<XOR32>(d, h, true);
    one<MBCNT>(d, h, false);
    one<LSHL64>(d, h, false);
    one<CMP64>(d, h, false);
    one<CMP32>(d, h, false);
    one<BITOP3>(d, h, false);
    one<ALIGNBIT>(d, h, false);
    one<EVAL64>(d, h, false);
    one<EVAL32>(d, h, false);
    one<FMA64>(d, h, false);
    one<XOR64E>(d, h, false);
    one<CMPE32>(d, h, false);
    one<CMPE64ND>(d, h, false);
    one<MAD24>(d, h, false);
    one<SADD>(d, h, false);
    one<MIX>(d, h, false);
    printf("}\n");
    hipFree(d);
    return 0;
}
