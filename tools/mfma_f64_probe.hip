// Probe (diagnostic, not product): v_mfma_f64_16x16x4_f64 operand layout and rounding on gfx950,
// before chunk_consensus's residuals move onto it.  (1) layout: A[i][k] = 100 i + k, B[k][j] =
// 7 j + 1000 k + 1 (asymmetric, exact integers) against the host product under the guide's maps
// (A/B: lane l holds [l & 15][l >> 4] / [l >> 4][l & 15]; C/D: col = l & 15, row = (l >> 4) +
// 4 reg); (2) numerics: random doubles, D compared bit for bit with the k-ordered fma chain
// fma(a3, b3, fma(a2, b2, fma(a1, b1, fma(a0, b0, c)))) and with the correctly rounded sum.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/mfma_f64_probe tools/mfma_f64_probe.hip
#include <hip/hip_runtime.h>
#include <cmath>
#include <cstdint>
#include <cstdio>
#include <cstring>
#include <random>

typedef double d4 __attribute__((ext_vector_type(4)));

__global__ void probe(const double *A, const double *B, const double *C, double *D) {
    const int l = threadIdx.x;
    const double a = A[(l & 15) * 4 + (l >> 4)];  // A[i][k], row-major [16][4]
    const double b = B[(l >> 4) * 16 + (l & 15)];  // B[k][j], row-major [4][16]
    d4 c;
    for (int r = 0; r < 4; r++) c[r] = C[((l >> 4) + 4 * r) * 16 + (l & 15)];
    const d4 d = __builtin_amdgcn_mfma_f64_16x16x4f64(a, b, c, 0, 0, 0);
    for (int r = 0; r < 4; r++) D[((l >> 4) + 4 * r) * 16 + (l & 15)] = d[r];
}

static long double exact4(const double *a, const double *b, double c) {
    long double s = c;
    for (int k = 0; k < 4; k++) s += (long double)a[k] * b[k];
    return s;
}

int main() {
    double hA[64], hB[64], hC[256], hD[256];
    double *dA, *dB, *dC, *dD;
    (void)hipMalloc(&dA, 512);
    (void)hipMalloc(&dB, 512);
    (void)hipMalloc(&dC, 2048);
    (void)hipMalloc(&dD, 2048);
    auto run = [&]() {
        (void)hipMemcpy(dA, hA, 512, hipMemcpyHostToDevice);
        (void)hipMemcpy(dB, hB, 512, hipMemcpyHostToDevice);
        (void)hipMemcpy(dC, hC, 2048, hipMemcpyHostToDevice);
        hipLaunchKernelGGL(probe, dim3(1), dim3(64), 0, 0, dA, dB, dC, dD);
        (void)hipMemcpy(hD, dD, 2048, hipMemcpyDeviceToHost);
    };
    // (1) layout
    for (int i = 0; i < 16; i++)
        for (int k = 0; k < 4; k++) hA[i * 4 + k] = 100.0 * i + k;
    for (int k = 0; k < 4; k++)
        for (int j = 0; j < 16; j++) hB[k * 16 + j] = 7.0 * j + 1000.0 * k + 1.0;
    for (int e = 0; e < 256; e++) hC[e] = (double)e;
    run();
    int bad = 0;
    for (int i = 0; i < 16; i++)
        for (int j = 0; j < 16; j++) {
            double s = hC[i * 16 + j];
            for (int k = 0; k < 4; k++) s += hA[i * 4 + k] * hB[k * 16 + j];
            if (s != hD[i * 16 + j]) bad++;
        }
    printf("{\"layout_mismatches\": %d", bad);
    // (2) numerics
    std::mt19937_64 g(12345);
    std::uniform_real_distribution<double> u(-1.0, 1.0);
    long chain_eq = 0, rn_eq = 0, n = 0;
    double max_ulp_rn = 0;
    for (int rep = 0; rep < 200; rep++) {
        for (int e = 0; e < 64; e++) hA[e] = u(g) * std::ldexp(1.0, (int)(g() % 40) - 20);
        for (int e = 0; e < 64; e++) hB[e] = u(g) * std::ldexp(1.0, (int)(g() % 40) - 20);
        for (int e = 0; e < 256; e++) hC[e] = (rep & 1) ? 0.0 : u(g);
        run();
        for (int i = 0; i < 16; i++)
            for (int j = 0; j < 16; j++) {
                const double *a = hA + i * 4;
                double b[4];
                for (int k = 0; k < 4; k++) b[k] = hB[k * 16 + j];
                double ch = hC[i * 16 + j];
                for (int k = 0; k < 4; k++) ch = std::fma(a[k], b[k], ch);
                const double d = hD[i * 16 + j];
                chain_eq += (ch == d);
                const long double ex = exact4(a, b, hC[i * 16 + j]);
                const double rn = (double)ex;
                rn_eq += (rn == d);
                const double ulp = std::fabs((double)((long double)d - ex)) / std::ldexp(1.0, std::ilogb(rn) - 52);
                if (ulp > max_ulp_rn) max_ulp_rn = ulp;
                n++;
            }
    }
    printf(", \"results\": %ld, \"equal_k_ordered_fma_chain\": %ld, \"equal_rn_of_long_double_sum\": %ld, "
           "\"max_err_ulps_vs_long_double\": %.3f}\n", n, chain_eq, rn_eq, max_ulp_rn);
    return 0;
}
