// Which instructions SQ_INSTS_SALU counts (diagnostic, not product): one wave per kernel runs
// 256 x 8 of one instruction form; rocprofv3 --pmc SQ_INSTS_SALU SQ_INSTS_VALU SQ_WAVES per dispatch.
// Build: hipcc --offload-arch=gfx950 -O3 -o tools/ubench_nopcount tools/ubench_nopcount.hip
#include <hip/hip_runtime.h>
#include <cstdio>

#define REP8(x) x x x x x x x x
template <int K>
__global__ void form(int *out) {
    int s = threadIdx.x;
    for (int i = 0; i < 256; i++) {
        if (K == 0) asm volatile(REP8("s_nop 0\n\t"));
        if (K == 1) asm volatile(REP8("s_nop 1\n\t"));
        if (K == 2) asm volatile(REP8("s_nop 7\n\t"));
        if (K == 3) asm volatile(REP8("s_waitcnt lgkmcnt(0)\n\t"));
        if (K == 4) asm volatile(REP8("s_add_u32 s100, s100, 1\n\t") ::: "s100", "scc");
        if (K == 5) asm volatile(REP8("v_xor_b32 %0, 1, %0\n\t") : "+v"(s));
    }
    out[threadIdx.x] = s;
}

int main() {
    int *d;
    hipMalloc(&d, 64 * sizeof(int));
    form<0><<<1, 64>>>(d);
    form<1><<<1, 64>>>(d);
    form<2><<<1, 64>>>(d);
    form<3><<<1, 64>>>(d);
    form<4><<<1, 64>>>(d);
    form<5><<<1, 64>>>(d);
    hipDeviceSynchronize();
    printf("ok\n");
    hipFree(d);
    return 0;
}
