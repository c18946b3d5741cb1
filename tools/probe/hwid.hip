// probe: which SIMD does each wave of a 512-thread workgroup land on (HW_ID.SIMD_ID, bits 5:4)?
#include <hip/hip_runtime.h>
#include <cstdio>
__global__ __launch_bounds__(512, 1) void probe(unsigned* out) {
    extern __shared__ unsigned char pad[];
    unsigned id;
    asm volatile("s_getreg_b32 %0, hwreg(HW_REG_HW_ID)" : "=s"(id));
    if ((threadIdx.x & 63) == 0) out[blockIdx.x * 8 + (threadIdx.x >> 6)] = id;
    if (threadIdx.x == 9999) pad[0] = 1;
}
int main() {
    unsigned* d;
    const int nb = 256;
    hipMalloc(&d, nb * 8 * 4);
    hipFuncSetAttribute((const void*)probe, hipFuncAttributeMaxDynamicSharedMemorySize, 130 * 1024);
    hipLaunchKernelGGL(probe, dim3(nb), dim3(512), 130 * 1024, 0, d);
    unsigned h[nb * 8];
    hipMemcpy(h, d, sizeof(h), hipMemcpyDeviceToHost);
    int hist[8][4] = {};
    for (int b = 0; b < nb; ++b)
        for (int w = 0; w < 8; ++w) hist[w][(h[b * 8 + w] >> 4) & 3]++;
    for (int w = 0; w < 8; ++w) printf("wave %d: simd0 %d simd1 %d simd2 %d simd3 %d\n", w, hist[w][0], hist[w][1], hist[w][2], hist[w][3]);
    for (int b = 0; b < 3; ++b) {
        printf("block %d:", b);
        for (int w = 0; w < 8; ++w) printf(" %08x", h[b * 8 + w]);
        printf("\n");
    }
    return 0;
}
