// Diagnostic (not product code): the MFMA ceiling of THIS box -- bare bf16 MFMA loops on random operands, the
// 16x16x32 and 32x32x16 shapes at equal FLOPs per loop trip, B operands from registers or re-read from LDS with
// ds_read_b128 (the mrfv K loop's B path), 1-3 waves per SIMD, with the in-kernel clock (s_memtime / s_memrealtime
// stamps of wave 0 into a stamp buffer of their own).  The achievable fraction of the nominal 2.5 PF the MRF K loop
// is held against.   hipcc -O3 --offload-arch=gfx950 mfma_ceiling.hip -o mfma_ceiling
#include <hip/hip_runtime.h>
#include <cstdio>
#include <cstdlib>
#include <vector>
#include <algorithm>

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef __attribute__((ext_vector_type(16))) float f32x16;

#define CK(x) do { hipError_t e_ = (x); if (e_ != hipSuccess) { printf("HIP %s line %d\n", hipGetErrorString(e_), __LINE__); exit(1); } } while (0)

// SHAPE 16: 8 x 16x16x32 per trip on 4 accumulators; SHAPE 32: 4 x 32x32x16 per trip on 2 accumulators (same FLOPs)
// FILL: independent v_fma_f32 per 16 384 FLOP issued by the same wave between its MFMAs (16x16x32: FILL after each
// MFMA; 32x32x16: 2 FILL) -- the staging / epilogue VALU that shares the vector-issue port with the MFMAs in mrfv
template <int SHAPE, bool LDSB, int FILL = 0>
__global__ __launch_bounds__(256) void mfma_loop(const bf16x8* __restrict__ src, float* __restrict__ out,
                                                 unsigned long long* __restrict__ stamps, int iters) {
    __shared__ bf16x8 lds[8 * 256];
    const int tid = threadIdx.x, lane = tid & 63;
    const bf16x8 a = src[(blockIdx.x * 256 + tid + 4096 - 64) % 4096];
    bf16x8 b[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        b[j] = src[(blockIdx.x * 256 + tid + 512 * (j + 1)) % 4096];
        asm volatile("" : "+v"(b[j]));  // materialised once, before the loop
    }
    if (LDSB) {
#pragma unroll
        for (int j = 0; j < 8; ++j) lds[j * 256 + tid] = b[j];
        __syncthreads();
    }
    unsigned long long t0 = 0, r0 = 0;
    if (tid == 0) { t0 = __builtin_amdgcn_s_memtime(); r0 = __builtin_amdgcn_s_memrealtime(); }
    float sum = 0.f;
    // named accumulators (an acc[j & 3] array made hipcc rotate AGPRs with v_accvgpr moves every trip)
    // The mrfv K-step of one wave (32 output channels x 128 rows x 32 input channels = 262 144 FLOP) in both shapes,
    // as two loop trips of half that: 16x16x32 -- 2 A (weight) fragments x 4 B (input-row) fragments, each B feeding
    // 2 MFMAs (8 per trip); 32x32x16 -- 1 A x 4 B, each B feeding 1 MFMA (4 per trip).  Per FLOP the same A and B
    // bytes either way (4 x 1 KB of B per 131 072 FLOP).  B is read for the NEXT trip while this trip's MFMAs run
    // (the mrfv look-ahead).  The MFMAs are inline asm on AGPR accumulators: with the builtins hipcc rotated the
    // accumulators through v_accvgpr moves every trip, which is not the loop under test.
    const bf16x8 a1 = b[7];
    float f0 = lane * 1e-3f, f1 = f0 + 1.f, f2 = f0 + 2.f, f3 = f0 + 3.f, f4 = f0 + 4.f, f5 = f0 + 5.f, f6 = f0 + 6.f,
          f7 = f0 + 7.f;
#define FILLN(n) _Pragma("unroll") for (int q = 0; q < (n); ++q) {                                                  \
        switch (q & 7) {                                                                                              \
            case 0: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f0)); break;                                      \
            case 1: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f1)); break;                                      \
            case 2: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f2)); break;                                      \
            case 3: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f3)); break;                                      \
            case 4: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f4)); break;                                      \
            case 5: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f5)); break;                                      \
            case 6: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f6)); break;                                      \
            default: asm volatile("v_fma_f32 %0, %0, %0, 1.0" : "+v"(f7)); break;                                     \
        } }
    // two trips per loop iteration, ping-ponging the B registers (no copies)
#define LDB(dst, t) do { if (LDSB) { _Pragma("unroll") for (int j = 0; j < 4; ++j) \
        dst[j] = lds[j * 256 + (tid & ~63) + ((lane + (t)) & 63)]; } } while (0)
    bf16x8 b0[4], b1[4];
#pragma unroll
    for (int j = 0; j < 4; ++j) b0[j] = b1[j] = LDSB ? lds[j * 256 + (tid & ~63) + lane] : b[j];
    if constexpr (SHAPE == 16) {
        f32x4 c[8] = {};
#define TRIP16(cur, nxt, t)                                                                                           \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                               \
            if (LDSB) nxt[j] = lds[j * 256 + (tid & ~63) + ((lane + (t)) & 63)];                                       \
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c[2 * j]) : "v"(a), "v"(cur[j]));           \
            FILLN(FILL)                                                                                               \
            asm volatile("v_mfma_f32_16x16x32_bf16 %0, %1, %2, %0" : "+a"(c[2 * j + 1]) : "v"(a1), "v"(cur[j]));      \
            FILLN(FILL)                                                                                               \
        }
        for (int it = 0; it < iters; it += 2) {
            TRIP16(b0, b1, it + 1)
            TRIP16(b1, b0, it + 2)
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) sum += c[j][0] + c[j][1] + c[j][2] + c[j][3];
    } else {
        f32x16 c[4] = {};
#define TRIP32(cur, nxt, t, aa)                                                                                       \
        _Pragma("unroll") for (int j = 0; j < 4; ++j) {                                                               \
            if (LDSB) nxt[j] = lds[j * 256 + (tid & ~63) + ((lane + (t)) & 63)];                                       \
            asm volatile("v_mfma_f32_32x32x16_bf16 %0, %1, %2, %0" : "+a"(c[j]) : "v"(aa), "v"(cur[j]));             \
            FILLN(2 * FILL)                                                                                           \
        }
        for (int it = 0; it < iters; it += 2) {
            TRIP32(b0, b1, it + 1, a)
            TRIP32(b1, b0, it + 2, a1)
        }
#pragma unroll
        for (int j = 0; j < 4; ++j)
#pragma unroll
            for (int r = 0; r < 16; ++r) sum += c[j][r];
    }
#undef LDB
#undef FILLN
    sum += f0 + f1 + f2 + f3 + f4 + f5 + f6 + f7;
    if (tid == 0) {
        const unsigned long long t1 = __builtin_amdgcn_s_memtime(), r1 = __builtin_amdgcn_s_memrealtime();
        stamps[2 * blockIdx.x] = t1 - t0;
        stamps[2 * blockIdx.x + 1] = r1 - r0;
    }
    out[blockIdx.x * 256 + tid] = sum;
}

template <int SHAPE, bool LDSB, int FILL = 0>
static void run(const bf16x8* src, float* out, unsigned long long* st, int wps) {
    const int blocks = 256 * wps, iters = 20000;
    auto k = mfma_loop<SHAPE, LDSB, FILL>;
    hipEvent_t e0, e1;
    CK(hipEventCreate(&e0));
    CK(hipEventCreate(&e1));
    // warm the clock governor: ~2 s of back-to-back launches first
    for (int i = 0; i < 600 / wps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, src, out, st, iters);
    CK(hipDeviceSynchronize());
    const int reps = 20;
    CK(hipEventRecord(e0));
    for (int i = 0; i < reps; ++i) hipLaunchKernelGGL(k, dim3(blocks), dim3(256), 0, 0, src, out, st, iters);
    CK(hipEventRecord(e1));
    CK(hipEventSynchronize(e1));
    float ms = 0;
    CK(hipEventElapsedTime(&ms, e0, e1));
    std::vector<unsigned long long> h(2 * blocks);
    CK(hipMemcpy(h.data(), st, h.size() * 8, hipMemcpyDeviceToHost));
    std::vector<double> ghz;
    for (int b = 0; b < blocks; ++b) ghz.push_back(h[2 * b + 1] ? (double)h[2 * b] / (double)h[2 * b + 1] * 0.1 : 0.0);
    std::sort(ghz.begin(), ghz.end());
    const double flop = 2.0 * 16 * 16 * 32 * 8 * (double)iters * blocks * 4 * reps;  // 4 waves per block
    const double tfs = flop / (ms * 1e-3) / 1e12;
    printf("%-9s B from %-4s fill %d %d wave(s)/SIMD: %8.1f TFLOP/s = %.3f of 2.5 PF, in-kernel clock median %.2f GHz "
           "(%.3f of 2.5 PF x 2.4 GHz / clock)\n", SHAPE == 16 ? "16x16x32" : "32x32x16", LDSB ? "LDS" : "regs", FILL, wps,
           tfs, tfs / 2500.0, ghz[blocks / 2], tfs / 2500.0 * 2.4 / ghz[blocks / 2]);
}

int main() {
    std::vector<unsigned short> h(4096 * 8);
    srand(12345);
    for (auto& v : h) {  // random bf16 in [-1, 1): sign, exponent 126/127, random mantissa
        const unsigned s = rand() & 1, e = 126 + (rand() & 1), m = rand() & 0x7F;
        v = (unsigned short)((s << 15) | (e << 7) | m);
    }
    bf16x8* src;
    float* out;
    unsigned long long* st;
    CK(hipMalloc(&src, h.size() * 2));
    CK(hipMalloc(&out, 256 * 3 * 256 * 4));
    CK(hipMalloc(&st, 256 * 3 * 2 * 8));
    CK(hipMemcpy(src, h.data(), h.size() * 2, hipMemcpyHostToDevice));
    for (int wps = 1; wps <= 3; ++wps) {
        run<16, false>(src, out, st, wps);
        run<32, false>(src, out, st, wps);
        run<16, true>(src, out, st, wps);
        run<32, true>(src, out, st, wps);
    }
    for (int wps = 2; wps <= 3; ++wps) {
        run<16, true, 1>(src, out, st, wps);
        run<32, true, 1>(src, out, st, wps);
        run<16, true, 2>(src, out, st, wps);
        run<32, true, 2>(src, out, st, wps);
        run<16, true, 3>(src, out, st, wps);
        run<32, true, 3>(src, out, st, wps);
        run<16, true, 4>(src, out, st, wps);
        run<32, true, 4>(src, out, st, wps);
    }
    CK(hipFree(src));
    CK(hipFree(out));
    CK(hipFree(st));
    return 0;
}
