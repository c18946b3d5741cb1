// The LDS-DMA GEMM of the linears (csrc/conv.hip's dispatcher routes STZS_CONV_A_DMA linears and every fp8 linear
// here): both operands stream through an LDS-DMA ring, in-launch split-K, the fused epilogue of conv_common.hpp
// compiled in per variant.
#include "conv_common.hpp"

namespace {

STZS_DEV void glds16(const void* src, void* dst) {
    __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                     (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
}

// Pure GEMM for linears (ks = 1, no prologue): BOTH operands stream through an LDS-DMA ring, one
// 64-byte-per-row K-step per slot (bf16: 32 k; fp8: 64 k.  A: BTM rows, B: 128 cols, 8 KB each at
// BTM = 128), 4 slots filled three K-steps ahead.  The A image takes the same XOR swizzle as B
// through its per-lane SOURCE addresses (LDS-DMA writes lane-linearly), so both fragment reads are
// conflict-free ds_read_b128.  Per K-step: counted vmcnt + one s_barrier, then the NEXT K-step's
// fragments are read between the current K-step's MFMAs (as csrc/mrf.hip); the body is branch-free
// (a fill past the end re-copies the last K-step into a retired slot) and the last K-step is peeled.
// F8 (configs[4] denoiser): e4m3fn operands; each 16-B fragment feeds TWO v_mfma_f32_16x16x32_fp8_fp8
// (bytes 0-7 and 8-15: both operands use the same k permutation, so the dot product is unchanged),
// and acc * x_scale[row] * w_scale[col] enters the epilogue.
template <int BTM>
constexpr int gslot() { return BTM * 64 + SLOT_BYTES; }  // A (BTM rows x 64 B) + B of one K-step
// SK > 1 (stzs_conv_args.splitk, BTM = 64, bf16): workgroup z of a tile runs K-steps [z NK/SK, (z+1) NK/SK) and
// hands its fp32 partial to the tile's last arriver (splitk_combine), which then runs the epilogue.
template <int BTM, int SK>
STZS_DEV bool splitk_combine(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem);
// STZS_GEMM_PROF (a probe build only, tools/gemm_phase.py): lane 0 of every workgroup stamps s_memtime at the kernel's
// start, after the first K-step landed, after the K loop, after the epilogue's stores issued and after they drained,
// into splitk_ws (unused by the SK = 1 kernels) -- 8 words per workgroup.  Never defined in the library build.
#ifdef STZS_GEMM_PROF
#define GPROF(i)                                                                                              \
    if (SK == 1 && a.splitk_ws && threadIdx.x == 0)                                                            \
        reinterpret_cast<unsigned long long*>(a.splitk_ws)[(long)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = \
            __builtin_amdgcn_s_memtime();
#else
#define GPROF(i)
#endif
// LDS of one workgroup: the K-step ring (4 slots) aliased with the epilogue's fp32 tile + bias / gate rows (a linear
// has no channel statistics).  64-row tiles: 48 KB -> three workgroups per CU (<= 136 VGPRs); 128-row: 68.6 KB -> two.
template <int BTM>
constexpr size_t gemm_lds() {
    const size_t ring = 4 * (size_t)gslot<BTM>(), epi = (size_t)BTM * EP_PITCH * 4 + 2 * BCO * 4;
    return ring > epi ? ring : epi;
}
template <typename TOut, int BTM, bool F8, int SK = 1, int EP = -1>
__global__ __launch_bounds__(NTHR, BTM == 64 ? 3 : 2) void gemm_glds(const stzs_conv_args a) {
    GPROF(0)
    constexpr int MT = BTM / 32;           // 16-row tiles per wave (2 x 2 waves)
    constexpr int GS = gslot<BTM>();
    constexpr int AP = BTM / 64;           // A pieces (1 KB) per wave per K-step
    constexpr int ESZ = F8 ? 1 : 2;        // operand bytes per element
    constexpr int NMF = MT * 4 * (F8 ? 2 : 1);  // MFMAs per K-step
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    // XCD-aware tile order (the dispatcher deals workgroup ids round-robin over the 8 XCDs): every XCD gets a
    // contiguous range of tiles, column tile fastest, so the tiles one XCD runs at a time share their A rows and
    // the whole weight matrix (<= 2 MB for every linear) stays resident in that XCD's 4-MB L2 instead of being
    // re-fetched from the fabric by each XCD for every row tile.  Same tiles, same K order: bit-identical.
    const int gy = gridDim.y;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * gridDim.x + blockIdx.x
                                                      : xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gy);
    const int by = (a.flags & STZS_CONV_LINEAR_IDS) ? (int)blockIdx.y : lin % gy;
    const int bx = (a.flags & STZS_CONV_LINEAR_IDS) ? (int)blockIdx.x : lin / gy;
    const long row0 = (long)bx * BTM;
    const long nR = (long)a.B * a.T_in;
    const int NK = a.ci_pad / (64 / ESZ);
    const int NKS = NK / SK;                                  // K-steps of this workgroup's slice
    const int kb = SK > 1 ? (int)blockIdx.z * NKS : 0;
    const unsigned char* Wt = reinterpret_cast<const unsigned char*>(a.w) + (long)by * NK * SLOT_BYTES;
    const unsigned char* X = reinterpret_cast<const unsigned char*>(a.x);
    long asrc[AP];  // byte offsets
#pragma unroll
    for (int i = 0; i < AP; ++i) {
        const int o = wave * AP * 1024 + i * 1024 + lane * 16;
        const int r = o >> 6, p = (o >> 4) & 3;
        long R = row0 + r;
        R = R < nR ? R : nR - 1;
        const long bb = rowdiv(R, a.T_in, 1.f / (float)a.T_in, nR < (1L << 22));
        asrc[i] = (bb * a.bsx + (R - bb * a.T_in) * a.ldx) * ESZ + ((p ^ gswz(r)) << 4);
    }
    auto fill = [&](int k) {
        const int kc = kb + (k < NKS ? k : NKS - 1);
        const unsigned char* src = Wt + (long)kc * SLOT_BYTES + wave * 2048 + lane * 16;
        unsigned char* da = smem + (k & 3) * GS + wave * AP * 1024;
        unsigned char* db = smem + (k & 3) * GS + BTM * 64 + wave * 2048;
        glds16(src, db);
        glds16(src + 1024, db + 1024);
#pragma unroll
        for (int i = 0; i < AP; ++i) glds16(X + asrc[i] + kc * 64, da + i * 1024);
    };
    int aoff0, boff0;
    {
        const int ra = wt * (BTM / 2) + (lane & 15);
        aoff0 = ra * 64 + (((lane >> 4) ^ gswz(ra)) << 4);
        const int rb = wc * 64 + (lane & 15);
        boff0 = BTM * 64 + rb * 64 + (((lane >> 4) ^ gswz(rb)) << 4);
    }
    f32x4 acc[MT][4];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    bf16x8 fa0[MT], fb0[4], fa1[MT], fb1[4];
    auto rd = [&](bf16x8 (&fa)[MT], bf16x8 (&fb)[4], int k) {
        const unsigned char* sl = smem + (k & 3) * GS;
#pragma unroll
        for (int i = 0; i < MT; ++i) fa[i] = *reinterpret_cast<const bf16x8*>(sl + aoff0 + i * 1024);
#pragma unroll
        for (int i = 0; i < 4; ++i) fb[i] = *reinterpret_cast<const bf16x8*>(sl + boff0 + i * 1024);
    };
    auto mma = [&](const bf16x8 (&fa)[MT], const bf16x8 (&fb)[4]) {
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                if constexpr (F8) {
                    const i64x2 va = __builtin_bit_cast(i64x2, fa[mt]);
                    const i64x2 vb = __builtin_bit_cast(i64x2, fb[nt]);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(va[0], vb[0], acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_fp8_fp8(va[1], vb[1], acc[mt][nt], 0, 0, 0);
                } else {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb[nt], acc[mt][nt], 0, 0, 0);
                }
            }
    };
    constexpr int PER_FILL = 2 + AP;  // LDS-DMA instructions per wave per K-step
    fill(0);
    fill(1);
    __builtin_amdgcn_s_waitcnt(0x0F70 | PER_FILL);  // K-step 0 landed (K-step 1 may be in flight)
    __builtin_amdgcn_s_barrier();
    GPROF(1)
    fill(2);
    rd(fa0, fb0, 0);
#define STZS_GEMM_STEP(FA, FB, NA, NB)                                          \
    {                                                                           \
        __builtin_amdgcn_s_waitcnt(0x0F70 | PER_FILL);                          \
        __builtin_amdgcn_s_barrier();                                           \
        fill(k + 3);                                                            \
        __builtin_amdgcn_sched_barrier(0);                                      \
        rd(NA, NB, k + 1);                                                      \
        mma(FA, FB);                                                            \
        _Pragma("unroll") for (int ii = 0; ii < MT + 4; ++ii) {                 \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                  \
        }                                                                       \
        __builtin_amdgcn_sched_group_barrier(0x008, NMF - MT - 4, 0);           \
        __builtin_amdgcn_sched_barrier(0);                                      \
        ++k;                                                                    \
    }
    int k = 0;
    const int nsteps = (a.flags & 2) ? 1 : NKS;
    for (; k + 2 < nsteps;) {
        STZS_GEMM_STEP(fa0, fb0, fa1, fb1)
        STZS_GEMM_STEP(fa1, fb1, fa0, fb0)
    }
    if (k + 1 < nsteps) {
        STZS_GEMM_STEP(fa0, fb0, fa1, fb1)
        mma(fa1, fb1);
    } else {
        mma(fa0, fb0);
    }
#undef STZS_GEMM_STEP
    GPROF(2)
    if constexpr (F8) {  // dequantise: row scale (flat row, clamped like the A rows) x column scale
        float sw[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) sw[nt] = a.w_scale[by * BCO + wc * 64 + nt * 16 + (lane & 15)];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                long R = row0 + wt * (BTM / 2) + mt * 16 + (lane >> 4) * 4 + r;
                R = R < nR ? R : nR - 1;
                const float sx = a.x_scale[R];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) acc[mt][nt][r] *= sx * sw[nt];
            }
    }
    if constexpr (SK > 1) {
        if (!splitk_combine<BTM, SK>(a, acc, smem)) return;
    }
    finish<TOut, true, BTM, EP>(a, acc, smem, 0, 0, row0, by);
#ifdef STZS_GEMM_PROF
    GPROF(3)
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    GPROF(4)
#endif
}

// In-launch split-K hand-off (MI355X guide: cdna_hip_programming.md, "In-launch split-K reduction", the sc1
// form of the Guideline 16 counter hand-off).  Slab of (tile, slice s): [NV][NTHR] f32x4, thread-linear so
// every store / load is one coalesced 16-B access per lane.  Producer: write-through (sc1) stores, every
// wave's vmcnt(0) (which also drains the ring's trailing LDS-DMA fills), workgroup barrier, lane 0 takes a
// relaxed agent-scope ticket.  The ticket SK - 1 is the last arriver: it resets the counter for the next
// launch, reads EVERY slab (its own included) with sc1 loads and sums them in slice order, so the value is
// the same whichever workgroup combines.  Correct for any placement of the slices over CUs / XCDs.
template <int BTM, int SK>
STZS_DEV bool splitk_combine(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem) {
    constexpr int NV = BTM / 32 * 4;         // f32x4 accumulators per thread
    constexpr int SLAB = NV * NTHR * 16;     // bytes per (tile, slice)
    const int tid = threadIdx.x;
    const long tile = blockIdx.x + (long)gridDim.x * blockIdx.y;
    unsigned char* base = reinterpret_cast<unsigned char*>(a.splitk_ws) + tile * (long)(SK * SLAB);
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(base, 0, SK * SLAB, 0x00020000);
    const int z = blockIdx.z;
#pragma unroll
    for (int i = 0; i < NV; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i >> 2][i & 3]), wr,
                                               (z * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(smem);  // the ring is idle: its fills drained above
    if (tid == 0) {
        typedef __attribute__((address_space(1))) unsigned int gu32;
        gu32* ctr = (gu32*)(a.splitk_ctr + tile);
        const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        const int last = old == (unsigned)(SK - 1);
        if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
        *flag = last;
    }
    __syncthreads();
    if (!*flag) return false;
    u32x4 v[SK][NV];
#pragma unroll
    for (int s = 0; s < SK; ++s)
#pragma unroll
        for (int i = 0; i < NV; ++i)
            v[s][i] = __builtin_amdgcn_raw_buffer_load_b128(wr, (s * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
#pragma unroll
    for (int i = 0; i < NV; ++i) {
        f32x4 t = __builtin_bit_cast(f32x4, v[0][i]);
#pragma unroll
        for (int s = 1; s < SK; ++s) t += __builtin_bit_cast(f32x4, v[s][i]);
        acc[i >> 2][i & 3] = t;
    }
    return true;
}

// the gemm_glds instance with the launch's epilogue variant compiled in (EP, finish)
template <typename TOut, int BTM, bool F8, int SK>
void (*pick_gemm(int ep))(stzs_conv_args) {
    switch (ep) {
#define STZS_EPK(e) case e: return gemm_glds<TOut, BTM, F8, SK, e>;
        STZS_EPK(0) STZS_EPK(1) STZS_EPK(2) STZS_EPK(3) STZS_EPK(4) STZS_EPK(5) STZS_EPK(6) STZS_EPK(7)
        STZS_EPK(8) STZS_EPK(9) STZS_EPK(10) STZS_EPK(11) STZS_EPK(12) STZS_EPK(13) STZS_EPK(14) STZS_EPK(15)
#undef STZS_EPK
        default: return gemm_glds<TOut, BTM, F8, SK, -1>;
    }
}

template <typename TOut, bool F8>
int gemm_launch(const stzs_conv_args& a, hipStream_t s) {
    dim3 grid((unsigned)(((long)a.B * a.T_out + BT - 1) / BT), a.co_pad / BCO);
    // tile height by wave quantisation: 128-row tiles run two workgroups per CU, 64-row tiles three; a 64-row tile
    // costs ~0.6 of a 128-row one (the fill and the epilogue do not halve).  STZS_GEMM_TILE=64|128 forces one.
    const long n_cu = stzs_cu_count();
    const long n128 = (long)grid.x * grid.y, n64 = (((long)a.B * a.T_out + 63) / 64) * grid.y;
    const long r128 = (n128 + 2 * n_cu - 1) / (2 * n_cu), r64 = (n64 + 3 * n_cu - 1) / (3 * n_cu);
    bool small = 6 * r64 < 10 * r128;
    static const int force = [] {
        const char* e = getenv("STZS_GEMM_TILE");
        return e ? atoi(e) : 0;
    }();
    if (force == 64 || force == 128) small = force == 64;
    size_t lg = small ? gemm_lds<64>() : gemm_lds<128>();
    const int ep = ep_index(a, epi_vec(a));
    auto kg = small ? pick_gemm<TOut, 64, F8, 1>(ep) : pick_gemm<TOut, 128, F8, 1>(ep);
    if (a.splitk > 1) {  // split-K: 64-row tiles at every row count (the K order must not depend on M)
        const int NK = a.ci_pad / 32;
        if (F8 || (a.splitk != 2 && a.splitk != 4) || NK % a.splitk || !a.splitk_ws || !a.splitk_ctr ||
            !stzs_aligned(a.splitk_ws, 16) || !stzs_aligned(a.splitk_ctr, 4))
            return STZS_EINVAL;
        if constexpr (!F8) kg = a.splitk == 2 ? pick_gemm<TOut, 64, false, 2>(ep) : pick_gemm<TOut, 64, false, 4>(ep);
        small = true;
        grid.z = (unsigned)a.splitk;
        lg = gemm_lds<64>();
    }
    if (small) grid.x = (unsigned)(((long)a.B * a.T_out + 63) / 64);
    (void)hipFuncSetAttribute((const void*)kg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lg);
    hipLaunchKernelGGL(kg, grid, dim3(NTHR), lg, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

}  // namespace

// internal entry (csrc/conv.hip stzs_conv1d_core): a validated flat linear with LDS-DMA-readable rows, bf16 or fp8 in
__attribute__((visibility("hidden"))) int stzs_gemm_glds_launch(const stzs_conv_args& a, hipStream_t s) {
    const bool f8 = a.in_dtype == STZS_F8;
    if (a.out_dtype == STZS_BF16) return f8 ? gemm_launch<bf16_t, true>(a, s) : gemm_launch<bf16_t, false>(a, s);
    if (a.out_dtype == STZS_F32) return f8 ? gemm_launch<float, true>(a, s) : gemm_launch<float, false>(a, s);
    return STZS_EDTYPE;
}
