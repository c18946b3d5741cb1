// Small-M linear on the whole chip (STZS_CONV_ROWS): the batch-1 denoiser linears of configs[1] (SURVEY.md
// §8(a) a2: 100 CFG rows x d 512; at B = 1 "weight-BW and launch bound").
//
// gemm_glds gives a linear co_pad/128 x ceil(M/64) workgroups (ffn2 at M = 100: 8), each streaming ALL of K for
// its 128 columns through one CU's LDS-DMA ring (~35-55 GB/s per CU): ffn2 takes 15 us for 2 MB of weights.  Here
// a workgroup owns a 16-COLUMN tile, every row of the (small) row block and 1/Z of K, so a linear spreads over
// N/16 x Z workgroups (qkv 96, ff1 128, ffn2 at Z = 4: 128) and each CU reads 8-32 KB of weights:
//   * operands go straight to VGPRs in MFMA fragment order, no LDS staging and no ring: the B fragment of a
//     16-column K-step is 16 rows x 64 B of the packed KSTEP stream = ONE contiguous 1 KB (the XOR swizzle only
//     permutes lanes), the A fragments are the activation rows (L2-resident, shared by every column tile);
//   * the 4 waves take interleaved K-steps (wave w: z NKZ + w, + 4, ...), every load of a wave issued before its
//     first MFMA (a 4-K-step register ring beyond 4 per wave), v_mfma_f32_16x16x32_bf16 into fp32;
//   * the 4 wave partials are summed in LDS in wave order; with Z > 1 the workgroup publishes its partial with
//     16-B write-through stores and takes a ticket, and the tile's LAST arriver sums the Z partials in z order
//     (the in-launch split-K hand-off of csrc/conv.hip) before the epilogue;
//   * epilogue operands (bias, residual, accumulate-input) are loaded at kernel entry, so their latency hides
//     under the K loop; the fused epilogue is gemm_glds': bias, GELU / SiLU / LeakyReLU, the per-utterance DiT
//     gate, residual, alpha, beta * acc_in.
// The summation order of an output element -- sequential MFMA chain per wave, waves 0..3, then slices 0..Z-1 --
// depends on K and Z only, never on the row count: results are batch-invariant (row blocks of up to 128 rows
// tile larger M with identical per-element arithmetic).
#include "common.hpp"

namespace {

constexpr int NTHR = 256;

STZS_DEV int gswz(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }

STZS_DEV float fast_erf(float x) {  // Abramowitz & Stegun 7.1.26, as csrc/conv.hip
    const float ax = fabsf(x);
    const float t = __builtin_amdgcn_rcpf(fmaf(0.3275911f, ax, 1.f));
    const float p = t * fmaf(t, fmaf(t, fmaf(t, fmaf(t, 1.061405429f, -1.453152027f), 1.421413741f), -0.284496736f),
                             0.254829592f);
    const float y = 1.f - p * __expf(-ax * ax);
    return copysignf(y, x);
}

template <int EACT>
STZS_DEV float epi_act(float x, float slope) {
    if constexpr (EACT == STZS_ACT_GELU) return 0.5f * x * (1.f + fast_erf(x * 0.70710678118654752f));
    else if constexpr (EACT == STZS_ACT_SILU) return x / (1.f + __expf(-x));
    else if constexpr (EACT == STZS_ACT_LEAKY) return x >= 0.f ? x : x * slope;
    else return x;
}

typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
typedef __attribute__((address_space(1))) unsigned int gu32;

// A fragment of 16 rows x 32 k from TIn rows (bf16: one 16-B load; fp32: two, scaled by cscale and rounded RNE)
template <typename TIn> struct AFrag;
template <> struct AFrag<bf16_t> {
    typedef uint4 R;
    static STZS_DEV R load(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
    static STZS_DEV bf16x8 cvt(const R& r, float) { return __builtin_bit_cast(bf16x8, r); }
};
struct F8x { float4 a, b; };
template <> struct AFrag<float> {
    typedef F8x R;
    static STZS_DEV R load(const float* p) {
        return F8x{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
    }
    static STZS_DEV bf16x8 cvt(const R& r, float sc) {
        const float v[8] = {r.a.x * sc, r.a.y * sc, r.a.z * sc, r.a.w * sc, r.b.x * sc, r.b.y * sc, r.b.z * sc, r.b.w * sc};
        return __builtin_bit_cast(bf16x8, pack8(v));
    }
};

template <typename TIn, typename TOut, int MT, int KPW, int EACT, bool SPLIT>
__global__ __launch_bounds__(NTHR) void gemm_rows(const stzs_conv_args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[4 * MT * 64 * 16];
    auto red = reinterpret_cast<float4 (*)[MT][64]>(lds);
    __shared__ int s_last;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int ct = blockIdx.x;               // 16-column tile
    const int r0 = blockIdx.y * (16 * MT);   // row block
    const int z = blockIdx.z, Z = gridDim.z;
    const int T = a.T_in, nR = a.B * T;
    const int NK = a.ci_pad / 32;
    const int NKZ = NK / Z;
    const int kbase = z * NKZ + wave;  // this wave's K-steps: kbase + 4 j, j < KPW
    // flat row R -> (utterance, step): q = trunc(R * (1 / T)) is within one of R / T for R < 2^22, one
    // correction step makes it exact (a handful of VALU ops instead of hipcc's integer-division expansion)
    const float invT = 1.f / (float)T;
    auto bdiv = [&](int R) -> int {
        int q = (int)((float)R * invT);
        const int r = R - q * T;
        q += r < 0 ? -1 : (r >= T ? 1 : 0);
        return q;
    };
    auto roff = [&](int R, int64_t ld, int64_t bs) -> int64_t {
        R = R < nR ? R : nR - 1;
        const int bb = bdiv(R);
        return (int64_t)bb * bs + (int64_t)(R - bb * T) * ld;
    };
    // ---- epilogue operands first: UNCONDITIONAL loads from valid addresses (an absent operand reads a stand-in and
    // is dropped by a select), so hipcc keeps them in flight under the K loop instead of draining each one ----
    // slot (mt, lane) holds rows r0 + mt*16 + (lane>>4)*4 + i (i < 4) of column n = ct*16 + (lane & 15); thread tid
    // owns slots tid + 256 s
    constexpr int NSLOT = (MT * 64 + NTHR - 1) / NTHR;
    const int n = ct * 16 + (lane & 15);
    const bool col_ok = n < a.Co;
    const int nc = col_ok ? n : a.Co - 1;
    const bool hr = a.res != nullptr, ha = a.acc_in != nullptr, hg = a.gate != nullptr, hb = a.bias != nullptr;
    const TOut* Rp = reinterpret_cast<const TOut*>(hr ? a.res : a.y);
    const TOut* AI = reinterpret_cast<const TOut*>(ha ? a.acc_in : a.y);
    const int64_t ldr = hr ? a.ldr : a.ldy, bsr = hr ? a.bsr : a.bsy, lda = ha ? a.lda : a.ldy, bsa = ha ? a.bsa : a.bsy;
    const float* stand_in = reinterpret_cast<const float*>(a.w);  // >= 64 B per output column: index nc is valid
    const float braw = (hb ? a.bias : stand_in)[nc];
    float res_v[NSLOT][4], ai_v[NSLOT][4], g_v[NSLOT][4];
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
        const int mt = ((tid + s * NTHR) >> 6) % MT;  // slots past MT*64 (none for MT 4 / 8) alias valid rows
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = r0 + mt * 16 + (lane >> 4) * 4 + i;
            res_v[s][i] = DT<TOut>::ld(Rp + roff(R, ldr, bsr) + nc);
            ai_v[s][i] = DT<TOut>::ld(AI + roff(R, lda, bsa) + nc);
            const int Rc = R < nR ? R : nR - 1;
            g_v[s][i] = (hg ? a.gate : stand_in)[hg ? (int64_t)bdiv(Rc) * a.gate_bs + nc : (int64_t)nc];
        }
    }
    // ---- operand addresses ----
    const TIn* X = reinterpret_cast<const TIn*>(a.x);
    int64_t aoff[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) aoff[mt] = roff(r0 + mt * 16 + (lane & 15), a.ldx, a.bsx) + 8 * (lane >> 4);
    const int cot = ct >> 3, rr = (ct & 7) * 16 + (lane & 15);
    const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.w) + ((int64_t)cot * NK * 128 + rr) * 64 +
                              (((lane >> 4) ^ gswz(rr)) << 4);
    const float sc = a.pro_cscale;
    constexpr int RING = sizeof(TIn) == 2 ? 4 : 2;  // K-steps per wave whose loads are in flight
    using AR = typename AFrag<TIn>::R;
    AR ar[RING][MT];
    uint4 br[RING];
    auto issue = [&](int j) {
        const int k = kbase + 4 * j;
        const int slot = j % RING;
        br[slot] = *reinterpret_cast<const uint4*>(Wb + (int64_t)k * 128 * 64);
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) ar[slot][mt] = AFrag<TIn>::load(X + aoff[mt] + k * 32);
    };
    f32x4 acc[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < (KPW < RING ? KPW : RING); ++j) issue(j);
    // keep every issued load ahead of the first MFMA (hipcc otherwise interleaves them to save registers, leaving
    // only a few loads in flight per wave)
    __builtin_amdgcn_sched_barrier(0);
#pragma unroll
    for (int j = 0; j < KPW; ++j) {
        const int slot = j % RING;
        const bf16x8 fb = __builtin_bit_cast(bf16x8, br[slot]);
        bf16x8 fa[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) fa[mt] = AFrag<TIn>::cvt(ar[slot][mt], sc);
        if (j + RING < KPW) {
            issue(j + RING);
            __builtin_amdgcn_sched_barrier(0);
        }
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa[mt], fb, acc[mt], 0, 0, 0);
    }
    // ---- the 4 wave partials, summed in wave order ----
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) red[wave][mt][lane] = make_float4(acc[mt][0], acc[mt][1], acc[mt][2], acc[mt][3]);
    __syncthreads();
    f32x4 v[NSLOT];
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
        const int slot = tid + s * NTHR;
        if (slot < MT * 64) {
            const int mt = slot >> 6, l = slot & 63;
            const float4 p0 = red[0][mt][l], p1 = red[1][mt][l], p2 = red[2][mt][l], p3 = red[3][mt][l];
            v[s] = f32x4{((p0.x + p1.x) + p2.x) + p3.x, ((p0.y + p1.y) + p2.y) + p3.y, ((p0.z + p1.z) + p2.z) + p3.z,
                         ((p0.w + p1.w) + p2.w) + p3.w};
        }
    }
    if constexpr (SPLIT) {
        // in-launch split-K hand-off: slab [tile][z][slot] f32x4, write-through stores, drain, barrier, ticket
        const int64_t tile = (int64_t)blockIdx.y * gridDim.x + ct;
        const int SLAB = MT * 64 * 16;
        unsigned char* base = reinterpret_cast<unsigned char*>(a.splitk_ws) + tile * (int64_t)Z * SLAB;
        const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(base, 0, Z * SLAB, 0x00020000);
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) {
            const int slot = tid + s * NTHR;
            if (slot < MT * 64) __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, v[s]), wr, z * SLAB + slot * 16, 0, 16);
        }
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            gu32* ctr = (gu32*)(a.splitk_ctr + tile);
            const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == (unsigned)(Z - 1);
            if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
#pragma unroll
        for (int s = 0; s < NSLOT; ++s) {
            const int slot = tid + s * NTHR;
            if (slot < MT * 64) {
                u32x4 pv[16];
                for (int q = 0; q < Z; ++q)  // every slab (its own too) by sc1 loads, all in flight
                    pv[q] = __builtin_amdgcn_raw_buffer_load_b128(wr, q * SLAB + slot * 16, 0, 16);
                f32x4 t = __builtin_bit_cast(f32x4, pv[0]);
                for (int q = 1; q < Z; ++q) t += __builtin_bit_cast(f32x4, pv[q]);  // slice order
                v[s] = t;
            }
        }
    }
    // ---- fused epilogue ----
    TOut* Y = reinterpret_cast<TOut*>(a.y);
    const float bias = hb ? braw : 0.f;
#pragma unroll
    for (int s = 0; s < NSLOT; ++s) {
        const int slot = tid + s * NTHR;
        if (slot >= MT * 64 || !col_ok) continue;
        const int mt = slot >> 6;
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = r0 + mt * 16 + (lane >> 4) * 4 + i;
            if (R >= nR) break;
            float x = epi_act<EACT>(v[s][i] + bias, a.epi_slope);
            x = hg ? x * g_v[s][i] : x;
            x = hr ? x + res_v[s][i] : x;
            x *= a.alpha;
            x = ha ? x + a.beta * ai_v[s][i] : x;
            DT<TOut>::st(Y + roff(R, a.ldy, a.bsy) + n, x);
        }
    }
}

// epilogue activations: none, GELU (ffn1), SiLU (the sigma-embedding MLP)
template <typename TIn, typename TOut, int MT, int KPW, bool SPLIT>
void* pick_act(int act) {
    switch (act) {
        case STZS_ACT_GELU: return (void*)gemm_rows<TIn, TOut, MT, KPW, STZS_ACT_GELU, SPLIT>;
        case STZS_ACT_SILU: return (void*)gemm_rows<TIn, TOut, MT, KPW, STZS_ACT_SILU, SPLIT>;
        case STZS_ACT_NONE: return (void*)gemm_rows<TIn, TOut, MT, KPW, STZS_ACT_NONE, SPLIT>;
        default: return nullptr;
    }
}

template <typename TIn, typename TOut, int MT>
void* pick_kpw(int kpw, bool split, int act) {
#define STZS_ROWS_K(n) \
    case n: return split ? pick_act<TIn, TOut, MT, n, true>(act) : pick_act<TIn, TOut, MT, n, false>(act);
    switch (kpw) {
        STZS_ROWS_K(1)
        STZS_ROWS_K(2)
        STZS_ROWS_K(4)
        STZS_ROWS_K(8)
        STZS_ROWS_K(16)
        default: return nullptr;
    }
#undef STZS_ROWS_K
}

template <typename TIn, typename TOut>
void* pick(int mt, int kpw, bool split, int act) {
    return mt == 4 ? pick_kpw<TIn, TOut, 4>(kpw, split, act) : pick_kpw<TIn, TOut, 8>(kpw, split, act);
}

}  // namespace

// 16-row tiles per workgroup: 64-row blocks up to 64 rows, 128-row blocks beyond (speed only: the per-element
// arithmetic does not depend on the row blocking)
static int rows_mt(long M) { return M <= 64 ? 4 : 8; }

extern "C" size_t stzs_conv_rows_workspace(int64_t rows, int32_t Co, int32_t kgroups) {
    if (rows <= 0 || Co <= 0 || kgroups < 1) return 0;
    const int mt = rows_mt(rows);
    const long nblk = (rows + 16 * mt - 1) / (16 * mt);
    const long tiles = nblk * ((Co + 15) / 16);
    if (kgroups <= 1) return 0;
    const size_t rows_form = (size_t)tiles * kgroups * mt * 64 * 16;
    // the K-slice form of csrc/lnrows.hip (rows16 split, stzs_ln_linear with ln = NULL) writes one 4-KB slab per
    // (16-row x 64-column tile, slice): larger than this file's layout when Co % 64 is in (0, 48]
    const size_t r16 = (size_t)((rows + 15) / 16) * ((Co + 63) / 64) * kgroups * 4096;
    return rows_form > r16 ? rows_form : r16;
}

// validates the linear and launches
int stzs_rows_gemm_launch(const stzs_conv_args& a, hipStream_t s) {
    const bool lin = a.ks == 1 && a.stride == 1 && a.pad == 0 && a.ups == 0 && a.T_in == a.T_out &&
                     a.pro_mode == STZS_PRO_NONE && a.pro_act == STZS_ACT_NONE && !a.stat_part && !a.x_scale;
    if (!lin || (a.flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_W_X3 |
                            STZS_CONV_W_FRAG32)))
        return STZS_EINVAL;
    if (a.in_dtype == STZS_F8) return STZS_EDTYPE;
    if (a.in_dtype == STZS_BF16 ? a.pro_cscale != 1.f : false) return STZS_EINVAL;
    if (a.res && a.res_tdiv != 1) return STZS_EINVAL;  // gemm_rows reads the residual at the output row itself
    const int NK = a.ci_pad / 32;
    const int Z = a.splitk > 1 ? a.splitk : 1;
    if (a.ci_pad % 32 || NK % (4 * Z) || Z > 16) return STZS_ESHAPE;  // every wave of every slice runs the same K-step count
    const int kpw = NK / (4 * Z);
    if (kpw != 1 && kpw != 2 && kpw != 4 && kpw != 8 && kpw != 16) return STZS_ESHAPE;
    if (Z > 1 && (!a.splitk_ws || !a.splitk_ctr || !stzs_aligned(a.splitk_ws, 16) || !stzs_aligned(a.splitk_ctr, 4)))
        return STZS_EINVAL;
    if (a.ldx < a.ci_pad && a.in_dtype == STZS_BF16) return STZS_ESHAPE;  // fragments read [0, ci_pad) of each row
    if (a.in_dtype == STZS_F32 && a.ldx < a.ci_pad) return STZS_ESHAPE;
    const long M = (long)a.B * a.T_in;
    const int mt = rows_mt(M);
    dim3 grid((unsigned)((a.Co + 15) / 16), (unsigned)((M + 16 * mt - 1) / (16 * mt)), (unsigned)Z);
    void* k = nullptr;
    const bool split = Z > 1;
    if (a.in_dtype == STZS_BF16 && a.out_dtype == STZS_BF16) k = pick<bf16_t, bf16_t>(mt, kpw, split, a.epi_act);
    else if (a.in_dtype == STZS_BF16 && a.out_dtype == STZS_F32) k = pick<bf16_t, float>(mt, kpw, split, a.epi_act);
    else if (a.in_dtype == STZS_F32 && a.out_dtype == STZS_F32) k = pick<float, float>(mt, kpw, split, a.epi_act);
    else return STZS_EDTYPE;
    if (!k) return STZS_EINVAL;  // an epilogue activation this form does not instantiate
    hipLaunchKernelGGL(reinterpret_cast<void (*)(stzs_conv_args)>(k), grid, dim3(NTHR), 0, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
