// LayerNorm-fed small-M linear in ONE launch: y = epilogue(LN(x) W^T) (the configs[1] batch-1 denoiser, SURVEY.md
// §8(a) a2: every adaLN / affine LayerNorm of a DiT layer feeds exactly one linear -- qkv, the cross-attention query,
// ffn1, the output projection).  At 200 rows stzs_row_layernorm + the rows GEMM were two launches (~4.8 + ~8 us,
// profiles/r04_j_lat_trace.txt: 196 LayerNorm launches of the 913 per batch-1 synthesis).
//
// A workgroup owns 16 rows (one MFMA row tile) and 64 output columns (4 waves x one 16-column tile):
//   * at entry every wave puts ALL K-steps of its weight tile in flight (one 16-B load per lane per K-step of the
//     STZS_PACK_KSTEP stream, as csrc/rows.hip reads it), and each 16-lane group loads one row (lane: 8-value vectors
//     l, l + 16, ...) with the modulation vectors of the row's group;
//   * two-pass statistics over the 16 lanes (xor 8, 4, 2, 1), (gadd + G) x_hat + Bt rounded to bf16 (RNE) into an LDS
//     operand image [16 rows][K] (16-B row skew): the LayerNorm of stzs_row_layernorm with its sums associated per
//     16-lane group instead of per wave (within one bf16 ulp of it; tests/test_gpu_lnrows.py);
//   * one barrier, then each wave runs its 16 columns over all of K: A fragments from LDS, B from registers,
//     v_mfma_f32_16x16x32_bf16 in one sequential chain per output element (K order only: batch-invariant);
//   * epilogue as the rows GEMM: bias, NONE | GELU | SILU, alpha, beta * acc_in.
// Every column group recomputes its rows' LayerNorm from L2-resident rows (qkv at 100 rows: 24 column groups x 7 row
// blocks, 16 KB of rows each) instead of a launch and a global round trip of the normalised rows.  The first form (64
// rows per workgroup, one row per wave at a time) spent ~12 us per launch in the per-wave row loop (r04_q).
#include "conv_common.hpp"

namespace {

constexpr int LR_ROWS = 16;  // rows per workgroup (one 16-row MFMA tile; 4 rows per wave in the LayerNorm)

// sum over the 16 lanes of a lane group: the xor-8, 4, 2, 1 butterfly on DPP row rotations (r06; it ran on ds_bpermute
// shuffles).  After the xor-8 step every value has period 8 within the row (x_j + x_(j^8) == x_(j^8) + x_j bitwise),
// so rotating by 4 fetches exactly the xor-4 partner's value, and likewise by 2 and 1: the same bits as the shuffles.
STZS_DEV float sum16(float v) {
    v += dpp_f32<0x128>(v);  // row_ror:8 (= xor 8)
    v += dpp_f32<0x124>(v);  // row_ror:4
    v += dpp_f32<0x122>(v);  // row_ror:2
    v += dpp_f32<0x121>(v);  // row_ror:1
    return v;
}

template <typename TI, typename TOut, int NK, int EACT>
__global__ __launch_bounds__(NTHR) void ln_rows(const stzs_conv_args a, const stzs_rowln_args ln) {
    constexpr int K = NK * 32;
    constexpr int PITCH = K * 2 + 16;  // bytes per LDS row (16-B skew: conflict-free fragment reads)
    constexpr int NV = NK / 4;         // 8-value vectors per lane of its row (16 lanes per row)
    __shared__ __attribute__((aligned(16))) unsigned char lds[LR_ROWS * PITCH];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nR = ln.R;
    const int r0 = blockIdx.y * LR_ROWS;
    // ---- this wave's 16-column weight tile: every K-step in flight from the start ----
    const int ct = blockIdx.x * 4 + wave;
    const bool wact = ct * 16 < a.Co;  // (wave-uniform)
    const int ctc = wact ? ct : 0;
    const int cot = ctc >> 3, rr = (ctc & 7) * 16 + (lane & 15);
    const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.w) + ((int64_t)cot * NK * 128 + rr) * 64 +
                              (((lane >> 4) ^ gswz(rr)) << 4);
    uint4 br[NK];
#pragma unroll
    for (int j = 0; j < NK; ++j) br[j] = *reinterpret_cast<const uint4*>(Wb + (int64_t)j * 128 * 64);
    // ---- LayerNorm: row wave * 4 + (lane >> 4) of the block on a 16-lane group, vectors (lane & 15) + 16 m ----
    const int rl = wave * 4 + (lane >> 4);
    const int r = r0 + rl < nR ? r0 + rl : nR - 1;
    const int l16 = lane & 15;
    const TI* X = reinterpret_cast<const TI*>(ln.x) + (int64_t)r * ln.ldx;
    const long grp = (ln.gs == 0 && ln.bs == 0) ? 0 : r / ln.gdiv;
    float v[NV][8], g[NV][8], bt[NV][8];
#pragma unroll
    for (int m = 0; m < NV; ++m) {
        load8(X + (l16 + 16 * m) * 8, v[m]);
        if (ln.G) load8(ln.G + grp * ln.gs + (l16 + 16 * m) * 8, g[m]);
        if (ln.Bt) load8(ln.Bt + grp * ln.bs + (l16 + 16 * m) * 8, bt[m]);
    }
    float s = 0.f;
#pragma unroll
    for (int m = 0; m < NV; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) s += v[m][j];
    const float mu = sum16(s) / (float)K;
    float q = 0.f;
#pragma unroll
    for (int m = 0; m < NV; ++m)
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float d = v[m][j] - mu;
            q += d * d;
        }
    const float rstd = 1.f / sqrtf(sum16(q) / (float)K + ln.eps);
    unsigned char* dst = lds + rl * PITCH;
#pragma unroll
    for (int m = 0; m < NV; ++m) {
        float o[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            const float gg = ln.gadd + (ln.G ? g[m][j] : 0.f);
            o[j] = (v[m][j] - mu) * rstd * gg + (ln.Bt ? bt[m][j] : 0.f);
        }
        *reinterpret_cast<uint4*>(dst + (l16 + 16 * m) * 16) = pack8(o);
    }
    __syncthreads();
    if (!wact) return;
    // ---- 16 rows x 16 columns over all of K ----
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* A0 = lds + (lane & 15) * PITCH + (lane >> 4) * 16;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
        const bf16x8 fa = *reinterpret_cast<const bf16x8*>(A0 + j * 64);
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, __builtin_bit_cast(bf16x8, br[j]), acc, 0, 0, 0);
    }
    // ---- epilogue (csrc/rows.hip's order: act(v + bias), alpha, + beta acc_in) ----
    const int n = ct * 16 + (lane & 15);
    if (n >= a.Co) return;
    const float bias = a.bias ? a.bias[n] : 0.f;
    const TOut* AI = reinterpret_cast<const TOut*>(a.acc_in);
    TOut* Y = reinterpret_cast<TOut*>(a.y);
    const int T = a.T_in;
    const float invT = 1.f / (float)T;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = r0 + (lane >> 4) * 4 + i;
        if (R >= nR) continue;
        float x = epi_act<EACT>(acc[i] + bias, a.epi_slope);
        x *= a.alpha;
        const long bb = rowdiv(R, T, invT, true);
        const long t = R - bb * T;
        if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + t * a.lda + n);
        DT<TOut>::st(Y + bb * a.bsy + t * a.ldy + n, x);
    }
}

// The plain small-M linear on 16-row workgroups of WPG 16-column tiles (stzs_ln_linear with ln = NULL; the batch-1
// denoiser's attention output projections, ffn2 and input projection, the per-utterance linears): A fragments
// straight from the x rows into registers (bf16, or fp32 x pro_cscale rounded to bf16 as csrc/rows.hip), up to 16
// K-steps of both operands in flight, no LDS; the epilogue adds the FLAT DiT gate and the residual.
// SPLIT (splitk = Z in {2, 4}): workgroup z runs K-steps [z NKS, (z+1) NKS) and hands its fp32 partials to the tile's
// last arriver as csrc/rows.hip does (16-B write-through stores, drain, barrier, agent-scope ticket; the last arriver
// sums the Z slabs in slice order with sc1 loads): the value does not depend on the arrival order or the row count.
template <typename TI, typename TOut, int NKS, int EACT, bool SPLIT, int WPG = 4>
__global__ __launch_bounds__(NTHR) void rows16(const stzs_conv_args a) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int T = a.T_in, nR = a.B * T;
    const int r0 = blockIdx.y * LR_ROWS;
    const int ct = blockIdx.x * WPG + wave;  // (WPG waves per workgroup, one 16-column tile each)
    if (!SPLIT && ct * 16 >= a.Co) return;  // (wave-uniform; no barrier without K slices)
    const int ctc = ct * 16 < a.Co ? ct : 0;  // (with K slices every wave reaches the barriers)
    const int NK = a.ci_pad / 32, kz = SPLIT ? (int)blockIdx.z * NKS : 0;
    const int cot = ctc >> 3, rr = (ctc & 7) * 16 + (lane & 15);
    const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.w) +
                              (((int64_t)cot * NK + kz) * 128 + rr) * 64 + (((lane >> 4) ^ gswz(rr)) << 4);
    // K-steps in flight per wave: all of them up to 16 (fp32 A: 8), then a ring refilled as each is consumed
    constexpr int CH = NKS < (sizeof(TI) == 2 ? 16 : 8) ? NKS : (sizeof(TI) == 2 ? 16 : 8);
    const float invT = 1.f / (float)T;
    int Ra = r0 + (lane & 15);  // this lane's A row; k offset 8 (lane >> 4) in every K-step
    Ra = Ra < nR ? Ra : nR - 1;
    const long ba = rowdiv(Ra, T, invT, true);
    const TI* X = reinterpret_cast<const TI*>(a.x) + ba * a.bsx + (Ra - ba * T) * a.ldx + (lane >> 4) * 8 + kz * 32;
    uint4 br[CH];
    typename Raw<TI>::T ar[CH];
#pragma unroll
    for (int j = 0; j < CH; ++j) {
        br[j] = *reinterpret_cast<const uint4*>(Wb + (int64_t)j * 128 * 64);
        ar[j] = Raw<TI>::load(X + j * 32);
    }
    // every load issued before the first MFMA (hipcc otherwise interleaves them to save registers)
    __builtin_amdgcn_sched_barrier(0);
    f32x4 acc = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
    for (int j = 0; j < NKS; ++j) {
        bf16x8 fa;
        if constexpr (sizeof(TI) == 2) {
            fa = __builtin_bit_cast(bf16x8, ar[j % CH]);
        } else {
            float v[8];
            Raw<TI>::cvt(ar[j % CH], v);
#pragma unroll
            for (int e = 0; e < 8; ++e) v[e] *= a.pro_cscale;
            fa = __builtin_bit_cast(bf16x8, pack8(v));
        }
        const bf16x8 fb = __builtin_bit_cast(bf16x8, br[j % CH]);
        if (j + CH < NKS) {
            br[j % CH] = *reinterpret_cast<const uint4*>(Wb + (int64_t)(j + CH) * 128 * 64);
            ar[j % CH] = Raw<TI>::load(X + (j + CH) * 32);
        }
        acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc, 0, 0, 0);
    }
    if constexpr (SPLIT) {
        __shared__ int s_last;
        const int Z = gridDim.z, z = blockIdx.z;
        constexpr int SLAB = NTHR * 16;  // one f32x4 per thread
        const int64_t tile = (int64_t)blockIdx.y * gridDim.x + blockIdx.x;
        unsigned char* base = reinterpret_cast<unsigned char*>(a.splitk_ws) + tile * (int64_t)Z * SLAB;
        const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(base, 0, Z * SLAB, 0x00020000);
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc), wr, z * SLAB + tid * 16, 0, 16);
        asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
        __syncthreads();
        if (tid == 0) {
            typedef __attribute__((address_space(1))) unsigned int gu32;
            gu32* ctr = (gu32*)(a.splitk_ctr + tile);
            const unsigned old = __hip_atomic_fetch_add(ctr, 1u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            const int last = old == (unsigned)(Z - 1);
            if (last) __hip_atomic_store(ctr, 0u, __ATOMIC_RELAXED, __HIP_MEMORY_SCOPE_AGENT);
            s_last = last;
        }
        __syncthreads();
        if (!s_last) return;
        u32x4 pv[4];
#pragma unroll
        for (int q = 0; q < 4; ++q)  // every slab (its own too) by sc1 loads, all in flight
            if (q < Z) pv[q] = __builtin_amdgcn_raw_buffer_load_b128(wr, q * SLAB + tid * 16, 0, 16);
        acc = __builtin_bit_cast(f32x4, pv[0]);
#pragma unroll
        for (int q = 1; q < 4; ++q)  // slice order
            if (q < Z) acc += __builtin_bit_cast(f32x4, pv[q]);
        if (ct * 16 >= a.Co) return;
    }
    // ---- epilogue (csrc/rows.hip's order: act(v + bias), gate, + residual, alpha, + beta acc_in) ----
    const int n = ct * 16 + (lane & 15);
    if (n >= a.Co) return;
    const float bias = a.bias ? a.bias[n] : 0.f;
    const TOut* Rp = reinterpret_cast<const TOut*>(a.res);
    const TOut* AI = reinterpret_cast<const TOut*>(a.acc_in);
    TOut* Y = reinterpret_cast<TOut*>(a.y);
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int R = r0 + (lane >> 4) * 4 + i;
        if (R >= nR) continue;
        const long bb = rowdiv(R, T, invT, true);
        const long t = R - bb * T;
        float x = epi_act<EACT>(acc[i] + bias, a.epi_slope);
        if (a.gate) x *= a.gate[bb * a.gate_bs + n];
        if (Rp) x += DT<TOut>::ld(Rp + bb * a.bsr + t * a.ldr + n);
        x *= a.alpha;
        if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + t * a.lda + n);
        DT<TOut>::st(Y + bb * a.bsy + t * a.ldy + n, x);
    }
}

template <typename TI, typename TOut, int NKS, bool SPLIT, int WPG = 4>
void* pick_plain_act(int act) {
    switch (act) {
        case STZS_ACT_GELU: return (void*)rows16<TI, TOut, NKS, STZS_ACT_GELU, SPLIT, WPG>;
        case STZS_ACT_SILU: return (void*)rows16<TI, TOut, NKS, STZS_ACT_SILU, SPLIT, WPG>;
        case STZS_ACT_NONE: return (void*)rows16<TI, TOut, NKS, STZS_ACT_NONE, SPLIT, WPG>;
        default: return nullptr;
    }
}

// nks: K-steps per slice; split: Z > 1 (slices of 4 / 8 / 16 K-steps)
template <typename TI, typename TOut>
void* pick_plain(int nks, bool split, int act, int wpg) {
    if (wpg == 2 && !split) {  // 2-wave, 32-column workgroups
        switch (nks) {
            case 4: return pick_plain_act<TI, TOut, 4, false, 2>(act);
            case 8: return pick_plain_act<TI, TOut, 8, false, 2>(act);
            case 16: return pick_plain_act<TI, TOut, 16, false, 2>(act);
            default: return nullptr;
        }
    }
    if (wpg == 1 && !split) {  // one-wave, 16-column workgroups (the default)
        switch (nks) {
            case 4: return pick_plain_act<TI, TOut, 4, false, 1>(act);
            case 8: return pick_plain_act<TI, TOut, 8, false, 1>(act);
            case 16: return pick_plain_act<TI, TOut, 16, false, 1>(act);
            default: return nullptr;
        }
    }
    if (split) {
        switch (nks) {
            case 4: return pick_plain_act<TI, TOut, 4, true>(act);
            case 8: return pick_plain_act<TI, TOut, 8, true>(act);
            case 16: return pick_plain_act<TI, TOut, 16, true>(act);
            default: return nullptr;
        }
    }
    switch (nks) {
        case 4: return pick_plain_act<TI, TOut, 4, false>(act);
        case 8: return pick_plain_act<TI, TOut, 8, false>(act);
        case 16: return pick_plain_act<TI, TOut, 16, false>(act);
        case 32: return pick_plain_act<TI, TOut, 32, false>(act);
        case 64: return pick_plain_act<TI, TOut, 64, false>(act);
        default: return nullptr;
    }
}

template <typename TI, typename TOut, int NK>
void* pick_act(int act) {
    switch (act) {
        case STZS_ACT_GELU: return (void*)ln_rows<TI, TOut, NK, STZS_ACT_GELU>;
        case STZS_ACT_SILU: return (void*)ln_rows<TI, TOut, NK, STZS_ACT_SILU>;
        case STZS_ACT_NONE: return (void*)ln_rows<TI, TOut, NK, STZS_ACT_NONE>;
        default: return nullptr;
    }
}

template <typename TI, typename TOut>
void* pick(int nk, int act) {
    switch (nk) {
        case 4: return pick_act<TI, TOut, 4>(act);
        case 8: return pick_act<TI, TOut, 8>(act);
        case 16: return pick_act<TI, TOut, 16>(act);
        default: return nullptr;
    }
}

}  // namespace

// (the K-slice form's slabs: ceil(M / 16) x ceil(Co / 64) tiles x Z x 4 KB, which stzs_conv_rows_workspace(M, Co, Z)
// covers (it returns the larger of this layout and csrc/rows.hip's); its tickets: one per tile)
static int plain_launch(const stzs_conv_args* a, hipStream_t s) {
    if (!a->x) return STZS_EINVAL;
    const bool lin = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->T_in == a->T_out &&
                     a->pro_mode == STZS_PRO_NONE && a->pro_act == STZS_ACT_NONE && !a->stat_part && !a->x_scale &&
                     (a->splitk <= 1 || a->splitk == 2 || a->splitk == 4) && (!a->res || a->res_tdiv == 1);
    if (!lin || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_W_X3 |
                             STZS_CONV_W_FRAG32 | STZS_CONV_UPS_NOISE)))
        return STZS_EINVAL;
    const int nk = a->ci_pad / 32, Z = a->splitk > 1 ? a->splitk : 1, nks = nk / Z;
    const bool split = Z > 1;
    if (a->B <= 0 || a->T_in <= 0 || a->Co <= 0 || a->Co > a->co_pad || a->co_pad % 128 || a->Ci > a->ci_pad ||
        a->ci_pad % 32 || nk % Z || (split ? (nks != 4 && nks != 8 && nks != 16)
                                           : (nks != 4 && nks != 8 && nks != 16 && nks != 32 && nks != 64)) ||
        (long)a->B * a->T_in >= (1 << 22) - LR_ROWS)
        return STZS_ESHAPE;
    if (split && (!a->splitk_ws || !a->splitk_ctr || !stzs_aligned(a->splitk_ws, 16) || !stzs_aligned(a->splitk_ctr, 4)))
        return STZS_EINVAL;
    // A rows are read over [0, ci_pad) in 16-B (bf16) / 32-B (fp32) pieces
    if (a->ldx < a->ci_pad || a->ldx % 8 || a->bsx % 8 || !stzs_aligned(a->x, 16)) return STZS_ESHAPE;
    void* k = nullptr;
    if (a->in_dtype == STZS_BF16 && a->pro_cscale != 1.f) return STZS_EINVAL;
    // waves (16-column tiles) per workgroup of the unsliced form: 1 (STZS_ROWS16_WPG = 1 | 2 | 4; the sliced form: 4).
    // More, smaller workgroups: batch-1 p50 6.83 (4) -> 6.65 (2) -> 6.52 ms (1), profiles/r04_af_lat.log, r04_ag_lat.log
    static const int env_wpg = [] {
        const char* e = getenv("STZS_ROWS16_WPG");
        const int v = e ? atoi(e) : 1;
        return v == 2 || v == 4 ? v : 1;
    }();
    const int wpg = (!split && nks <= 16) ? env_wpg : 4;
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) k = pick_plain<bf16_t, bf16_t>(nks, split, a->epi_act, wpg);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) k = pick_plain<bf16_t, float>(nks, split, a->epi_act, wpg);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) k = pick_plain<float, float>(nks, split, a->epi_act, wpg);
    else return STZS_EDTYPE;
    if (!k) return STZS_EINVAL;
    dim3 grid((unsigned)((a->Co + 16 * wpg - 1) / (16 * wpg)), (unsigned)(((long)a->B * a->T_in + LR_ROWS - 1) / LR_ROWS),
              (unsigned)Z);
    hipLaunchKernelGGL(reinterpret_cast<void (*)(stzs_conv_args)>(k), grid, dim3(64 * wpg), 0, s, *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_ln_linear(const stzs_conv_args* a, const stzs_rowln_args* ln, void* stream) {
    if (!a || !a->w || !a->y) return STZS_EINVAL;
    if (!ln) return plain_launch(a, reinterpret_cast<hipStream_t>(stream));
    if (!ln->x) return STZS_EINVAL;
    const bool lin = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->T_in == a->T_out &&
                     a->pro_mode == STZS_PRO_NONE && a->pro_act == STZS_ACT_NONE && !a->stat_part && !a->x_scale &&
                     !a->res && !a->gate && a->splitk <= 1;
    if (!lin || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_W_X3 |
                             STZS_CONV_W_FRAG32 | STZS_CONV_UPS_NOISE)))
        return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->Co <= 0 || a->Co > a->co_pad || a->co_pad % 128) return STZS_ESHAPE;
    // the linear's K is the LayerNorm's row: C = Ci = ci_pad, 4 / 8 / 16 K-steps
    const int C = ln->C, nk = C / 32;
    if (C != a->Ci || C != a->ci_pad || C % 32 || (nk != 4 && nk != 8 && nk != 16)) return STZS_ESHAPE;
    if ((long)ln->R != (long)a->B * a->T_in || ln->R >= (1 << 22) - LR_ROWS || ln->ldx % 8 || ln->gdiv <= 0 ||
        !stzs_aligned(ln->x, 16))
        return STZS_ESHAPE;
    if ((ln->G && (ln->gs % 8 || !stzs_aligned(ln->G, 32))) || (ln->Bt && (ln->bs % 8 || !stzs_aligned(ln->Bt, 32))))
        return STZS_ESHAPE;
    if (ln->out_dtype != STZS_BF16) return STZS_EDTYPE;  // the linear's operand is the LayerNorm's bf16 rounding
    if (ln->act != STZS_ACT_NONE) return STZS_EINVAL;      // (the denoiser's LayerNorms: no activation)
    void* k = nullptr;
    if (ln->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) k = pick<float, bf16_t>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) k = pick<float, float>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) k = pick<bf16_t, bf16_t>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) k = pick<bf16_t, float>(nk, a->epi_act);
    else return STZS_EDTYPE;
    if (!k) return STZS_EINVAL;  // an epilogue activation this form does not instantiate
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((unsigned)((a->Co + 63) / 64), (unsigned)((ln->R + LR_ROWS - 1) / LR_ROWS));
    hipLaunchKernelGGL(reinterpret_cast<void (*)(stzs_conv_args, stzs_rowln_args)>(k), grid, dim3(NTHR), 0, s, *a, *ln);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
