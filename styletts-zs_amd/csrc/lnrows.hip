// LayerNorm-fed small-M linear in ONE launch: y = epilogue(LN(x) W^T) (the configs[1] batch-1 denoiser, SURVEY.md
// §8(a) a2: every adaLN / affine LayerNorm of a DiT layer feeds exactly one linear -- qkv, the cross-attention query,
// ffn1, the output projection).  At 200 rows stzs_row_layernorm + the rows GEMM were two launches (~4.8 + ~8 us,
// profiles/r04_j_lat_trace.txt: 196 LayerNorm launches of the 913 per batch-1 synthesis).
//
// A workgroup owns 64 rows and 64 output columns (4 waves x one 16-column tile):
//   * at entry every wave puts the first (up to 16) K-steps of its weight tile in flight (one 16-B load per lane per
//     K-step of the STZS_PACK_KSTEP stream, as csrc/rows.hip reads it) and the modulation vectors of its rows' groups;
//   * each wave normalises 16 of the 64 rows with stzs_row_layernorm's own row arithmetic (csrc/rowln.hpp: two-pass
//     statistics, (gadd + G) x_hat + Bt, activation, bf16 RNE) into an LDS operand image [64 rows][K] bf16 (16-B row
//     skew: conflict-free fragment reads) -- the values the unfused LayerNorm would have stored;
//   * one barrier, then each wave runs its 16 columns x 64 rows over all of K: A fragments from LDS, B from registers,
//     v_mfma_f32_16x16x32_bf16 in one sequential chain per output element (K order only: batch-invariant);
//   * epilogue as the rows GEMM: bias, NONE | GELU | SILU, alpha, beta * acc_in.
// The LayerNorm is recomputed by every column group (ceil(Co / 64) of them) from L2-resident rows: 128 KB per
// workgroup instead of a launch, a global round trip of the normalised rows and the rows GEMM's fixed cost.
#include "conv_common.hpp"
#include "rowln.hpp"

namespace {

constexpr int LR_ROWS = 64;  // rows per workgroup (4 waves x 16)

template <typename TI, typename TOut, int MAXV, int NK, int EACT>
__global__ __launch_bounds__(NTHR) void ln_rows(const stzs_conv_args a, const stzs_rowln_args ln) {
    extern __shared__ __attribute__((aligned(16))) unsigned char lds[];
    constexpr int K = NK * 32;
    constexpr int PITCH = K * 2 + 16;              // bytes per LDS row
    constexpr int BR = NK < 16 ? NK : 16;          // K-steps of weights in flight per wave
    constexpr int RBAT = 8;                        // rows whose loads are in flight together
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int nR = ln.R;
    const int r0 = blockIdx.y * LR_ROWS;
    // ---- this wave's weight tile: the first BR K-steps in flight from the start ----
    const int ct = blockIdx.x * 4 + wave;
    const bool wact = ct * 16 < a.Co;  // (wave-uniform)
    const int ctc = wact ? ct : 0;
    const int cot = ctc >> 3, rr = (ctc & 7) * 16 + (lane & 15);
    const unsigned char* Wb = reinterpret_cast<const unsigned char*>(a.w) + ((int64_t)cot * NK * 128 + rr) * 64 +
                              (((lane >> 4) ^ gswz(rr)) << 4);
    uint4 br[BR];
#pragma unroll
    for (int j = 0; j < BR; ++j) br[j] = *reinterpret_cast<const uint4*>(Wb + (int64_t)j * 128 * 64);
    // ---- LayerNorm of the wave's 16 rows into the LDS operand image ----
    const int rw = r0 + wave * 16;
    const int rl = rw + 15 < nR ? rw + 15 : nR - 1;
    const bool onegrp = ln.gs == 0 && ln.bs == 0;  // (an affine LayerNorm: every row reads the same vectors)
    auto group = [&](int r) { return onegrp ? 0 : r / ln.gdiv; };
    const int g0 = group(rw < nR ? rw : nR - 1), g1 = group(rl);
    float mg[2][MAXV][8], mb[2][MAXV][8];
    stzs_ln::ln_mod_load<MAXV>(ln, g0, lane, mg[0], mb[0]);
    stzs_ln::ln_mod_load<MAXV>(ln, g1, lane, mg[1], mb[1]);
    const int nv = ln.C >> 3;
#pragma unroll
    for (int b0 = 0; b0 < 16; b0 += RBAT) {
        float v[RBAT][MAXV][8];
#pragma unroll
        for (int i = 0; i < RBAT; ++i) {
            const int r = rw + b0 + i < nR ? rw + b0 + i : nR - 1;
            const TI* X = reinterpret_cast<const TI*>(ln.x) + (int64_t)r * ln.ldx;
#pragma unroll
            for (int m = 0; m < MAXV; ++m)
                if (lane + m * 64 < nv) load8(X + (lane + m * 64) * 8, v[i][m]);
        }
#pragma unroll
        for (int i = 0; i < RBAT; ++i) {
            float mu, rstd;
            stzs_ln::ln_row_stats<MAXV>(ln, lane, v[i], mu, rstd);
            const int r = rw + b0 + i < nR ? rw + b0 + i : nR - 1;
            const int gi = group(r);
            float gs[MAXV][8], bs[MAXV][8];
#pragma unroll
            for (int m = 0; m < MAXV; ++m)
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    gs[m][j] = gi == g0 ? mg[0][m][j] : mg[1][m][j];
                    bs[m][j] = gi == g0 ? mb[0][m][j] : mb[1][m][j];
                }
            if (gi != g0 && gi != g1) stzs_ln::ln_mod_load<MAXV>(ln, gi, lane, gs, bs);  // (groups < 16 rows)
            unsigned char* dst = lds + (wave * 16 + b0 + i) * PITCH;
            stzs_ln::ln_row_out<MAXV>(ln, lane, v[i], mu, rstd, gs, bs, [&](int, int vi, const float* o) {
                *reinterpret_cast<uint4*>(dst + vi * 16) = pack8(o);
            });
        }
    }
    __syncthreads();
    if (!wact) return;
    // ---- 64 rows x 16 columns over all of K ----
    f32x4 acc[4];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) acc[mt] = f32x4{0.f, 0.f, 0.f, 0.f};
    const unsigned char* A0 = lds + (lane & 15) * PITCH + (lane >> 4) * 16;
#pragma unroll
    for (int j = 0; j < NK; ++j) {
        const bf16x8 fb = __builtin_bit_cast(bf16x8, br[j % BR]);
        if (j + BR < NK) br[j % BR] = *reinterpret_cast<const uint4*>(Wb + (int64_t)(j + BR) * 128 * 64);
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            const bf16x8 fa = *reinterpret_cast<const bf16x8*>(A0 + mt * 16 * PITCH + j * 64);
            acc[mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fa, fb, acc[mt], 0, 0, 0);
        }
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
    for (int mt = 0; mt < 4; ++mt)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const int R = r0 + mt * 16 + (lane >> 4) * 4 + i;
            if (R >= nR) continue;
            float x = epi_act<EACT>(acc[mt][i] + bias, a.epi_slope);
            x *= a.alpha;
            const long bb = rowdiv(R, T, invT, true);
            const long t = R - bb * T;
            if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + t * a.lda + n);
            DT<TOut>::st(Y + bb * a.bsy + t * a.ldy + n, x);
        }
}

template <typename TI, typename TOut, int MAXV, int NK>
void* pick_act(int act) {
    switch (act) {
        case STZS_ACT_GELU: return (void*)ln_rows<TI, TOut, MAXV, NK, STZS_ACT_GELU>;
        case STZS_ACT_SILU: return (void*)ln_rows<TI, TOut, MAXV, NK, STZS_ACT_SILU>;
        case STZS_ACT_NONE: return (void*)ln_rows<TI, TOut, MAXV, NK, STZS_ACT_NONE>;
        default: return nullptr;
    }
}

template <typename TI, typename TOut>
void* pick(int nk, int act) {
    switch (nk) {
        case 4: return pick_act<TI, TOut, 1, 4>(act);
        case 8: return pick_act<TI, TOut, 1, 8>(act);
        case 16: return pick_act<TI, TOut, 1, 16>(act);
        case 32: return pick_act<TI, TOut, 2, 32>(act);
        default: return nullptr;
    }
}

}  // namespace

extern "C" int stzs_ln_linear(const stzs_conv_args* a, const stzs_rowln_args* ln, void* stream) {
    if (!a || !ln || !a->w || !a->y || !ln->x) return STZS_EINVAL;
    const bool lin = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->T_in == a->T_out &&
                     a->pro_mode == STZS_PRO_NONE && a->pro_act == STZS_ACT_NONE && !a->stat_part && !a->x_scale &&
                     !a->res && !a->gate && a->splitk <= 1;
    if (!lin || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_W_X3 |
                             STZS_CONV_W_FRAG32 | STZS_CONV_UPS_NOISE)))
        return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->Co <= 0 || a->Co > a->co_pad || a->co_pad % 128) return STZS_ESHAPE;
    // the linear's K is the LayerNorm's row: C = Ci = ci_pad, 4 / 8 / 16 / 32 K-steps
    const int C = ln->C, nk = C / 32;
    if (C != a->Ci || C != a->ci_pad || C % 32 || (nk != 4 && nk != 8 && nk != 16 && nk != 32)) return STZS_ESHAPE;
    if ((long)ln->R != (long)a->B * a->T_in || ln->R >= (1 << 22) - LR_ROWS || ln->ldx % 8 || ln->gdiv <= 0)
        return STZS_ESHAPE;
    if ((ln->G && (ln->gs % 8 || !stzs_aligned(ln->G, 32))) || (ln->Bt && (ln->bs % 8 || !stzs_aligned(ln->Bt, 32))))
        return STZS_ESHAPE;
    if (ln->out_dtype != STZS_BF16) return STZS_EDTYPE;  // the linear's operand is the LayerNorm's bf16 rounding
    void* k = nullptr;
    if (ln->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) k = pick<float, bf16_t>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) k = pick<float, float>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) k = pick<bf16_t, bf16_t>(nk, a->epi_act);
    else if (ln->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) k = pick<bf16_t, float>(nk, a->epi_act);
    else return STZS_EDTYPE;
    if (!k) return STZS_EINVAL;  // an epilogue activation this form does not instantiate
    const size_t lds = (size_t)LR_ROWS * (C * 2 + 16);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 grid((unsigned)((a->Co + 63) / 64), (unsigned)((ln->R + LR_ROWS - 1) / LR_ROWS));
    (void)hipFuncSetAttribute(k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(reinterpret_cast<void (*)(stzs_conv_args, stzs_rowln_args)>(k), grid, dim3(NTHR), lds, s, *a, *ln);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
