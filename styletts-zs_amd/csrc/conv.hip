// The universal MFMA conv1d / linear of the hot path.
//
// Implicit GEMM on gfx950 matrix cores: M = output time rows, N = output channels,
// K = taps x input channels.  One 256-thread workgroup (4 waves, 2x2) owns a BT x BCO output
// tile; each wave a (BT/2) x (BCO/2) sub-tile of 16x16 accumulators fed by
// v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32 accumulate).
//
// Per input-channel chunk (cic = 32|64 channels):
//   1. the input rows of the tile INCLUDING the dilation halo are staged ONCE into LDS
//      (channels-last rows, 16-B padded pitch), with the AdaIN / cscale prologue and the
//      activation (LeakyReLU / Snake) applied on the way in -> no separate norm/activation pass;
//   2. the taps re-read that LDS tile at row offset tap*dil (the halo is never re-fetched);
//   3. per-tap weight tiles [BCO][cic] are double-buffered in LDS with register prefetch of the
//      next tap issued before the MFMAs of the current one (T14 split: issue early, write late).
// The epilogue fuses bias, activation, DiT gate, residual (optionally read at t/res_tdiv, i.e.
// a nearest-x2 shortcut), scaling and an fp32/bf16 accumulate-input (MRF sum, EDM c_skip*x),
// and the polyphase ConvTranspose1d scatter (+ ReflectionPad(1,0)) when `ups` > 0.
#include "common.hpp"

namespace {

constexpr int NTHR = 256;

template <typename TIn, typename TOut, int BT, int BCO, bool FLAT>
__global__ __launch_bounds__(NTHR) void conv_mfma(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int WT = BT / 2, WC = BCO / 2, MT = WT / 16, NT = WC / 16;
    constexpr int WV_MAX = BCO * 8 / NTHR;  // 16-B weight vectors per thread at cic = 64
    const int cic = a.cic;
    const int lrow = cic + 8;
    const int ks = FLAT ? 1 : a.ks;
    const int rows_in = FLAT ? BT : (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    bf16_t* in_lds = reinterpret_cast<bf16_t*>(smem);
    bf16_t* w_lds = in_lds + rows_in * lrow;
    float* c_sc = reinterpret_cast<float*>(w_lds + 2 * BCO * lrow);
    float* c_sh = c_sc + 64;
    float* c_al = c_sh + 64;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    const int n0 = blockIdx.y * BCO;
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)blockIdx.x * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = blockIdx.x / tpb;
        t0 = (blockIdx.x - bq * tpb) * BT;
    }

    f32x4 acc[MT][NT];
#pragma unroll
    for (int i = 0; i < MT; ++i)
#pragma unroll
        for (int j = 0; j < NT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const TIn* X = reinterpret_cast<const TIn*>(a.x);
    const bf16_t* W = reinterpret_cast<const bf16_t*>(a.w);
    const int nchunk = a.ci_pad / cic;
    const int vpr = cic >> 3;
    const int wvec = BCO * vpr;
    uint4 wreg[WV_MAX];

    auto load_w = [&](int tap, int cc) {
#pragma unroll
        for (int i = 0; i < WV_MAX; ++i) {
            const int v = tid + i * NTHR;
            if (v < wvec) {
                const int r = v / vpr, cv = v - r * vpr;
                wreg[i] = *reinterpret_cast<const uint4*>(
                    W + ((long)tap * a.co_pad + n0 + r) * a.ci_pad + cc * cic + cv * 8);
            }
        }
    };
    auto store_w = [&](int buf) {
        bf16_t* dst = w_lds + buf * BCO * lrow;
#pragma unroll
        for (int i = 0; i < WV_MAX; ++i) {
            const int v = tid + i * NTHR;
            if (v < wvec) {
                const int r = v / vpr, cv = v - r * vpr;
                *reinterpret_cast<uint4*>(dst + r * lrow + cv * 8) = wreg[i];
            }
        }
    };

    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();
        if (tid < cic) {
            const int ci = cc * cic + tid;
            float sc = 0.f, sh = 0.f, al = 1.f;
            if (ci < a.Ci) {
                if (a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = a.pro_mean[(long)bq * a.stat_bs + ci];
                    const float rs = a.pro_rstd[(long)bq * a.stat_bs + ci];
                    const float g = a.pro_gb[(long)bq * a.gb_bs + ci];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + ci];
                    sc = (1.f + g) * rs;
                    sh = be - mu * sc;
                } else {
                    sc = a.pro_cscale;
                }
                if (a.pro_alpha) al = a.pro_alpha[ci];
            }
            c_sc[tid] = sc;
            c_sh[tid] = sh;
            c_al[tid] = al;
        }
        load_w(0, cc);
        __syncthreads();
        const int nv = rows_in * vpr;
        for (int v = tid; v < nv; v += NTHR) {
            const int r = v / vpr, cv = v - r * vpr;
            const int ci = cc * cic + cv * 8;
            float f[8];
            bool ok;
            const TIn* src;
            if (FLAT) {
                const long R = row0 + r;
                ok = R < (long)a.B * a.T_in;
                const long bb = R / a.T_in;
                const long tt = R - bb * a.T_in;
                src = X + bb * a.bsx + tt * a.ldx + ci;
            } else {
                const int tin = t0 * a.stride - a.pad + r;
                ok = tin >= 0 && tin < a.T_in;
                src = X + (long)bq * a.bsx + (long)tin * a.ldx + ci;
            }
            ok = ok && (ci < a.Ci);
            if (ok) {
                load8(src, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float y = f[j] * c_sc[cv * 8 + j] + c_sh[cv * 8 + j];
                    f[j] = act_apply(a.pro_act, y, a.pro_slope, c_al[cv * 8 + j]);
                }
            } else {
#pragma unroll
                for (int j = 0; j < 8; ++j) f[j] = 0.f;
            }
            *reinterpret_cast<uint4*>(in_lds + r * lrow + cv * 8) = pack8(f);
        }
        store_w(0);
        __syncthreads();
        for (int tap = 0; tap < ks; ++tap) {
            const int buf = tap & 1;
            if (tap + 1 < ks) load_w(tap + 1, cc);
            const bf16_t* wl = w_lds + buf * BCO * lrow;
            const int roff = FLAT ? 0 : tap * a.dil;
            const int rstr = FLAT ? 1 : a.stride;
            for (int kk = 0; kk < cic; kk += 32) {
                const int kc = kk + 8 * (lane >> 4);
                bf16x8 af[MT], bw[NT];
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const int r = (wt * WT + mt * 16 + (lane & 15)) * rstr + roff;
                    af[mt] = *reinterpret_cast<const bf16x8*>(in_lds + r * lrow + kc);
                }
#pragma unroll
                for (int nt = 0; nt < NT; ++nt) {
                    const int c = wc * WC + nt * 16 + (lane & 15);
                    bw[nt] = *reinterpret_cast<const bf16x8*>(wl + c * lrow + kc);
                }
#pragma unroll
                for (int mt = 0; mt < MT; ++mt)
#pragma unroll
                    for (int nt = 0; nt < NT; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
            }
            if (tap + 1 < ks) store_w(buf ^ 1);
            __syncthreads();
        }
    }

    // ---- epilogue ----
    const TOut* Rp = reinterpret_cast<const TOut*>(a.res);
    const TOut* AI = reinterpret_cast<const TOut*>(a.acc_in);
    TOut* Y = reinterpret_cast<TOut*>(a.y);
    const int ncol = a.ups > 0 ? a.ups * a.Co : a.Co;
    const long nrows_flat = (long)a.B * a.T_out;
#pragma unroll
    for (int mt = 0; mt < MT; ++mt)
#pragma unroll
        for (int nt = 0; nt < NT; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r) {
                const int tl = wt * WT + mt * 16 + (lane >> 4) * 4 + r;
                const int n = n0 + wc * WC + nt * 16 + (lane & 15);
                if (n >= ncol) continue;
                long bb, t;
                if (FLAT) {
                    const long Rr = row0 + tl;
                    if (Rr >= nrows_flat) continue;
                    bb = Rr / a.T_out;
                    t = Rr - bb * a.T_out;
                } else {
                    bb = bq;
                    t = t0 + tl;
                    if (t >= a.T_out) continue;
                }
                int co = n;
                if (a.ups > 0) {
                    const int p = n / a.Co;
                    co = n - p * a.Co;
                    t = t * a.ups + p - a.ups_pad;
                    if (t < 0 || t >= a.T_final) continue;
                    t += a.refl;
                }
                float u = acc[mt][nt][r];
                if (a.bias) u += a.bias[co];
                u = act_apply(a.epi_act, u, a.epi_slope, 1.f);
                if (a.gate) u *= a.gate[bb * a.gate_bs + co];
                const int ntgt = (a.ups > 0 && a.refl && t == 2) ? 2 : 1;
                for (int q = 0; q < ntgt; ++q) {
                    const long tt = q == 0 ? t : 0;
                    float v = u;
                    if (Rp) v += DT<TOut>::ld(Rp + bb * a.bsr + (tt / a.res_tdiv) * a.ldr + co);
                    v *= a.alpha;
                    if (AI) v += a.beta * DT<TOut>::ld(AI + bb * a.bsa + tt * a.lda + co);
                    DT<TOut>::st(Y + bb * a.bsy + tt * a.ldy + co, v);
                }
            }
}

size_t lds_bytes(int BT, int BCO, int rows_in, int cic) {
    const int lrow = cic + 8;
    return (size_t)rows_in * lrow * 2 + (size_t)2 * BCO * lrow * 2 + 3 * 64 * 4;
}

template <typename TIn, typename TOut, int BT, int BCO>
int launch_cfg(const stzs_conv_args& a, hipStream_t s, bool flat) {
    const int rows_in = flat ? BT : (BT - 1) * a.stride + (a.ks - 1) * a.dil + 1;
    const size_t lds = lds_bytes(BT, BCO, rows_in, a.cic);
    if (lds > 160 * 1024) return STZS_ESHAPE;
    unsigned gx = flat ? (unsigned)(((long)a.B * a.T_out + BT - 1) / BT)
                       : (unsigned)a.B * (unsigned)((a.T_out + BT - 1) / BT);
    dim3 grid(gx, a.co_pad / BCO);
    if (flat) {
        auto k = conv_mfma<TIn, TOut, BT, BCO, true>;
        if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, a);
    } else {
        auto k = conv_mfma<TIn, TOut, BT, BCO, false>;
        if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, a);
    }
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

template <typename TIn, typename TOut>
int launch_dt(const stzs_conv_args& a, hipStream_t s) {
    const bool flat = (a.ks == 1 && a.stride == 1 && a.pad == 0 && a.ups == 0 && a.pro_mode == STZS_PRO_NONE &&
                       a.T_in == a.T_out);
    const int BCO = (a.co_pad % 128 == 0) ? 128 : 64;
    int BT = 128;
    if (!flat) {
        const int rows128 = 127 * a.stride + (a.ks - 1) * a.dil + 1;
        if (a.T_out <= 64 || lds_bytes(128, BCO, rows128, a.cic) > 64 * 1024) BT = 64;
    } else if ((long)a.B * a.T_out <= 64) {
        BT = 64;
    }
    if (BT == 128 && BCO == 128) return launch_cfg<TIn, TOut, 128, 128>(a, s, flat);
    if (BT == 128 && BCO == 64) return launch_cfg<TIn, TOut, 128, 64>(a, s, flat);
    if (BT == 64 && BCO == 128) return launch_cfg<TIn, TOut, 64, 128>(a, s, flat);
    return launch_cfg<TIn, TOut, 64, 64>(a, s, flat);
}

}  // namespace

extern "C" int stzs_conv1d(const stzs_conv_args* a, void* stream) {
    if (!a || !a->x || !a->w || !a->y) return STZS_EINVAL;
    if (a->cic != 32 && a->cic != 64) return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0 || a->ks <= 0 || a->dil <= 0 ||
        a->stride <= 0)
        return STZS_ESHAPE;
    if (a->ci_pad % a->cic || a->ci_pad < a->Ci || a->co_pad % 64) return STZS_ESHAPE;
    const int ncol = a->ups > 0 ? a->ups * a->Co : a->Co;
    if (a->co_pad < ncol) return STZS_ESHAPE;
    if (a->ldx % 8 || a->bsx % 8 || a->ldx < ((a->Ci + 7) / 8) * 8) return STZS_ESHAPE;
    if (!stzs_aligned(a->x, 32) || !stzs_aligned(a->w, 16)) return STZS_EINVAL;
    if (a->ups > 0) {
        if (a->ks != 2 || a->pad != 1 || a->stride != 1 || a->dil != 1 || a->T_out != a->T_in + 1) return STZS_ESHAPE;
        if (a->refl && a->T_final < 2) return STZS_ESHAPE;
    } else if (a->refl) {
        return STZS_EINVAL;
    }
    if (a->res && a->res_tdiv <= 0) return STZS_EINVAL;
    if (a->pro_mode == STZS_PRO_ADAIN && (!a->pro_mean || !a->pro_rstd || !a->pro_gb)) return STZS_EINVAL;
    if (a->pro_act == STZS_ACT_SNAKE && !a->pro_alpha) return STZS_EINVAL;
    // the output row range the kernel may address must be non-negative and consistent
    const long t_last = a->ups > 0 ? (long)a->T_final + a->refl : a->T_out;
    if (t_last <= 0) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) return launch_dt<bf16_t, bf16_t>(*a, s);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) return launch_dt<bf16_t, float>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) return launch_dt<float, bf16_t>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) return launch_dt<float, float>(*a, s);
    return STZS_EDTYPE;
}
