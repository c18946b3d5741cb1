// The universal MFMA conv1d / linear of the hot path.
//
// Implicit GEMM on gfx950 matrix cores: M = output time rows, N = output channels, K = taps x
// input channels.  One 256-thread workgroup (4 waves as 2x2) owns a 128 x 128 output tile; each
// wave a 64 x 64 sub-tile = 4 x 4 accumulators of v_mfma_f32_16x16x32_bf16 (bf16 operands, fp32
// accumulate).  Two workgroups fit per CU (<= 80 KB LDS each), so one's staging/epilogue VALU
// overlaps the other's MFMAs.
//
//  * INPUT: per input-channel chunk (cic = 32|64|128) the tile's rows INCLUDING the dilation halo
//    are staged ONCE into LDS through registers, with the AdaIN/cscale prologue and the
//    activation (LeakyReLU / Snake with the hardware v_sin) applied on the way in.  Rows use a
//    16-B padded pitch (conflict-light ds_read_b128 for the A fragments).  Every tap re-reads that
//    tile at row offset tap*dil: the halo is fetched once, no separate norm/activation pass exists.
//  * WEIGHTS: pre-packed per 128-column tile as a stream of K-steps, each [128 co][32 ci] bf16 =
//    8 KB, already XOR-swizzled into the LDS image order (stzs/weights.py) so that a lane-linear
//    LDS-DMA copy (global_load_lds_dwordx4, 1 KB per wave instruction) lands a conflict-free
//    B-fragment layout.  A 3-slot ring keeps two K-steps in flight: counted s_waitcnt vmcnt + one
//    raw s_barrier per K-step, never a vmcnt(0) drain inside the K loop.
//  * EPILOGUE: accumulators go through LDS (fp32, padded rows) and leave as 16-B vectors per lane:
//    bias, activation, DiT gate, residual (optionally at t/res_tdiv = nearest-x2 shortcut), scale,
//    fp32/bf16 accumulate-input (MRF sum, EDM c_skip*x), the polyphase ConvTranspose1d scatter and
//    ReflectionPad(1,0) when ups > 0.
#include "common.hpp"

namespace {

constexpr int NTHR = 256;
constexpr int BT = 128, BCO = 128;
constexpr int NSLOT = 3;
constexpr int SLOT_BYTES = BCO * 32 * 2;  // one K-step of weights
constexpr int EP_PITCH = BCO + 4;         // fp32 epilogue row pitch (floats)

STZS_DEV int gswz(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }

// flat row R -> (utterance q, step R - q T) without a 64-bit integer division (hipcc expands `long / int` into a
// ~100-instruction routine: the FLAT epilogue ran one per output row vector, r04 gemm_phase).  For R < 2^22 the float
// quotient R (1 / T) is within one of R / T and one correction step makes it exact (as csrc/rows.hip); beyond, the
// plain division.  `small` must be uniform (nR < 2^22).
STZS_DEV long rowdiv(long R, int T, float invT, bool small) {
    if (small) {
        int q = (int)((float)(int)R * invT);
        const int r = (int)R - q * T;
        q += r < 0 ? -1 : (r >= T ? 1 : 0);
        return q;
    }
    return R / T;
}

template <int PACT>
STZS_DEV float pro_act(float x, float slope, float alpha, float ialpha) {
    if constexpr (PACT == STZS_ACT_SNAKE) {
        const float s = __sinf(alpha * x);  // v_sin_f32 (hardware, revolutions)
        return x + s * s * ialpha;
    } else if constexpr (PACT == STZS_ACT_LEAKY) {
        return x >= 0.f ? x : x * slope;
    } else {
        return x;
    }
}

template <typename T> struct Raw;
template <> struct Raw<bf16_t> {
    typedef uint4 T;
    static STZS_DEV uint4 load(const bf16_t* p) { return *reinterpret_cast<const uint4*>(p); }
    static STZS_DEV void cvt(const uint4& u, float* v) {
        const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            v[2 * i] = __uint_as_float(w[i] << 16);
            v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
        }
    }
};
struct F8 { float4 a, b; };
template <> struct Raw<float> {
    typedef F8 T;
    static STZS_DEV F8 load(const float* p) {
        return F8{*reinterpret_cast<const float4*>(p), *reinterpret_cast<const float4*>(p + 4)};
    }
    static STZS_DEV void cvt(const F8& u, float* v) {
        v[0] = u.a.x; v[1] = u.a.y; v[2] = u.a.z; v[3] = u.a.w;
        v[4] = u.b.x; v[5] = u.b.y; v[6] = u.b.z; v[7] = u.b.w;
    }
};

template <typename T> STZS_DEV void store8v(T* p, const float* v) { store8(p, v); }

STZS_DEV void waitcnt_vm(int n) {
    if (n >= 2)
        __builtin_amdgcn_s_waitcnt(0x0F70 | 2);
    else
        __builtin_amdgcn_s_waitcnt(0x0F70 | 0);
}

// Epilogue pass: each thread owns ONE 8-channel vector column (cv = tid & 15, so bias/gate sit in
// registers) and walks rows 16 apart; EB vectors per batch, residual / accumulate loads issued
// unconditionally from clamped addresses (all in flight) before any is consumed.
// erf by Abramowitz & Stegun 7.1.26 (|error| <= 1.5e-7; one v_exp + one v_rcp instead of libm erff)
STZS_DEV float fast_erf(float x) {
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

template <typename TOut, bool FLAT, bool VEC, bool HR, bool HA, int EACT, int BTM>
STZS_DEV void epilogue(const stzs_conv_args& a, const float* ep, const float* c_bias, const float* c_gate, int bq,
                       int t0, long row0, int tid, int by) {
    const TOut* Rp = reinterpret_cast<const TOut*>(a.res);
    const TOut* AI = reinterpret_cast<const TOut*>(a.acc_in);
    TOut* Y = reinterpret_cast<TOut*>(a.y);
    const int ncol = a.ups > 0 ? a.ups * a.Co : a.Co;
    const long nrows_flat = (long)a.B * a.T_out;
    const bool small_rows = nrows_flat + BTM < (1L << 22);
    const float invTo = 1.f / (float)a.T_out;
    const long t_hi = a.ups > 0 ? (long)a.T_final + a.refl - 1 : (long)a.T_out - 1;
    const int cv = tid & 15;
    const int n = by * BCO + cv * 8;
    const bool col_ok = n < ncol;
    int co = n, p = 0;
    if (a.ups > 0) {
        p = n / a.Co;
        co = n - p * a.Co;
    }
    const int cc = col_ok ? co : 0;
    float kb[8], kg[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) {
        kb[j] = c_bias[cv * 8 + j];
        kg[j] = c_gate[cv * 8 + j];
    }
    const bool stat = !FLAT && a.stat_part != nullptr;
    const bool gate_vec = (reinterpret_cast<uintptr_t>(a.gate) & 15) == 0 && a.gate_bs % 4 == 0;
    float st_s[8], st_q[8];
#pragma unroll
    for (int j = 0; j < 8; ++j) st_s[j] = st_q[j] = 0.f;
    constexpr int EB = 4;
    float* red = const_cast<float*>(c_gate) + BCO;  // [2 halves][4 waves][BCO][2] statistics partials
    // (sum, sumsq) per column over 64 valid rows: 4 lanes per wave share a column vector (xor 16, 32),
    // lanes < 16 park the wave's partial in LDS; the 4 waves are combined after the loop.
    auto stat_flush = [&](int half) {
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            st_s[j] += __shfl_xor(st_s[j], 16, 64);
            st_s[j] += __shfl_xor(st_s[j], 32, 64);
            st_q[j] += __shfl_xor(st_q[j], 16, 64);
            st_q[j] += __shfl_xor(st_q[j], 32, 64);
        }
        const int wv = tid >> 6;
        if ((tid & 63) < 16) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                red[((half * 4 + wv) * BCO + cv * 8 + j) * 2] = st_s[j];
                red[((half * 4 + wv) * BCO + cv * 8 + j) * 2 + 1] = st_q[j];
            }
        }
#pragma unroll
        for (int j = 0; j < 8; ++j) st_s[j] = st_q[j] = 0.f;
    };
    static_assert(BT * (BCO / 8) == 2 * EB * NTHR, "two epilogue passes = two 64-row halves");
    for (int v0 = 0; v0 < BTM * (BCO / 8); v0 += EB * NTHR) {
        long pb[EB], pt[EB];
        bool pv[EB];
        float rr[EB][8], ai[EB][8], gvv[EB][8];
#pragma unroll
        for (int i = 0; i < EB; ++i) {
            const int tl = ((v0 + tid) >> 4) + i * (NTHR >> 4);
            bool ok = col_ok;
            long bb, t;
            if (FLAT) {
                const long Rr = row0 + tl;
                ok = ok && Rr < nrows_flat;
                bb = rowdiv(Rr, a.T_out, invTo, small_rows);
                t = Rr - bb * a.T_out;
            } else {
                bb = bq;
                t = t0 + tl;
                ok = ok && t < a.T_out;
            }
            if (a.ups > 0) {
                t = t * a.ups + p - a.ups_pad;
                ok = ok && t >= 0 && t < a.T_final;
                t += a.refl;
            }
            const long tc = t < 0 ? 0 : (t > t_hi ? t_hi : t);
            const long bc = bb < a.B ? bb : a.B - 1;
            pb[i] = bb;
            pt[i] = t;
            pv[i] = ok;
            if constexpr (VEC) {
                // (res_tdiv 1 but for the upsampling AdaIN blocks: a uniform test instead of a 64-bit division per row)
                const long tr = a.res_tdiv == 1 ? tc : (long)((int)tc / a.res_tdiv);
                if constexpr (HR) load8(Rp + bc * a.bsr + tr * a.ldr + cc, rr[i]);
                if constexpr (HA) load8(AI + bc * a.bsa + tc * a.lda + cc, ai[i]);
            }
            if (FLAT && a.gate) {  // DiT gate of this row's utterance, in flight with the residual rows
                const float* gp = a.gate + bc * a.gate_bs;
                if (gate_vec && co + 8 <= a.Co) {
                    load8(gp + co, gvv[i]);
                } else {
#pragma unroll
                    for (int j = 0; j < 8; ++j) gvv[i][j] = gp[min(co + j, a.Co - 1)];
                }
            }
        }
#pragma unroll
        for (int i = 0; i < EB; ++i) {
            if (!pv[i]) continue;
            const int tl = ((v0 + tid) >> 4) + i * (NTHR >> 4);
            const long bb = pb[i], t = pt[i];
            float u[8];
            const float* er = ep + tl * EP_PITCH + cv * 8;
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                float x = epi_act<EACT>(er[j] + kb[j], a.epi_slope);
                if (FLAT) {
                    if (a.gate) x *= gvv[i][j];
                } else {
                    x *= kg[j];
                }
                u[j] = x;
            }
            if constexpr (VEC) {
                float o[8];
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    float x = u[j];
                    if constexpr (HR) x += rr[i][j];
                    x *= a.alpha;
                    if constexpr (HA) x += a.beta * ai[i][j];
                    o[j] = x;
                }
                if constexpr (sizeof(TOut) == 2) {
                    const uint4 pk = pack8(o);
                    *reinterpret_cast<uint4*>(Y + bb * a.bsy + t * a.ldy + co) = pk;
                    if (stat) {  // statistics of the value as stored (bf16-rounded)
                        const uint32_t w[4] = {pk.x, pk.y, pk.z, pk.w};
#pragma unroll
                        for (int j = 0; j < 4; ++j) {
                            const float lo = __uint_as_float(w[j] << 16), hi = __uint_as_float(w[j] & 0xFFFF0000u);
                            st_s[2 * j] += lo;
                            st_q[2 * j] = fmaf(lo, lo, st_q[2 * j]);
                            st_s[2 * j + 1] += hi;
                            st_q[2 * j + 1] = fmaf(hi, hi, st_q[2 * j + 1]);
                        }
                    }
                } else {
                    store8(Y + bb * a.bsy + t * a.ldy + co, o);
                    if (stat) {
#pragma unroll
                        for (int j = 0; j < 8; ++j) {
                            st_s[j] += o[j];
                            st_q[j] = fmaf(o[j], o[j], st_q[j]);
                        }
                    }
                }
            } else {
                for (int j = 0; j < 8 && co + j < a.Co; ++j) {
                    float x = u[j];
                    if (Rp) x += DT<TOut>::ld(Rp + bb * a.bsr + (t / a.res_tdiv) * a.ldr + co + j);
                    x *= a.alpha;
                    if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + t * a.lda + co + j);
                    DT<TOut>::st(Y + bb * a.bsy + t * a.ldy + co + j, x);
                }
            }
            if (a.ups > 0 && a.refl && t == 2) {  // ReflectionPad(1,0): row 0 mirrors source row 1
                for (int j = 0; j < 8 && co + j < a.Co; ++j) {
                    float x = u[j];
                    if (Rp) x += DT<TOut>::ld(Rp + bb * a.bsr + co + j);
                    x *= a.alpha;
                    if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + co + j);
                    DT<TOut>::st(Y + bb * a.bsy + co + j, x);
                }
            }
        }
        if (stat) stat_flush(v0 == 0 ? 0 : 1);
    }
    if (stat) {
        __syncthreads();
        // one deterministic fp32 partial per (utterance, 64-row chunk, channel)
        const int half = tid >> 7, cl = tid & (BCO - 1);
        const int c = by * BCO + cl;
        const int r0 = t0 + half * 64;
        if (c < a.Co && r0 < a.T_out) {
            float ss = 0.f, qq = 0.f;
#pragma unroll
            for (int w = 0; w < 4; ++w) {
                ss += red[((half * 4 + w) * BCO + cl) * 2];
                qq += red[((half * 4 + w) * BCO + cl) * 2 + 1];
            }
            const int nch = (a.T_out + 63) / 64;
            float* P = reinterpret_cast<float*>(a.stat_part);
            const long o = (((long)bq * nch + r0 / 64) * a.stat_ld + c) * 2;
            P[o] = ss;
            P[o + 1] = qq;
        }
    }
}

template <typename TOut, bool FLAT, bool VEC, bool HR, bool HA, int BTM>
STZS_DEV void epilogue_act(const stzs_conv_args& a, const float* ep, const float* c_bias, const float* c_gate, int bq,
                           int t0, long row0, int tid, int by) {
    switch (a.epi_act) {
        case STZS_ACT_GELU: epilogue<TOut, FLAT, VEC, HR, HA, STZS_ACT_GELU, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by); break;
        case STZS_ACT_SILU: epilogue<TOut, FLAT, VEC, HR, HA, STZS_ACT_SILU, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by); break;
        case STZS_ACT_LEAKY: epilogue<TOut, FLAT, VEC, HR, HA, STZS_ACT_LEAKY, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by); break;
        default: epilogue<TOut, FLAT, VEC, HR, HA, STZS_ACT_NONE, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by); break;
    }
}

template <int BTM>
STZS_DEV bool splitk_combine_rt(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int SK);
// EP: the epilogue variant compiled into the calling kernel.  -1: all of them behind runtime tests (the conv kernels);
// 0..15: ONE vectorised variant, HR = bit 0, HA = bit 1, activation index (ep_act) = bits 2-3 (the GEMM kernels:
// with all twenty variants inlined a gemm_glds instance was ~73 k instructions and its epilogue ran from a cold
// instruction cache)
template <typename TOut, bool FLAT, int BTM = BT, int EP = -1>
STZS_DEV void finish(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int bq, int t0, long row0,
                     int by);
constexpr int ep_act(int i) { return i == 0 ? STZS_ACT_NONE : (i == 1 ? STZS_ACT_GELU : (i == 2 ? STZS_ACT_SILU : STZS_ACT_LEAKY)); }
// the EP index of a launch (-1: no specialised variant)
inline int ep_index(const stzs_conv_args& a, bool vec) {
    if (!vec) return -1;
    const int ai = a.epi_act == STZS_ACT_NONE ? 0 : a.epi_act == STZS_ACT_GELU ? 1 : a.epi_act == STZS_ACT_SILU ? 2
                 : a.epi_act == STZS_ACT_LEAKY ? 3 : -1;
    if (ai < 0) return -1;
    return (a.res ? 1 : 0) | (a.acc_in ? 2 : 0) | (ai << 2);
}

// 8-wide vector epilogue legal (every output / residual / accumulate row 16-B aligned)
__host__ __device__ inline bool epi_vec(const stzs_conv_args& a) {
    return (a.Co % 8 == 0) && (a.ldy % 8 == 0) && (!a.res || a.ldr % 8 == 0) && (!a.acc_in || a.lda % 8 == 0) &&
           (a.bsy % 8 == 0) && (!a.res || a.bsr % 8 == 0) && (!a.acc_in || a.bsa % 8 == 0);
}

template <typename TIn, typename TOut, bool FLAT, int PACT>
__global__ __launch_bounds__(NTHR, 2) void conv_mfma(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int cic = a.cic;
    const int pitch = cic * 2 + 16;
    const int ks = FLAT ? 1 : a.ks;
    const int rows_in = FLAT ? BT : (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    unsigned char* in_lds = smem;
    unsigned char* ring = smem + ((rows_in * pitch + 15) & ~15);
    float* c_sc = reinterpret_cast<float*>(ring + NSLOT * SLOT_BYTES);
    float* c_sh = c_sc + 128;
    float* c_al = c_sh + 128;
    float* c_ia = c_al + 128;

    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    // XCD-aware tile order (as gemm_glds): each XCD runs a contiguous range of tiles, output-channel tile fastest,
    // so the workgroups one XCD holds at a time share their staged input rows (one fabric fetch per XCD instead
    // of one per channel tile).  Same tiles, same K order: bit-identical to the linear order.
    const int gy = gridDim.y;
    const bool lin_ids = (a.flags & STZS_CONV_LINEAR_IDS) != 0;
    const int lin = lin_ids ? 0 : xcd_remap(blockIdx.y * gridDim.x + blockIdx.x, gridDim.x * gy);
    const int by = lin_ids ? (int)blockIdx.y : lin % gy;
    const int bx = lin_ids ? (int)blockIdx.x : lin / gy;
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)bx * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = bx / tpb;
        t0 = (bx - bq * tpb) * BT;
    }
    const int nchunk = a.ci_pad / cic;
    const int kpc = cic >> 5;
    const int NK = nchunk * ks * kpc;
    const bf16_t* Wt = reinterpret_cast<const bf16_t*>(a.w) + (long)by * NK * (BCO * 32);
    // in-launch split-K over input-channel chunks (stzs_conv_args.splitk, grid.z slices): slice z stages and runs
    // chunks [cc_lo, cc_hi) -- K-steps [k_lo, k_hi) of the chunk-major weight stream -- and hands its fp32 partial
    // to the tile's last arriver (splitk_combine_rt), which runs the fused epilogue.  For the small grids of the
    // batch-1 front end (text-encoder k5 convs: 4 workgroups x 80 K-steps at batch 1).
    // Slice z takes chunks [z n / S, (z+1) n / S): equal slices when S divides n, otherwise sizes differing by one
    // (the decoder / predictor AdaIN convs of the batch-1 engine: 9 chunks in 3 or 4 slices)
    const int SKr = a.splitk > 1 ? a.splitk : 1;
    const int cc_lo = SKr > 1 ? (int)blockIdx.z * nchunk / SKr : 0;
    const int cc_hi = SKr > 1 ? ((int)blockIdx.z + 1) * nchunk / SKr : nchunk;
    const int k_lo = cc_lo * ks * kpc, k_hi = cc_hi * ks * kpc;

    auto fill = [&](int k) {
        const bf16_t* src = Wt + (long)k * (BCO * 32) + wave * 1024 + lane * 8;
        unsigned char* dst = ring + (k % NSLOT) * SLOT_BYTES + wave * 2048;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 512),
                                         (__attribute__((address_space(3))) void*)(dst + 1024), 16, 0, 0);
    };

    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const TIn* X = reinterpret_cast<const TIn*>(a.x);
    const int vpr = cic >> 3;
    const int rstr = FLAT ? 1 : a.stride;
    // B-fragment LDS byte offsets inside a slot (fixed per lane): row rr, chunk (lane>>4) swizzled
    int boff[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int rr = wc * 64 + nt * 16 + (lane & 15);
        boff[nt] = rr * 64 + (((lane >> 4) ^ gswz(rr)) << 4);
    }

    fill(k_lo);
    if (k_lo + 1 < k_hi) fill(k_lo + 1);
    int k = k_lo;
    for (int cc = cc_lo; cc < cc_hi; ++cc) {
        __syncthreads();
        const int nv = (a.flags & 1) ? 0 : rows_in * vpr;
        // Staging: ONE batch of SB independent 16-B loads per thread (every MRF tile fits), issued
        // BEFORE the per-chunk coefficient loads so both latencies overlap in the same wait.  Loads are
        // UNCONDITIONAL from clamped (always valid) addresses and masked afterwards (a runtime-
        // conditioned load makes hipcc drain vmcnt(0) per element).  vpr = cic/8 is a power of two
        // dividing NTHR, so a thread's channel vector cv is the same for every row it stages.
        constexpr int SB = sizeof(TIn) == 2 ? 12 : 4;
        using RawT = typename Raw<TIn>::T;
        const int lv = cic == 128 ? 4 : (cic == 64 ? 3 : 2);
        const int cv = tid & (vpr - 1);
        const int ci = cc * cic + cv * 8;
        const bool ci_ok = ci < a.Ci;
        const int cic0 = ci_ok ? ci : 0;
        const int rstep = NTHR >> lv;
        RawT raw[SB];
        bool okv[SB];
        const float invTi = 1.f / (float)a.T_in;  // (FLAT rows -> utterance, rowdiv)
        auto issue = [&](int v0) {
            const int rb = (v0 >> lv) + (tid >> lv);
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rb + i * rstep;
                bool ok = ci_ok && r < rows_in;
                long off;
                if (FLAT) {
                    long R = row0 + r;
                    const long nR = (long)a.B * a.T_in;
                    ok = ok && R < nR;
                    R = R < nR ? R : nR - 1;
                    const long bb = rowdiv(R, a.T_in, invTi, nR < (1L << 22));
                    off = bb * a.bsx + (R - bb * a.T_in) * a.ldx + cic0;
                } else {
                    int tin = t0 * a.stride - a.pad + r;
                    ok = ok && tin >= 0 && tin < a.T_in;
                    tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                    off = (long)bq * a.bsx + (long)tin * a.ldx + cic0;
                }
                okv[i] = ok;
                raw[i] = Raw<TIn>::load(X + off);
            }
        };
        if (nv > 0) issue(0);
        if (tid < cic) {
            const int cg = cc * cic + tid;
            float sc = 0.f, sh = 0.f, al = 1.f;
            if (cg < a.Ci) {
                if (a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = a.pro_mean[(long)bq * a.stat_bs + cg];
                    const float rs = a.pro_rstd[(long)bq * a.stat_bs + cg];
                    const float g = a.pro_gb[(long)bq * a.gb_bs + cg];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + cg];
                    sc = (1.f + g) * rs;
                    sh = be - mu * sc;
                } else {
                    sc = a.pro_cscale;
                }
                if (a.pro_alpha) al = a.pro_alpha[cg];
            }
            c_sc[tid] = sc;
            c_sh[tid] = sh;
            c_al[tid] = al;
            c_ia[tid] = 1.f / al;
        }
        __syncthreads();
        float k_sc[8], k_sh[8], k_al[8], k_ia[8];
#pragma unroll
        for (int j = 0; j < 8; ++j) {
            k_sc[j] = c_sc[cv * 8 + j];
            k_sh[j] = c_sh[cv * 8 + j];
            k_al[j] = c_al[cv * 8 + j];
            k_ia[j] = c_ia[cv * 8 + j];
        }
        for (int v0 = 0; v0 < nv; v0 += SB * NTHR) {
            if (v0 > 0) issue(v0);
            const int rb = (v0 >> lv) + (tid >> lv);
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rb + i * rstep;
                if (r >= rows_in) break;
                float f[8], o[8];
                Raw<TIn>::cvt(raw[i], f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float y = pro_act<PACT>(f[j] * k_sc[j] + k_sh[j], a.pro_slope, k_al[j], k_ia[j]);
                    o[j] = okv[i] ? y : 0.f;
                }
                *reinterpret_cast<uint4*>(in_lds + r * pitch + cv * 16) = pack8(o);
            }
        }
        __syncthreads();
        for (int tap = 0; tap < ((a.flags & 2) ? 0 : ks); ++tap) {
            const int roff = FLAT ? 0 : tap * a.dil;
            for (int kq = 0; kq < kpc; ++kq, ++k) {
                waitcnt_vm(k + 1 < k_hi ? 2 : 0);
                __builtin_amdgcn_s_barrier();
                if (k + 2 < k_hi) fill(k + 2);
                const unsigned char* wl = ring + (k % NSLOT) * SLOT_BYTES;
                const int kb = (kq * 32 + 8 * (lane >> 4)) * 2;
                bf16x8 af[4], bw[4];
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    const int r = (wt * 64 + mt * 16 + (lane & 15)) * rstr + roff;
                    af[mt] = *reinterpret_cast<const bf16x8*>(in_lds + r * pitch + kb);
                }
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) bw[nt] = *reinterpret_cast<const bf16x8*>(wl + boff[nt]);
                __builtin_amdgcn_sched_barrier(0);  // issue all 8 fragment reads before the first MFMA
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[mt], bw[nt], acc[mt][nt], 0, 0, 0);
            }
        }
    }

    if (SKr > 1 && !splitk_combine_rt<BT>(a, acc, smem, SKr)) return;
    finish<TOut, FLAT>(a, acc, smem, bq, t0, row0, by);
}

// Accumulators -> LDS (fp32, padded rows) -> vectorised fused epilogue.
// STZS_GEMM_PROF probe build: the epilogue's own stamps (slots 5: accumulators in LDS, 6: bias / gate constants in LDS)
#ifdef STZS_GEMM_PROF
#define GPROF_E(i)                                                                                            \
    if (FLAT && a.splitk <= 1 && a.splitk_ws && threadIdx.x == 0)                                              \
        reinterpret_cast<unsigned long long*>(a.splitk_ws)[(long)(blockIdx.y * gridDim.x + blockIdx.x) * 8 + (i)] = \
            __builtin_amdgcn_s_memtime();
#else
#define GPROF_E(i)
#endif
template <typename TOut, bool FLAT, int BTM, int EP>
STZS_DEV void finish(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int bq, int t0, long row0,
                     int by) {
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    __syncthreads();
    float* ep = reinterpret_cast<float*>(smem);
#pragma unroll
    for (int mt = 0; mt < BTM / 32; ++mt)
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int r = 0; r < 4; ++r)
                ep[(wt * (BTM / 2) + mt * 16 + (lane >> 4) * 4 + r) * EP_PITCH + wc * 64 + nt * 16 + (lane & 15)] = acc[mt][nt][r];
    if (a.flags & 4) return;
    GPROF_E(5)
    float* c_bias = ep + BT * EP_PITCH;       // [BCO] bias, [BCO] gate (conv mode: one utterance)
    float* c_gate = c_bias + BCO;
    if (tid < BCO) {
        const int n = by * BCO + tid;
        const int co = a.ups > 0 ? n % a.Co : min(n, a.Co - 1);
        c_bias[tid] = a.bias ? a.bias[co] : 0.f;
        c_gate[tid] = (!FLAT && a.gate) ? a.gate[(long)bq * a.gate_bs + co] : 1.f;
    }
    __syncthreads();
    GPROF_E(6)
    if constexpr (EP >= 0) {
        epilogue<TOut, FLAT, true, (EP & 1) != 0, (EP & 2) != 0, ep_act(EP >> 2), BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
    } else if (epi_vec(a)) {
        if (a.res && a.acc_in) epilogue_act<TOut, FLAT, true, true, true, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
        else if (a.res) epilogue_act<TOut, FLAT, true, true, false, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
        else if (a.acc_in) epilogue_act<TOut, FLAT, true, false, true, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
        else epilogue_act<TOut, FLAT, true, false, false, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
    } else {
        epilogue_act<TOut, FLAT, false, true, true, BTM>(a, ep, c_bias, c_gate, bq, t0, row0, tid, by);
    }
}

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
typedef __attribute__((ext_vector_type(2))) long i64x2;
// SK > 1 (stzs_conv_args.splitk, BTM = 64, bf16): workgroup z of a tile runs K-steps [z NK/SK, (z+1) NK/SK) and
// hands its fp32 partial to the tile's last arriver (splitk_combine), which then runs the epilogue.
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;
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
template <typename TOut, int BTM, bool F8, int SK = 1, int EP = -1>
__global__ __launch_bounds__(NTHR, 2) void gemm_glds(const stzs_conv_args a) {
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

// splitk_combine with the slice count at run time (conv_mfma): the same slabs, ticket and slice-order sum, the
// slices loaded one at a time (no [SK][NV] register block).
template <int BTM>
STZS_DEV bool splitk_combine_rt(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int SK) {
    constexpr int NV = BTM / 32 * 4;
    constexpr int SLAB = NV * NTHR * 16;
    const int tid = threadIdx.x;
    const long tile = blockIdx.x + (long)gridDim.x * blockIdx.y;
    unsigned char* base = reinterpret_cast<unsigned char*>(a.splitk_ws) + tile * (long)SK * SLAB;
    const __amdgpu_buffer_rsrc_t wr = __builtin_amdgcn_make_buffer_rsrc(base, 0, SK * SLAB, 0x00020000);
    const int z = blockIdx.z;
#pragma unroll
    for (int i = 0; i < NV; ++i)
        __builtin_amdgcn_raw_buffer_store_b128(__builtin_bit_cast(u32x4, acc[i >> 2][i & 3]), wr,
                                               (z * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    __syncthreads();
    volatile int* flag = reinterpret_cast<volatile int*>(smem);  // staging / ring idle: every wave is past its K loop
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
#pragma unroll
    for (int i = 0; i < NV; ++i)
        acc[i >> 2][i & 3] = __builtin_bit_cast(f32x4, __builtin_amdgcn_raw_buffer_load_b128(wr, i * (NTHR * 16) + tid * 16, 0, 16));
    for (int sl = 1; sl < SK; ++sl) {
        u32x4 v[NV];
#pragma unroll
        for (int i = 0; i < NV; ++i)
            v[i] = __builtin_amdgcn_raw_buffer_load_b128(wr, (sl * NV + i) * (NTHR * 16) + tid * 16, 0, 16);
#pragma unroll
        for (int i = 0; i < NV; ++i) acc[i >> 2][i & 3] += __builtin_bit_cast(f32x4, v[i]);
    }
    return true;
}

// PRECISE (parity) mode, STZS_CONV_W_F32: fp32 operands on v_mfma_f32_16x16x4_f32 (products exact in
// fp32, fp32 accumulate), libm-accurate prologue (act_apply).  Same 128 x 128 tile, 2 x 2 waves and
// accumulator layout as conv_mfma (the 16x16 C/D map is dtype-independent on gfx950), so the whole
// fused epilogue (finish) is shared.  Per 32-channel input chunk the tile rows (+ halo) are staged once
// in fp32; per tap one [128 co][32 ci] fp32 weight K-step goes through LDS.  The 16-B fragment reads keep
// conv_mfma's k geometry: lane l holds k = 8 (l >> 4) + j of its row/column, and MFMA j sums the four k
// values {8 h + j}; A and B use the same map, so the eight MFMAs of a K-step cover all 32 k exactly once.
// Not a performance path: it exists so the decoder can be run at fp32 accuracy against the oracle.
constexpr int P32 = 36;  // fp32 LDS row pitch (32 + 4 floats)
template <typename TIn, typename TOut>
__global__ __launch_bounds__(NTHR, 1) void conv_f32(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = a.ks;
    const int rows_in = (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    float* xin = reinterpret_cast<float*>(smem);
    float* wl = xin + rows_in * P32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int bq = blockIdx.x / tpb;
    const int t0 = (blockIdx.x - bq * tpb) * BT;
    const int nchunk = a.ci_pad / 32;
    const float* Wt = reinterpret_cast<const float*>(a.w) + (long)blockIdx.y * nchunk * ks * (BCO * 32);
    const TIn* X = reinterpret_cast<const TIn*>(a.x) + (long)bq * a.bsx;
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();
        for (int v = tid; v < rows_in * 4; v += NTHR) {
            const int r = v >> 2, cv = v & 3;
            const int ci = cc * 32 + cv * 8;
            const int tin = t0 * a.stride - a.pad + r;
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
            if (tin >= 0 && tin < a.T_in && ci < a.Ci) {
                float f[8];
                load8(X + (long)tin * a.ldx + ci, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const int c = ci + j;
                    if (c >= a.Ci) break;
                    float sc = a.pro_cscale, sh = 0.f;
                    if (a.pro_mode == STZS_PRO_ADAIN) {
                        const float mu = a.pro_mean[(long)bq * a.stat_bs + c];
                        const float rs = a.pro_rstd[(long)bq * a.stat_bs + c];
                        const float g = a.pro_gb[(long)bq * a.gb_bs + c];
                        const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + c];
                        sc = (1.f + g) * rs;
                        sh = be - mu * sc;
                    }
                    o[j] = act_apply(a.pro_act, f[j] * sc + sh, a.pro_slope, a.pro_alpha ? a.pro_alpha[c] : 1.f);
                }
            }
            float* d = xin + r * P32 + cv * 8;
            *reinterpret_cast<float4*>(d) = make_float4(o[0], o[1], o[2], o[3]);
            *reinterpret_cast<float4*>(d + 4) = make_float4(o[4], o[5], o[6], o[7]);
        }
        for (int tap = 0; tap < ks; ++tap) {
            __syncthreads();  // staged rows visible; previous weight K-step consumed
            const float* src = Wt + (long)(cc * ks + tap) * (BCO * 32);
            for (int e = tid * 4; e < BCO * 32; e += NTHR * 4)
                *reinterpret_cast<float4*>(wl + (e >> 5) * P32 + (e & 31)) = *reinterpret_cast<const float4*>(src + e);
            __syncthreads();
            const int kb = 8 * (lane >> 4);
            float av[4][8], bv[4][8];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const float* p = xin + ((wt * 64 + mt * 16 + (lane & 15)) * a.stride + tap * a.dil) * P32 + kb;
#pragma unroll
                for (int j = 0; j < 8; ++j) av[mt][j] = p[j];
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float* p = wl + (wc * 64 + nt * 16 + (lane & 15)) * P32 + kb;
#pragma unroll
                for (int j = 0; j < 8; ++j) bv[nt][j] = p[j];
            }
#pragma unroll
            for (int j = 0; j < 8; ++j)
#pragma unroll
                for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                    for (int nt = 0; nt < 4; ++nt)
                        acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x4f32(av[mt][j], bv[nt][j], acc[mt][nt], 0, 0, 0);
        }
    }
    finish<TOut, false, BT>(a, acc, smem, bq, t0, 0, blockIdx.y);
}

// PRECISE mode on the bf16 matrix cores, STZS_CONV_W_X3: split-operand ("bf16x3") products.  Every fp32
// operand v is split into hi = bf16(v) and lo = bf16(v - hi) (v = hi + lo to ~2^-17 relative), and
// a*b ~= ah*bh + ah*bl + al*bh on v_mfma_f32_16x16x32_bf16 (each product exact in fp32, fp32 accumulate; the
// dropped al*bl is ~2^-16 of the rest).  Input rows are split ONCE when staged (after the libm-accurate
// AdaIN / activation prologue, in fp32); weights arrive pre-split as two K-step streams (hi, then lo) in
// conv_mfma's swizzled layout with 32-channel chunks (stzs/weights.py kstep_stream_x3).  Same 128 x 128 tile,
// 2 x 2 waves, accumulator layout and fused epilogue (finish) as conv_mfma; per K-step 3 x 16 MFMAs.
// tools/precision_probe.py: this arithmetic in every GEMM of the pipeline keeps the end-to-end log-mel L1 at
// 2.2e-4 of the fp32 oracle; ~3x the bf16 MFMA work instead of the 16x of fp32 MFMA (conv_f32).
constexpr int XSLOT_C = 2 * SLOT_BYTES;  // one K-step: hi + lo weights
constexpr int PX = 80;  // staged row pitch, bytes: 32 bf16 + 16 (conflict-light ds_read_b128) ...
constexpr int PX_TIGHT = 64;  // ... or unpadded when the padded tiles would not fit (stride-6 noise convs: 774 rows)
__host__ __device__ inline int x3_pitch(int rows_in) {
    return 2 * ((rows_in * PX + 15) & ~15) + NSLOT * XSLOT_C + 3 * 32 * 4 <= 160 * 1024 ? PX : PX_TIGHT;
}
constexpr int XSLOT = XSLOT_C;
template <typename TIn, typename TOut, int PACT, bool FLAT>
__global__ __launch_bounds__(NTHR, 2) void conv_x3(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = FLAT ? 1 : a.ks;
    const int rows_in = (BT - 1) * a.stride + (ks - 1) * a.dil + 1;
    const int px = x3_pitch(rows_in);
    unsigned char* thi = smem;
    unsigned char* tlo = smem + ((rows_in * px + 15) & ~15);
    unsigned char* ring = tlo + ((rows_in * px + 15) & ~15);
    float* c_sc = reinterpret_cast<float*>(ring + NSLOT * XSLOT);
    float* c_sh = c_sc + 32;
    float* c_al = c_sh + 32;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    // FLAT (linears: ks 1, no prologue): 128 consecutive rows of the [B * T] row space per tile
    int bq = 0, t0 = 0;
    long row0 = 0;
    if (FLAT) {
        row0 = (long)blockIdx.x * BT;
    } else {
        const int tpb = (a.T_out + BT - 1) / BT;
        bq = blockIdx.x / tpb;
        t0 = (blockIdx.x - bq * tpb) * BT;
    }
    const int nchunk = a.ci_pad / 32;
    const int NK = nchunk * ks;
    const long stream_el = (long)(a.co_pad / BCO) * NK * (BCO * 32);  // bf16 elements of one (hi | lo) stream
    const bf16_t* Wh = reinterpret_cast<const bf16_t*>(a.w) + (long)blockIdx.y * NK * (BCO * 32);
    const TIn* X = reinterpret_cast<const TIn*>(a.x) + (FLAT ? 0 : (long)bq * a.bsx);
    const long nR = (long)a.B * a.T_in;
    const float invTi = 1.f / (float)a.T_in;  // (FLAT rows -> utterance, rowdiv)
    auto fill = [&](int k) {
        const bf16_t* src = Wh + (long)k * (BCO * 32) + wave * 1024 + lane * 8;
        unsigned char* dst = ring + (k % NSLOT) * XSLOT + wave * 2048;
#pragma unroll
        for (int h = 0; h < 2; ++h) {  // hi, lo
            const bf16_t* sh = src + h * stream_el;
            unsigned char* dh = dst + h * SLOT_BYTES;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)sh,
                                             (__attribute__((address_space(3))) void*)dh, 16, 0, 0);
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(sh + 512),
                                             (__attribute__((address_space(3))) void*)(dh + 1024), 16, 0, 0);
        }
    };
    int boff[4];
#pragma unroll
    for (int nt = 0; nt < 4; ++nt) {
        const int rr = wc * 64 + nt * 16 + (lane & 15);
        boff[nt] = rr * 64 + (((lane >> 4) ^ gswz(rr)) << 4);
    }
    f32x4 acc[4][4];
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    fill(0);
    if (NK > 1) fill(1);
    int k = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();  // previous chunk's tiles / constants consumed
        if (tid < 32) {   // per-channel prologue constants of this chunk (fp32, the oracle's formula)
            const int c = cc * 32 + tid;
            float sc = 0.f, sh = 0.f, al = 1.f;
            if (c < a.Ci) {
                sc = a.pro_cscale;
                if (a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = a.pro_mean[(long)bq * a.stat_bs + c];
                    const float rs = a.pro_rstd[(long)bq * a.stat_bs + c];
                    const float g = a.pro_gb[(long)bq * a.gb_bs + c];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + c];
                    sc = (1.f + g) * rs;
                    sh = be - mu * sc;
                }
                if (a.pro_alpha) al = a.pro_alpha[c];
            }
            c_sc[tid] = sc;
            c_sh[tid] = sh;
            c_al[tid] = al;
        }
        __syncthreads();
        // staging: rows_in x 4 vectors of 8 channels, prologue in fp32, split into the hi / lo tiles
        for (int v = tid; v < rows_in * 4; v += NTHR) {
            const int r = v >> 2, cv = v & 3;
            const int ci = cc * 32 + cv * 8;
            long off;
            bool rok;
            if (FLAT) {
                const long R = row0 + r;
                const long bb = rowdiv(R, a.T_in, invTi, nR + BT < (1L << 22));
                rok = R < nR;
                off = bb * a.bsx + (R - bb * a.T_in) * a.ldx;
            } else {
                const int tin = t0 * a.stride - a.pad + r;
                rok = tin >= 0 && tin < a.T_in;
                off = (long)tin * a.ldx;
            }
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) o[j] = 0.f;
            if (rok && ci < a.Ci) {
                float f[8];
                load8(X + off + ci, f);
#pragma unroll
                for (int j = 0; j < 8; ++j) {
                    const float y = f[j] * c_sc[cv * 8 + j] + c_sh[cv * 8 + j];
                    float z = y;
                    if constexpr (PACT == STZS_ACT_SNAKE) {
                        const float al = c_al[cv * 8 + j];
                        const float sn = sinf(al * y);
                        z = y + sn * sn / al;
                    } else if constexpr (PACT == STZS_ACT_LEAKY) {
                        z = y >= 0.f ? y : y * a.pro_slope;
                    }
                    o[j] = ci + j < a.Ci ? z : 0.f;
                }
            }
            float lo[8];
            uint4 hp = pack8(o);
            float hf[8];
            unpack8(hp, hf);
#pragma unroll
            for (int j = 0; j < 8; ++j) lo[j] = o[j] - hf[j];  // exact (Sterbenz-range subtraction)
            *reinterpret_cast<uint4*>(thi + r * px + cv * 16) = hp;
            *reinterpret_cast<uint4*>(tlo + r * px + cv * 16) = pack8(lo);
        }
        __syncthreads();
        for (int tap = 0; tap < ks; ++tap, ++k) {
            waitcnt_vm(k + 1 < NK ? 4 : 0);  // this K-step's 4 LDS-DMA pieces landed (the next may fly)
            __builtin_amdgcn_s_barrier();
            if (k + 2 < NK) fill(k + 2);
            const unsigned char* wl = ring + (k % NSLOT) * XSLOT;
            const int kb = 16 * (lane >> 4);
            bf16x8 ah[4], alo[4], bh[4], bl[4];
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) {
                const int r = (wt * 64 + mt * 16 + (lane & 15)) * a.stride + tap * a.dil;
                ah[mt] = *reinterpret_cast<const bf16x8*>(thi + r * px + kb);
                alo[mt] = *reinterpret_cast<const bf16x8*>(tlo + r * px + kb);
            }
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                bh[nt] = *reinterpret_cast<const bf16x8*>(wl + boff[nt]);
                bl[nt] = *reinterpret_cast<const bf16x8*>(wl + SLOT_BYTES + boff[nt]);
            }
            __builtin_amdgcn_sched_barrier(0);
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
#pragma unroll
                for (int nt = 0; nt < 4; ++nt) {
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(alo[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bl[nt], acc[mt][nt], 0, 0, 0);
                    acc[mt][nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ah[mt], bh[nt], acc[mt][nt], 0, 0, 0);
                }
        }
    }
    finish<TOut, FLAT, BT>(a, acc, smem, bq, t0, row0, blockIdx.y);
}

size_t x3_lds_bytes(int rows_in) {
    const size_t main = 2 * (((size_t)rows_in * x3_pitch(rows_in) + 15) & ~(size_t)15) + NSLOT * XSLOT + 3 * 32 * 4;
    const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
    return main > epi ? main : epi;
}

size_t lds_bytes(int rows_in, int cic) {
    const size_t main = (((size_t)rows_in * (cic * 2 + 16) + 15) & ~(size_t)15) + NSLOT * SLOT_BYTES + 4 * 128 * 4;
    const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
    return main > epi ? main : epi;
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

template <typename TIn, typename TOut, bool F8 = false>
int launch_dt(const stzs_conv_args& a, hipStream_t s) {
    const bool flat = (a.ks == 1 && a.stride == 1 && a.pad == 0 && a.ups == 0 && a.pro_mode == STZS_PRO_NONE &&
                       a.pro_act == STZS_ACT_NONE && a.T_in == a.T_out);
    const int rows_in = flat ? BT : (BT - 1) * a.stride + (a.ks - 1) * a.dil + 1;
    const size_t lds = lds_bytes(rows_in, a.cic);
    if (lds > 160 * 1024) return STZS_ESHAPE;
    const unsigned gx = flat ? (unsigned)(((long)a.B * a.T_out + BT - 1) / BT)
                             : (unsigned)a.B * (unsigned)((a.T_out + BT - 1) / BT);
    dim3 grid(gx, a.co_pad / BCO);
    if (flat && a.stat_part) return STZS_EINVAL;  // fused statistics: per-utterance tiles only
    void (*k)(stzs_conv_args);
    if (F8 || (flat && sizeof(TIn) == 2 && (a.flags & STZS_CONV_A_DMA) && a.pro_cscale == 1.f)) {
        // 64-row tiles when 128-row tiles would leave the GPU under-filled (< 2 workgroups per CU)
        const int n_cu = stzs_cu_count();
        bool small = (long)grid.x * grid.y < 2L * n_cu;
        size_t lg = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
        const size_t lr = 4 * (size_t)(small ? gslot<64>() : gslot<128>());
        lg = lg > lr ? lg : lr;
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
            lg = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
            lg = lg > 4 * (size_t)gslot<64>() ? lg : 4 * (size_t)gslot<64>();
        }
        if (small) grid.x = (unsigned)(((long)a.B * a.T_out + 63) / 64);
        (void)hipFuncSetAttribute((const void*)kg, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lg);
        hipLaunchKernelGGL(kg, grid, dim3(NTHR), lg, s, a);
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
    if (a.splitk > 1) {  // conv_mfma: split over input-channel chunks (2..8 slices, at least one chunk each)
        if (F8 || a.splitk > 8 || a.splitk > a.ci_pad / a.cic || !a.splitk_ws || !a.splitk_ctr ||
            !stzs_aligned(a.splitk_ws, 16) || !stzs_aligned(a.splitk_ctr, 4))
            return STZS_EINVAL;
        grid.z = (unsigned)a.splitk;
    }
    if constexpr (F8) {
        return STZS_EDTYPE;  // (unreachable: fp8 is a pure linear)
    } else {
        if (flat)
            k = conv_mfma<TIn, TOut, true, STZS_ACT_NONE>;
        else if (a.pro_act == STZS_ACT_SNAKE)
            k = conv_mfma<TIn, TOut, false, STZS_ACT_SNAKE>;
        else if (a.pro_act == STZS_ACT_LEAKY)
            k = conv_mfma<TIn, TOut, false, STZS_ACT_LEAKY>;
        else
            k = conv_mfma<TIn, TOut, false, STZS_ACT_NONE>;
        if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, a);
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
}

}  // namespace

int stzs_mrf_conv_launch(const stzs_conv_args& a, hipStream_t s);     // csrc/mrf.hip
int stzs_narrow_conv_launch(const stzs_conv_args& a, hipStream_t s);  // csrc/mrf.hip

// the dispatcher proper; csrc/dispatch.hip routes the register-direct MRF form before it
__attribute__((visibility("hidden"))) int stzs_conv1d_core(const stzs_conv_args* a, void* stream) {
    if (!a || !a->x || !a->w || !a->y) return STZS_EINVAL;
    if (a->cic != 32 && a->cic != 64 && a->cic != 128) return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0 || a->ks <= 0 || a->dil <= 0 ||
        a->stride <= 0)
        return STZS_ESHAPE;
    if (a->ci_pad % a->cic || a->ci_pad < a->Ci || a->co_pad % BCO) return STZS_ESHAPE;
    if (a->splitk > 1 && (a->flags & (STZS_CONV_W_X3 | STZS_CONV_W_F32 | STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
        return STZS_EINVAL;
    const int ncol = a->ups > 0 ? a->ups * a->Co : a->Co;
    if (a->co_pad < ncol) return STZS_ESHAPE;
    if (a->ldx % 8 || a->bsx % 8 || a->ldx < ((a->Ci + 7) / 8) * 8) return STZS_ESHAPE;
    if (!stzs_aligned(a->x, 16) || !stzs_aligned(a->w, 16)) return STZS_EINVAL;
    if (a->ups > 0) {
        if (a->ks != 2 || a->pad != 1 || a->stride != 1 || a->dil != 1 || a->T_out != a->T_in + 1) return STZS_ESHAPE;
        if (a->Co % 8) return STZS_ESHAPE;
        if (a->refl && a->T_final < 2) return STZS_ESHAPE;
    } else if (a->refl) {
        return STZS_EINVAL;
    }
    if (a->res && a->res_tdiv <= 0) return STZS_EINVAL;
    if (a->pro_mode == STZS_PRO_ADAIN && (!a->pro_mean || !a->pro_rstd || !a->pro_gb)) return STZS_EINVAL;
    if (a->pro_act == STZS_ACT_SNAKE && !a->pro_alpha) return STZS_EINVAL;
    if (a->stat_part && (a->ups > 0 || !epi_vec(*a) || a->stat_ld < a->Co || !stzs_aligned(a->stat_part, 8)))
        return STZS_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->in_dtype == STZS_F8) {
        const bool lin = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->T_in == a->T_out &&
                         a->pro_mode == STZS_PRO_NONE && a->pro_act == STZS_ACT_NONE && a->pro_cscale == 1.f;
        if (!lin || !(a->flags & STZS_CONV_A_DMA) || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
            return STZS_EDTYPE;
        if (!a->x_scale || !a->w_scale || a->stat_part) return STZS_EINVAL;
        if (a->ci_pad % 64 || a->ldx % 16 || a->bsx % 16) return STZS_ESHAPE;
        if (a->out_dtype == STZS_BF16) return launch_dt<f8_t, bf16_t, true>(*a, s);
        if (a->out_dtype == STZS_F32) return launch_dt<f8_t, float, true>(*a, s);
        return STZS_EDTYPE;
    }
    if (a->flags & STZS_CONV_W_X3) {
        if (a->cic != 32 || a->ci_pad % 32 || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32)))
            return STZS_EINVAL;
        if (a->in_dtype == STZS_F32 ? (a->ldx % 8 || a->bsx % 8) : false) return STZS_ESHAPE;
        const int rows_in = (BT - 1) * a->stride + (a->ks - 1) * a->dil + 1;
        const size_t lds = x3_lds_bytes(rows_in);
        if (lds > 160 * 1024) return STZS_ESHAPE;
        void (*k)(stzs_conv_args) = nullptr;
        const bool flat = a->ks == 1 && a->stride == 1 && a->pad == 0 && a->ups == 0 && a->pro_mode == STZS_PRO_NONE &&
                          a->pro_act == STZS_ACT_NONE && a->T_in == a->T_out && !a->stat_part;
#define STZS_X3_PICK(TI, TO)                                                                         \
    k = flat ? conv_x3<TI, TO, STZS_ACT_NONE, true>                                                  \
        : a->pro_act == STZS_ACT_SNAKE ? conv_x3<TI, TO, STZS_ACT_SNAKE, false>                      \
        : a->pro_act == STZS_ACT_LEAKY ? conv_x3<TI, TO, STZS_ACT_LEAKY, false> : conv_x3<TI, TO, STZS_ACT_NONE, false>;
        if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) { STZS_X3_PICK(float, float) }
        else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) { STZS_X3_PICK(float, bf16_t) }
        else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) { STZS_X3_PICK(bf16_t, float) }
        else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) { STZS_X3_PICK(bf16_t, bf16_t) }
        else return STZS_EDTYPE;
#undef STZS_X3_PICK
        if (a->pro_act != STZS_ACT_NONE && a->pro_act != STZS_ACT_LEAKY && a->pro_act != STZS_ACT_SNAKE)
            return STZS_EINVAL;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        dim3 grid(flat ? (unsigned)(((long)a->B * a->T_out + BT - 1) / BT)
                       : (unsigned)a->B * (unsigned)((a->T_out + BT - 1) / BT), a->co_pad / BCO);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, *a);
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
    if (a->flags & STZS_CONV_W_F32) {
        if (a->cic != 32 || a->ci_pad % 32 || (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32)))
            return STZS_EINVAL;
        const int rows_in = (BT - 1) * a->stride + (a->ks - 1) * a->dil + 1;
        const size_t main = (size_t)(rows_in + BCO) * P32 * 4;
        const size_t epi = (size_t)BT * EP_PITCH * 4 + 2 * BCO * 4 + 2 * 4 * BCO * 2 * 4;
        const size_t lds = main > epi ? main : epi;
        if (lds > 160 * 1024) return STZS_ESHAPE;
        void (*k)(stzs_conv_args) = nullptr;
        if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) k = conv_f32<float, float>;
        else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) k = conv_f32<float, bf16_t>;
        else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) k = conv_f32<bf16_t, float>;
        else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) k = conv_f32<bf16_t, bf16_t>;
        else return STZS_EDTYPE;
        (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
        dim3 grid((unsigned)a->B * (unsigned)((a->T_out + BT - 1) / BT), a->co_pad / BCO);
        hipLaunchKernelGGL(k, grid, dim3(NTHR), lds, s, *a);
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
    if (a->flags & STZS_CONV_W_LANE16) return stzs_mrf_conv_launch(*a, s);
    if (a->flags & STZS_CONV_W_NARROW32) return stzs_narrow_conv_launch(*a, s);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16) return launch_dt<bf16_t, bf16_t>(*a, s);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32) return launch_dt<bf16_t, float>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16) return launch_dt<float, bf16_t>(*a, s);
    if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32) return launch_dt<float, float>(*a, s);
    return STZS_EDTYPE;
}

extern "C" size_t stzs_conv_splitk_workspace(int64_t rows, int32_t co_pad, int32_t splitk) {
    if (rows <= 0 || co_pad <= 0 || co_pad % BCO || (splitk != 2 && splitk != 4)) return 0;
    const int64_t tiles = (rows + 63) / 64 * (co_pad / BCO);
    return (size_t)tiles * splitk * (64 / 32 * 4) * NTHR * 16;
}

#ifdef STZS_GEMM_PROF
extern "C" int stzs_gemm_prof_conv(const stzs_conv_args* a, void* stream) { return stzs_conv1d_core(a, stream); }
#endif
