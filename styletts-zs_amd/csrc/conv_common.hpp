// Device code shared by the MFMA conv / GEMM kernels (csrc/conv.hip conv_mfma, csrc/gemm.hip gemm_glds,
// csrc/convx.hip conv_f32 / conv_x3): tile constants, the prologue activations, the staged-row readers and the fused
// LDS epilogue (finish).  Each including file gets its own internal copy (anonymous namespace).
#pragma once
#include "common.hpp"

namespace {

typedef __attribute__((ext_vector_type(2))) long i64x2;
typedef __attribute__((ext_vector_type(4))) unsigned int u32x4;

constexpr int NTHR = 256;
constexpr int BT = 128, BCO = 128;
constexpr int NSLOT = 3;
constexpr int SLOT_BYTES = BCO * 32 * 2;  // one K-step of weights
constexpr int EP_PITCH = BCO + 4;         // fp32 epilogue row pitch (floats)

// STZS_CONV_PROF probe build (tools/conv_phase.py --build): thread 0 of every workgroup stamps s_memtime at the phase
// boundaries of conv_mfma / finish into g_cprof[workgroup][16] (slot 15: s_memrealtime at entry, 14: at exit, 13: XCC id)
#ifdef STZS_CONV_PROF
__device__ unsigned long long g_cprof[16 * 8192];
#define CPROF(i)                                                                                                   \
    if (threadIdx.x == 0) {                                                                                        \
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                       \
        if (wg_ < 8192) g_cprof[wg_ * 16 + (i)] = __builtin_amdgcn_s_memtime();                                    \
    }
#define CPROF_RT(i)                                                                                                \
    if (threadIdx.x == 0) {                                                                                        \
        const unsigned wg_ = blockIdx.x + gridDim.x * (blockIdx.y + gridDim.y * blockIdx.z);                       \
        if (wg_ < 8192) g_cprof[wg_ * 16 + (i)] = __builtin_amdgcn_s_memrealtime();                                \
    }
#else
#define CPROF(i)
#define CPROF_RT(i)
#endif


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
    // (FLAT: a linear, never a ConvTranspose -- the ups / ReflectionPad paths are compiled out, and with them the scalar
    // loads whose waits the compiler hoisted to the top of every row vector)
    const bool ups = !FLAT && a.ups > 0;
    const int ncol = ups ? a.ups * a.Co : a.Co;
    const long nrows_flat = (long)a.B * a.T_out;
    const bool small_rows = nrows_flat + BTM < (1L << 22);
    const float invTo = 1.f / (float)a.T_out;
    const long t_hi = ups ? (long)a.T_final + a.refl - 1 : (long)a.T_out - 1;
    const int cv = tid & 15;
    const int n = by * BCO + cv * 8;
    const bool col_ok = n < ncol;
    int co = n, p = 0;
    if (ups) {
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
            st_s[j] = xor32_sum(xor16_sum(st_s[j]));  // (common.hpp: the xor-16 / xor-32 shuffles' bits)
            st_q[j] = xor32_sum(xor16_sum(st_q[j]));
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
            if (ups) {
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
        // the row vectors' results are kept and stored together after the loop: a store's data registers reused by the
        // next row vector made hipcc wait for the store (vmcnt(0)) between row vectors
        uint4 pkv[EB];
        float ofv[EB][8];
        TOut* dstv[EB];
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
                dstv[i] = Y + bb * a.bsy + t * a.ldy + co;
                if constexpr (sizeof(TOut) == 2) {
                    const uint4 pk = pack8(o);
                    pkv[i] = pk;
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
#pragma unroll
                    for (int j = 0; j < 8; ++j) ofv[i][j] = o[j];
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
            if (ups && a.refl && t == 2) {  // ReflectionPad(1,0): row 0 mirrors source row 1
                for (int j = 0; j < 8 && co + j < a.Co; ++j) {
                    float x = u[j];
                    if (Rp) x += DT<TOut>::ld(Rp + bb * a.bsr + co + j);
                    x *= a.alpha;
                    if (AI) x += a.beta * DT<TOut>::ld(AI + bb * a.bsa + co + j);
                    DT<TOut>::st(Y + bb * a.bsy + co + j, x);
                }
            }
        }
        if constexpr (VEC) {
#pragma unroll
            for (int i = 0; i < EB; ++i) {
                if (!pv[i]) continue;
                if constexpr (sizeof(TOut) == 2) *reinterpret_cast<uint4*>(dstv[i]) = pkv[i];
                else store8(dstv[i], ofv[i]);
            }
        }
        if (stat) stat_flush(v0 == 0 ? 0 : 1);
        CPROF(9 + (v0 > 0))
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

template <int BTM, int RB = 1>
STZS_DEV bool splitk_combine_rt(const stzs_conv_args& a, f32x4 (&acc)[BTM / 32][4], unsigned char* smem, int SK, int z);
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
    CPROF(7)
    float* c_bias = ep + BTM * EP_PITCH;      // [BCO] bias, [BCO] gate (conv mode: one utterance)
    float* c_gate = c_bias + BCO;
    if (tid < BCO) {
        const int n = by * BCO + tid;
        const int co = a.ups > 0 ? n % a.Co : min(n, a.Co - 1);
        c_bias[tid] = a.bias ? a.bias[co] : 0.f;
        c_gate[tid] = (!FLAT && a.gate) ? a.gate[(long)bq * a.gate_bs + co] : 1.f;
    }
    __syncthreads();
    GPROF_E(6)
    CPROF(8)
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

}  // namespace
