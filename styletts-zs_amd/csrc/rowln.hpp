// Row LayerNorm of one row per wave: two-pass mean / variance in registers,
// fused modulation (gadd + G) * x_hat + Bt and activation, bf16 / fp32 / e4m3fn (power-of-two row scale)
// output.  stzs_row_layernorm (csrc/norm.hip) is built from these
// building blocks (the row math is separated from the loads so other kernels can reuse it).
#pragma once
#include "common.hpp"

namespace stzs_ln {

template <int MAXV>
STZS_DEV void store_f8_row(f8_t* Y, float (&v)[MAXV][8], int nv, int lane, float amax, float* scale);

// the LayerNorm of one register-resident row in three steps (lane holds the 8-value vectors lane + 64 i): statistics,
// the modulation vectors of the row's group, the finished vectors -- stzs_row_layernorm runs them back to back,
// csrc/lnrows.hip takes the statistics of many rows before their (shared) modulation vectors arrive.  Same arithmetic.
template <int MAXV>
STZS_DEV void ln_row_stats(const stzs_rowln_args& a, int lane, const float (&v)[MAXV][8], float& mu, float& rstd) {
    const int nv = a.C >> 3;
    float s = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
        if (lane + i * 64 < nv)
#pragma unroll
            for (int j = 0; j < 8; ++j) s += v[i][j];
    mu = wave_sum(s) / a.C;
    float q = 0.f;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float d = v[i][j] - mu;
                q += d * d;
            }
        }
    }
    rstd = 1.f / sqrtf(wave_sum(q) / a.C + a.eps);
}

// modulation vectors (G, Bt rows of group grp) of this lane's channel vectors; absent ones are left unset
template <int MAXV>
STZS_DEV void ln_mod_load(const stzs_rowln_args& a, long grp, int lane, float (&g)[MAXV][8], float (&bt)[MAXV][8]) {
    const int nv = a.C >> 3;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
            if (a.G) load8(a.G + grp * a.gs + vi * 8, g[i]);
            if (a.Bt) load8(a.Bt + grp * a.bs + vi * 8, bt[i]);
        }
    }
}

// put(i, vi, o) receives each finished 8-value vector (register slot i, vector vi): the global store of
// stzs_row_layernorm, or csrc/lnrows.hip's LDS operand image
template <int MAXV, typename Put>
STZS_DEV void ln_row_out(const stzs_rowln_args& a, int lane, const float (&v)[MAXV][8], float mu, float rstd,
                         const float (&g)[MAXV][8], const float (&bt)[MAXV][8], Put put) {
    const int nv = a.C >> 3;
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
            float o[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                const float gg = a.gadd + (a.G ? g[i][j] : 0.f);
                o[j] = act_apply(a.act, (v[i][j] - mu) * rstd * gg + (a.Bt ? bt[i][j] : 0.f), a.slope, 1.f);
            }
            put(i, vi, o);
        }
    }
}

// normalise, modulate, activate and store row r whose values are in registers (lane holds the 8-value
// vectors lane + 64 i)
template <typename TO, int MAXV>
STZS_DEV void ln_row_finish(const stzs_rowln_args& a, long r, int lane, float (&v)[MAXV][8]) {
    const int nv = a.C >> 3;
    TO* Y = reinterpret_cast<TO*>(a.y) + r * a.ldy;
    // (modulation rows as 32-B vectors: gs, bs and the bases are multiples of 8 floats, checked on the host)
    constexpr bool F8 = sizeof(TO) == 1;
    float amax = 0.f, mu, rstd, g[MAXV][8], bt[MAXV][8];
    ln_row_stats<MAXV>(a, lane, v, mu, rstd);
    ln_mod_load<MAXV>(a, r / a.gdiv, lane, g, bt);
    ln_row_out<MAXV>(a, lane, v, mu, rstd, g, bt, [&](int i, int vi, const float* o) {
        if constexpr (F8) {  // (slot i was consumed above: overwritten with its result)
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                v[i][j] = o[j];
                amax = fmaxf(amax, fabsf(o[j]));
            }
        } else {
            store8(Y + vi * 8, o);
        }
    });
    if constexpr (F8) store_f8_row(reinterpret_cast<f8_t*>(Y), v, nv, lane, amax, a.y_scale + r);
}

// one row of stzs_row_layernorm on one wave (lane = lane id)
template <typename TI, typename TO>
STZS_DEV void row_ln_one(const stzs_rowln_args& a, long r, int lane) {
    constexpr int MAXV = 4;
    const TI* X = reinterpret_cast<const TI*>(a.x) + r * a.ldx;
    const int nv = a.C >> 3;
    float v[MAXV][8];
#pragma unroll
    for (int i = 0; i < MAXV; ++i)
        if (lane + i * 64 < nv) load8(X + (lane + i * 64) * 8, v[i]);
    ln_row_finish<TO, MAXV>(a, r, lane, v);
}

// quantise a register-resident row (lane holds vectors lane + 64 i) to e4m3fn with one row scale
template <int MAXV>
STZS_DEV void store_f8_row(f8_t* Y, float (&v)[MAXV][8], int nv, int lane, float amax, float* scale) {
    amax = wave_max(amax);
    // power-of-two row scale 2^k, the smallest with amax / 2^k <= 448 (e4m3fn max): the scaling itself is
    // exact, so the codes are a pure function of the fp32 values (host restatement: tests/test_gpu_fp8.py)
    int k = 0;
    if (amax > 0.f) {
        int e;
        const float m = frexpf(amax, &e);  // amax = m 2^e, m in [0.5, 1); 448 = 0.875 2^9
        k = m <= 0.875f ? e - 9 : e - 8;
    }
    const float inv = ldexpf(1.f, -k);
#pragma unroll
    for (int i = 0; i < MAXV; ++i) {
        const int vi = lane + i * 64;
        if (vi < nv) {
            float t[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) t[j] = f8_clamp(v[i][j] * inv);
            *reinterpret_cast<uint2*>(Y + vi * 8) = pack8f8(t);
        }
    }
    if (lane == 0) *scale = ldexpf(1.f, k);
}

}  // namespace stzs_ln
