// Shared device helpers for the gfx950 (CDNA4) kernels of libstzs_hip.so.
// Wave = 64 lanes everywhere; bf16 is stored as raw 16-bit words and converted with RNE.
#pragma once
#include <hip/hip_runtime.h>
#include <stdint.h>
#include <string.h>

#include "../../include/stzs.h"

typedef __attribute__((ext_vector_type(8))) __bf16 bf16x8;
typedef __attribute__((ext_vector_type(4))) float f32x4;
typedef uint16_t bf16_t;

#define STZS_DEV __device__ __forceinline__

STZS_DEV float bf2f(bf16_t v) { return __uint_as_float(((uint32_t)v) << 16); }
STZS_DEV bf16_t f2bf(float f) {
    __bf16 h = (__bf16)f;  // v_cvt_pk_bf16_f32: RNE, NaN-preserving on gfx950
    return __builtin_bit_cast(bf16_t, h);
}
typedef __attribute__((ext_vector_type(2))) __bf16 bf16x2;
typedef __attribute__((ext_vector_type(2))) float f32x2;
// two floats -> one packed bf16 pair (lo = a) in a single v_cvt_pk_bf16_f32
STZS_DEV uint32_t pack2bf(float a, float b) {
    return __builtin_bit_cast(uint32_t, __builtin_convertvector((f32x2){a, b}, bf16x2));
}

// XCD-aware bijective remap of a linear workgroup id: the dispatcher deals ids round-robin over the 8 XCDs
// (id % 8 labels the blocks that share an L2), so give each such group a CONTIGUOUS range of tiles --
// neighbouring time tiles then share their dilation halos (and weight K-steps) in one L2.  Speed only: any
// bijection is correct (cdna_hip_programming.md T1, bijective form for nwg % 8 != 0).
// InstanceNorm mean / rstd from the fp64 (sum, sumsq) of T rows, every rounding explicit (no contraction choice left
// to the compiler): stzs_chan_stats_final and the conv prologue's pro_part path (conv.hip) give the same bits
STZS_DEV void stat_finish(double s, double q, int T, float eps, float& mu, float& rs) {
#pragma clang fp contract(off)
    const double mean = s / (double)T;
    double var = q / (double)T - mean * mean;
    if (var < 0.0) var = 0.0;
    mu = (float)mean;
    rs = (float)(1.0 / __dsqrt_rn(var + (double)eps));
}

STZS_DEV int xcd_remap(int bid, int nwg) {
    const int q = nwg >> 3, r = nwg & 7, x = bid & 7;
    return (x < r ? x * (q + 1) : r * (q + 1) + (x - r) * q) + (bid >> 3);
}

template <typename T> struct DT;
template <> struct DT<float> {
    static STZS_DEV float ld(const float* p) { return *p; }
    static STZS_DEV void st(float* p, float v) { *p = v; }
};
template <> struct DT<bf16_t> {
    static STZS_DEV float ld(const bf16_t* p) { return bf2f(*p); }
    static STZS_DEV void st(bf16_t* p, float v) { *p = f2bf(v); }
};

// load 8 consecutive elements (16-B aligned for bf16, 32-B for f32) as floats
STZS_DEV void load8(const bf16_t* p, float* v) {
    uint4 u = *reinterpret_cast<const uint4*>(p);
    uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}
STZS_DEV void load8(const float* p, float* v) {
    float4 a = *reinterpret_cast<const float4*>(p);
    float4 b = *reinterpret_cast<const float4*>(p + 4);
    v[0] = a.x; v[1] = a.y; v[2] = a.z; v[3] = a.w;
    v[4] = b.x; v[5] = b.y; v[6] = b.z; v[7] = b.w;
}
STZS_DEV void unpack8(const uint4& u, float* v) {
    const uint32_t w[4] = {u.x, u.y, u.z, u.w};
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        v[2 * i] = __uint_as_float(w[i] << 16);
        v[2 * i + 1] = __uint_as_float(w[i] & 0xFFFF0000u);
    }
}
STZS_DEV uint4 pack8(const float* v) {
    uint32_t w[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) w[i] = pack2bf(v[2 * i], v[2 * i + 1]);
    return make_uint4(w[0], w[1], w[2], w[3]);
}
STZS_DEV void store8(bf16_t* p, const float* v) { *reinterpret_cast<uint4*>(p) = pack8(v); }
STZS_DEV void store8(float* p, const float* v) {
    *reinterpret_cast<float4*>(p) = make_float4(v[0], v[1], v[2], v[3]);
    *reinterpret_cast<float4*>(p + 4) = make_float4(v[4], v[5], v[6], v[7]);
}

// fp8 (OCP e4m3fn on gfx950): raw byte codes; per-row scaled so |v| <= 448 before conversion
typedef uint8_t f8_t;
// 8 floats already in [-448, 448] -> 8 e4m3fn codes (two v_cvt_pk_fp8_f32 per 4 values, RNE)
STZS_DEV uint2 pack8f8(const float* v) {
    int lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[0], v[1], 0, false);
    lo = __builtin_amdgcn_cvt_pk_fp8_f32(v[2], v[3], lo, true);
    int hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[4], v[5], 0, false);
    hi = __builtin_amdgcn_cvt_pk_fp8_f32(v[6], v[7], hi, true);
    return make_uint2((uint32_t)lo, (uint32_t)hi);
}
STZS_DEV float f8_clamp(float x) { return fminf(fmaxf(x, -448.f), 448.f); }

STZS_DEV float act_apply(int act, float x, float slope, float alpha) {
    switch (act) {
        case STZS_ACT_LEAKY: return x >= 0.f ? x : x * slope;
        case STZS_ACT_SNAKE: {
            float s = sinf(alpha * x);
            return x + s * s / alpha;
        }
        case STZS_ACT_GELU: return 0.5f * x * (1.f + erff(x * 0.70710678118654752f));
        case STZS_ACT_SILU: return x / (1.f + expf(-x));
        default: return x;
    }
}

// Cross-lane butterflies without ds_bpermute (r06).  xor 32 / xor 16: v_permlane32_swap / v_permlane16_swap with both
// operands = v (lanes 32-63 of one copy trade places with lanes 0-31 of the other, resp. the odd 16-lane rows with the
// even ones), whose two results are {own, partner} in some order -- their sum / max is the xor partner's, bit for bit
// (commutative).  xor 8 / 4 / 2 / 1 after those: DPP row rotations (row_ror 8 is xor 8; after it every value has period
// 8 within its row, so row_ror 4 fetches the xor-4 partner's value, likewise 2 and 1).  Same bits as the xor shuffles.
template <int CTRL>
STZS_DEV float dpp_f32(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
STZS_DEV float xor32_sum(float v) {
    const auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
STZS_DEV float xor16_sum(float v) {
    const auto r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    return __uint_as_float(r[0]) + __uint_as_float(r[1]);
}
STZS_DEV float wave_sum(float v) {
    v = xor32_sum(v);
    v = xor16_sum(v);
    v += dpp_f32<0x128>(v);  // row_ror:8
    v += dpp_f32<0x124>(v);
    v += dpp_f32<0x122>(v);
    v += dpp_f32<0x121>(v);
    return v;
}
STZS_DEV float wave_max(float v) {
    auto r = __builtin_amdgcn_permlane32_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    r = __builtin_amdgcn_permlane16_swap(__float_as_uint(v), __float_as_uint(v), false, false);
    v = fmaxf(__uint_as_float(r[0]), __uint_as_float(r[1]));
    v = fmaxf(v, dpp_f32<0x128>(v));
    v = fmaxf(v, dpp_f32<0x124>(v));
    v = fmaxf(v, dpp_f32<0x122>(v));
    v = fmaxf(v, dpp_f32<0x121>(v));
    return v;
}

#define STZS_LAUNCH_CHECK()                                          \
    do {                                                             \
        hipError_t e__ = hipGetLastError();                          \
        if (e__ != hipSuccess) return STZS_EHIP;                     \
    } while (0)

static inline bool stzs_aligned(const void* p, size_t a) { return ((uintptr_t)p % a) == 0; }

// CU count of the current device for grid sizing, queried once per process (a function-local static: C++11
// thread-safe initialisation, no racing writers).  One process drives one GPU.
static inline int stzs_cu_count() {
    static const int n = [] {
        int dev = 0, c = 0;
        if (hipGetDevice(&dev) != hipSuccess || hipDeviceGetAttribute(&c, hipDeviceAttributeMultiprocessorCount, dev) !=
                                                     hipSuccess || c <= 0)
            c = 256;
        return c;
    }();
    return n;
}
