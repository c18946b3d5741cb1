// Host-side helpers shared by the generic tensor-descriptor C-ABI translation units (csrc/abi.hip: packers and the
// single-kernel-family operators; csrc/abi_ops.hip: the composite denoiser / decoder-pre / F0-N operators): host bf16
// rounding, packed-conv geometry, descriptor checks, the workspace carve and the stzs_conv_args builders.
#pragma once
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include "common.hpp"

namespace stzs_abi {

// ------------------------------------------------------------------ host bf16 (RNE, NaN preserved)
inline uint16_t h_bf16(float f) {
    uint32_t u;
    memcpy(&u, &f, 4);
    if ((u & 0x7F800000u) == 0x7F800000u && (u & 0x007FFFFFu)) return (uint16_t)((u >> 16) | 0x40);  // quiet NaN
    const uint32_t r = 0x7FFFu + ((u >> 16) & 1u);
    return (uint16_t)((u + r) >> 16);
}

inline float h_f32(uint16_t h) {
    const uint32_t u = (uint32_t)h << 16;
    float f;
    memcpy(&f, &u, 4);
    return f;
}

inline int rup(int x, int m) { return (x + m - 1) / m * m; }
inline size_t rupz(size_t x, size_t m) { return (x + m - 1) / m * m; }

struct ConvGeom {
    int ks, ncol, cic, ci_pad, co_pad;
};
inline ConvGeom geom(int Co, int Ci, int ks, int ups) {
    ConvGeom g;
    g.ks = ups ? 2 : ks;
    g.ncol = ups ? ups * Co : Co;
    g.cic = Ci <= 32 ? 32 : (Ci <= 64 ? 64 : 128);
    g.ci_pad = rup(Ci, g.cic);
    g.co_pad = rup(g.ncol, 128);
    return g;
}
// ------------------------------------------------------------------ descriptor checks
inline bool act3(const stzs_tensor_t& t, int dtype) {  // [B, T, C] channels-last, unit channel stride
    return t.data && t.dtype == dtype && t.ndim == 3 && t.shape[0] > 0 && t.shape[1] > 0 && t.shape[2] > 0 &&
           t.stride[2] == 1 && t.stride[1] >= t.shape[2] && t.stride[0] >= t.stride[1] * t.shape[1];
}
inline bool vec(const stzs_tensor_t& t, int dtype, int64_t n) {
    return t.data && t.dtype == dtype && t.ndim >= 1 && (n < 0 || t.shape[0] * (t.ndim > 1 ? t.shape[1] : 1) >= n);
}
inline int64_t numel(const stzs_tensor_t& t) {
    int64_t n = 1;
    for (int d = 0; d < t.ndim; ++d) n *= t.shape[d];
    return n;
}
inline bool contiguous(const stzs_tensor_t& t) {
    int64_t s = 1;
    for (int d = t.ndim - 1; d >= 0; --d) {
        if (t.shape[d] > 1 && t.stride[d] != s) return false;
        s *= t.shape[d];
    }
    return true;
}

// bump allocator over the caller's workspace (256-B aligned pieces)
struct Carve {
    char* base;
    size_t off = 0;
    explicit Carve(void* b) : base((char*)b) {}
    void* take(size_t n) {
        void* p = base ? base + off : nullptr;
        off = rupz(off + n, 256);
        return p;
    }
};

inline stzs_conv_args conv_base() {
    stzs_conv_args a;
    memset(&a, 0, sizeof a);
    a.dil = 1;
    a.stride = 1;
    a.alpha = 1.f;
    a.res_tdiv = 1;
    a.pro_cscale = 1.f;
    a.in_dtype = a.out_dtype = STZS_BF16;
    return a;
}
inline void conv_weights(stzs_conv_args& a, const stzs_tensor_t& w, const float* bias, int Co, int Ci, int ks, int ups,
                  int form) {
    const ConvGeom g = geom(Co, Ci, ks, ups);
    a.w = w.data;
    a.bias = bias;
    a.Co = Co;
    a.Ci = Ci;
    a.ks = g.ks;
    a.ups = ups;
    a.ci_pad = g.ci_pad;
    a.co_pad = g.co_pad;
    a.cic = g.cic;
    a.flags |= form == STZS_PACK_LANE16 ? STZS_CONV_W_LANE16
             : form == STZS_PACK_FRAG32 ? STZS_CONV_W_FRAG32
             : form == STZS_PACK_NARROW32 ? STZS_CONV_W_NARROW32 : 0;
}

}  // namespace stzs_abi
