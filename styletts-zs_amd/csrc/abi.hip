// Generic tensor-descriptor C-ABI (include/stzs.h "Generic tensor-descriptor entry points"):
// native host-side composition of the per-kernel entry points into the §8(a) operators -- argument checks,
// workspace carving, launch order -- plus the host-side weight packers (stzs/weights.py pack_conv / pack_lstm
// restated in C++, bit-identical: tests/test_abi_generic.py).  No kernels are defined here.
#include <math.h>
#include <stdlib.h>
#include <string.h>

#include <vector>

#include "abi_util.hpp"

using namespace stzs_abi;

namespace {

const int GSWZ[4] = {0, 2, 3, 1};  // 16-B chunk swizzle of a K-step row (stzs/weights.py _GSWZ)

// the [ks][co_pad][ci_pad] fp32 matrix of a conv (ConvTranspose: polyphase, 2 taps of ups * Co columns)
std::vector<float> unfold(const float* w, int Co, int Ci, int ks, int ups, const ConvGeom& g) {
    std::vector<float> wp((size_t)g.ks * g.co_pad * g.ci_pad, 0.f);
    auto at = [&](int tap, int col, int ci) -> float& { return wp[((size_t)tap * g.co_pad + col) * g.ci_pad + ci]; };
    if (ups) {  // w [Ci][Co][2 ups]: tap 0 <- w[:, co, p + ups], tap 1 <- w[:, co, p]
        for (int p = 0; p < ups; ++p)
            for (int co = 0; co < Co; ++co)
                for (int ci = 0; ci < Ci; ++ci) {
                    at(0, p * Co + co, ci) = w[((size_t)ci * Co + co) * (2 * ups) + p + ups];
                    at(1, p * Co + co, ci) = w[((size_t)ci * Co + co) * (2 * ups) + p];
                }
    } else {  // w [Co][Ci][ks]
        for (int co = 0; co < Co; ++co)
            for (int ci = 0; ci < Ci; ++ci)
                for (int k = 0; k < ks; ++k) at(k, co, ci) = w[((size_t)co * Ci + ci) * ks + k];
    }
    return wp;
}

int lane16_row(int rr) { return (rr & 64) + ((rr >> 2) & 3) * 16 + ((rr >> 4) & 3) * 4 + (rr & 3); }
int frag32_row(int rr) { return (rr & 96) + ((rr >> 2) & 3) * 8 + ((rr >> 4) & 1) * 4 + (rr & 3); }
int narrow32_row(int rr) { return ((rr >> 2) & 3) * 8 + ((rr >> 4) & 1) * 4 + (rr & 3); }

}  // namespace

// ======================================================================== packers
extern "C" size_t stzs_pack_conv_size(int Co, int Ci, int ks, int ups, int form) {
    if (Co <= 0 || Ci <= 0 || ks <= 0 || ups < 0) return 0;
    const ConvGeom g = geom(Co, Ci, ks, ups);
    switch (form) {
        case STZS_PACK_KSTEP: return (size_t)g.ks * g.co_pad * g.ci_pad * 2;
        case STZS_PACK_LANE16: return (g.cic == 128 && Co % 16 == 0) ? (size_t)g.ks * g.co_pad * g.ci_pad * 2 : 0;
        case STZS_PACK_FRAG32:  // MRF / AdaIN-block convs (k 3 / 7 / 11), the blocks' 1x1 shortcuts, the polyphase
                                // ConvTranspose (csrc/ups.hip)
            return (g.cic == 128 && (ups ? Co % 32 == 0 : (Co % 8 == 0 && (ks == 1 || ks == 3 || ks == 7 || ks == 11))))
                       ? (size_t)g.ks * g.co_pad * g.ci_pad * 2 : 0;
        case STZS_PACK_NARROW32: return (!ups && g.cic == 128 && Co <= 32) ? (size_t)g.ks * 32 * g.ci_pad * 2 : 0;
        case STZS_PACK_X3: return 2 * (size_t)g.ks * g.co_pad * g.ci_pad * 2;
        case STZS_PACK_FRAG32X3:  // the precise register-direct convs (csrc/mrfx.hip): k 3 / 7 / 11 convs, k 1 linears
            return (!ups && g.cic == 128 && Co % 8 == 0 && (ks == 1 || ks == 3 || ks == 7 || ks == 11))
                       ? 2 * (size_t)g.ks * g.co_pad * g.ci_pad * 2 : 0;
        default: return 0;
    }
}

extern "C" int stzs_pack_conv(const float* w, int Co, int Ci, int ks, int ups, int form, void* packed) {
    if (!w || !packed) return STZS_EINVAL;
    if (!stzs_pack_conv_size(Co, Ci, ks, ups, form)) return STZS_ESHAPE;
    const ConvGeom g = geom(Co, Ci, ks, ups);
    std::vector<float> wp = unfold(w, Co, Ci, ks, ups, g);
    uint16_t* o = (uint16_t*)packed;
    const int nchunk = g.ci_pad / g.cic, kpc = g.cic / 32, ncot = g.co_pad / 128;
    auto W = [&](int tap, int col, int ci) { return wp[((size_t)tap * g.co_pad + col) * g.ci_pad + ci]; };
    if (form == STZS_PACK_X3) {
        // two KSTEP streams with 32-channel chunks: hi = bf16(w), then lo = bf16(w - hi)
        // (stzs/weights.py kstep_stream_x3): [hl][cot][cc][tap][128 rows][4 positions x 8]
        size_t n = 0;
        for (int hl = 0; hl < 2; ++hl)
            for (int cot = 0; cot < ncot; ++cot)
                for (int cc = 0; cc < g.ci_pad / 32; ++cc)
                    for (int tap = 0; tap < g.ks; ++tap)
                        for (int r = 0; r < 128; ++r)
                            for (int p = 0; p < 4; ++p) {
                                const int c = p ^ GSWZ[(r >> 2) & 3];
                                for (int e = 0; e < 8; ++e) {
                                    const float v = W(tap, cot * 128 + r, cc * 32 + c * 8 + e);
                                    const uint16_t hi = h_bf16(v);
                                    o[n++] = hl ? h_bf16(v - h_f32(hi)) : hi;
                                }
                            }
        return STZS_OK;
    }
    if (form == STZS_PACK_KSTEP || form == STZS_PACK_LANE16) {
        // [cot][cc][tap][kq][128 rows][4 positions x 8]: position p of row r holds chunk p ^ g((r >> 2) & 3)
        size_t n = 0;
        for (int cot = 0; cot < ncot; ++cot)
            for (int cc = 0; cc < nchunk; ++cc)
                for (int tap = 0; tap < g.ks; ++tap)
                    for (int kq = 0; kq < kpc; ++kq)
                        for (int r = 0; r < 128; ++r) {
                            const int col = cot * 128 + (form == STZS_PACK_LANE16 ? lane16_row(r) : r);
                            for (int p = 0; p < 4; ++p) {
                                const int c = p ^ GSWZ[(r >> 2) & 3];
                                for (int e = 0; e < 8; ++e) o[n++] = h_bf16(W(tap, col, cc * g.cic + kq * 32 + c * 8 + e));
                            }
                        }
    } else if (form == STZS_PACK_FRAG32 || form == STZS_PACK_FRAG32X3) {
        // [cot][chunk][tap][kq]([hl])[w][nt][g][i][8]: packed row w*32 + nt*16 + i (frag32-permuted), channels
        // kq*32 + 8g; FRAG32X3: per K-step the hi block (bf16(w)) then the lo block (bf16(w - hi))
        const int nhl = form == STZS_PACK_FRAG32X3 ? 2 : 1;
        size_t n = 0;
        for (int cot = 0; cot < ncot; ++cot)
            for (int cc = 0; cc < nchunk; ++cc)
                for (int tap = 0; tap < g.ks; ++tap)
                    for (int kq = 0; kq < 4; ++kq)
                        for (int hl = 0; hl < nhl; ++hl)
                            for (int wv = 0; wv < 4; ++wv)
                                for (int nt = 0; nt < 2; ++nt)
                                    for (int gg = 0; gg < 4; ++gg)
                                        for (int i = 0; i < 16; ++i) {
                                            const int col = cot * 128 + frag32_row(wv * 32 + nt * 16 + i);
                                            for (int e = 0; e < 8; ++e) {
                                                const float v = W(tap, col, cc * 128 + kq * 32 + gg * 8 + e);
                                                const uint16_t hi = h_bf16(v);
                                                o[n++] = hl ? h_bf16(v - h_f32(hi)) : hi;
                                            }
                                        }
    } else {  // NARROW32: [cc][tap][kq][32 rows][4 positions x 8], rows narrow32-permuted, same swizzle
        size_t n = 0;
        for (int cc = 0; cc < nchunk; ++cc)
            for (int tap = 0; tap < g.ks; ++tap)
                for (int kq = 0; kq < kpc; ++kq)
                    for (int r = 0; r < 32; ++r) {
                        const int col = narrow32_row(r);
                        for (int p = 0; p < 4; ++p) {
                            const int c = p ^ GSWZ[(r >> 2) & 3];
                            for (int e = 0; e < 8; ++e) o[n++] = h_bf16(W(tap, col, cc * g.cic + kq * 32 + c * 8 + e));
                        }
                    }
    }
    return STZS_OK;
}

extern "C" int stzs_pack_lstm(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                              const float* w_ih_rev, const float* w_hh_rev, const float* b_ih_rev,
                              const float* b_hh_rev, int In, int H, void* ih_packed, float* ih_bias, void* whh_frags) {
    if (!w_ih || !w_hh || !b_ih || !b_hh || !w_ih_rev || !w_hh_rev || !b_ih_rev || !b_hh_rev || !ih_packed ||
        !ih_bias || !whh_frags)
        return STZS_EINVAL;
    if (In <= 0 || H <= 0 || H % 32) return STZS_ESHAPE;
    const int G4 = 4 * H;
    std::vector<float> wih((size_t)2 * G4 * In);
    memcpy(wih.data(), w_ih, sizeof(float) * G4 * In);
    memcpy(wih.data() + (size_t)G4 * In, w_ih_rev, sizeof(float) * G4 * In);
    const int rc = stzs_pack_conv(wih.data(), 2 * G4, In, 1, 0, STZS_PACK_KSTEP, ih_packed);
    if (rc) return rc;
    for (int j = 0; j < G4; ++j) {
        ih_bias[j] = b_ih[j] + b_hh[j];
        ih_bias[G4 + j] = b_ih_rev[j] + b_hh_rev[j];
    }
    // W_hh^T B-fragments [dir][4H/16][H/32][64 lanes][8]: lane l, element e = W_hh[ct*16 + (l & 15)][ks*32 + 8(l >> 4) + e]
    uint16_t* o = (uint16_t*)whh_frags;
    size_t n = 0;
    for (int dir = 0; dir < 2; ++dir) {
        const float* W = dir ? w_hh_rev : w_hh;
        for (int ct = 0; ct < G4 / 16; ++ct)
            for (int ks = 0; ks < H / 32; ++ks)
                for (int l = 0; l < 64; ++l)
                    for (int e = 0; e < 8; ++e)
                        o[n++] = h_bf16(W[(size_t)(ct * 16 + (l & 15)) * H + ks * 32 + 8 * (l >> 4) + e]);
    }
    return STZS_OK;
}

extern "C" int stzs_pack_lstm_x3(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh,
                                 const float* w_ih_rev, const float* w_hh_rev, const float* b_ih_rev,
                                 const float* b_hh_rev, int In, int H, void* ih_packed, float* ih_bias, void* whh_frags) {
    if (!w_ih || !w_hh || !b_ih || !b_hh || !w_ih_rev || !w_hh_rev || !b_ih_rev || !b_hh_rev || !ih_packed ||
        !ih_bias || !whh_frags)
        return STZS_EINVAL;
    if (In <= 0 || H <= 0 || H % 32) return STZS_ESHAPE;
    const int G4 = 4 * H;
    std::vector<float> wih((size_t)2 * G4 * In);
    memcpy(wih.data(), w_ih, sizeof(float) * G4 * In);
    memcpy(wih.data() + (size_t)G4 * In, w_ih_rev, sizeof(float) * G4 * In);
    const int rc = stzs_pack_conv(wih.data(), 2 * G4, In, 1, 0, STZS_PACK_X3, ih_packed);
    if (rc) return rc;
    for (int j = 0; j < G4; ++j) {
        ih_bias[j] = b_ih[j] + b_hh[j];
        ih_bias[G4 + j] = b_ih_rev[j] + b_hh_rev[j];
    }
    uint16_t* o = (uint16_t*)whh_frags;  // [hl][dir][4H/16][H/32][64 lanes][8]
    size_t n = 0;
    for (int hl = 0; hl < 2; ++hl)
        for (int dir = 0; dir < 2; ++dir) {
            const float* W = dir ? w_hh_rev : w_hh;
            for (int ct = 0; ct < G4 / 16; ++ct)
                for (int ks = 0; ks < H / 32; ++ks)
                    for (int l = 0; l < 64; ++l)
                        for (int e = 0; e < 8; ++e) {
                            const float v = W[(size_t)(ct * 16 + (l & 15)) * H + ks * 32 + 8 * (l >> 4) + e];
                            const uint16_t hi = h_bf16(v);
                            o[n++] = hl ? h_bf16(v - h_f32(hi)) : hi;
                        }
        }
    return STZS_OK;
}

// ======================================================================== operators
#define STZS_GENERIC_ARGS \
    const stzs_tensor_t *inputs, int n_in, stzs_tensor_t *outputs, int n_out, const stzs_params_t *p, void *workspace, \
        size_t ws_bytes, void *stream
#define STZS_CHECK(rc)               \
    do {                             \
        const int rc__ = (rc);       \
        if (rc__ != STZS_OK) return rc__; \
    } while (0)

// ---- a3
extern "C" size_t stzs_cfg_euler_step_workspace(const stzs_tensor_t*, int, const stzs_params_t*) { return 0; }
extern "C" int stzs_cfg_euler_step(STZS_GENERIC_ARGS) {
    (void)workspace;
    (void)ws_bytes;
    if (!inputs || !outputs || !p || n_in < 2 || n_out < 1) return STZS_EINVAL;
    const stzs_tensor_t &x = inputs[0], &D = inputs[1], &y = outputs[0];
    if (!x.data || !D.data || !y.data) return STZS_EINVAL;
    if (x.dtype != STZS_F32 || D.dtype != STZS_F32 || y.dtype != STZS_F32) return STZS_EDTYPE;
    if (x.ndim < 2 || numel(x) <= 0 || numel(x) != numel(D) || numel(x) != numel(y) || !contiguous(x) ||
        !contiguous(D) || !contiguous(y))
        return STZS_ESHAPE;
    const int R = (int)x.shape[0], cfg = p->i[0] != 0;
    if (cfg && R % 2) return STZS_ESHAPE;
    const int64_t N = numel(x) / R;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (y.data != x.data && hipMemcpyAsync(y.data, x.data, (size_t)numel(x) * 4, hipMemcpyDeviceToDevice, s) != hipSuccess)
        return STZS_EHIP;
    return stzs_cfg_euler((float*)y.data, (const float*)D.data, cfg ? R / 2 : R, (int)N, cfg, p->f[0], p->f[1],
                          p->f[2] - p->f[1], stream);
}

// ---- a6
extern "C" size_t stzs_duration_head_workspace(const stzs_tensor_t*, int, const stzs_params_t*) { return 0; }
extern "C" int stzs_duration_head(STZS_GENERIC_ARGS) {
    (void)p;
    (void)workspace;
    (void)ws_bytes;
    if (!inputs || !outputs || n_in < 1 || n_out < 1) return STZS_EINVAL;
    const stzs_tensor_t& lg = inputs[0];
    if (!act3(lg, STZS_F32) || !outputs[0].data) return STZS_EINVAL;
    const int B = (int)lg.shape[0], T = (int)lg.shape[1];
    if (outputs[0].dtype != STZS_I32 || numel(outputs[0]) != (int64_t)B * T || !contiguous(outputs[0]))
        return STZS_ESHAPE;
    stzs_dur_args a;
    memset(&a, 0, sizeof a);
    a.logits = (const float*)lg.data;
    a.dur = (int32_t*)outputs[0].data;
    if (n_out > 1) {
        if (outputs[1].dtype != STZS_F32 || numel(outputs[1]) != (int64_t)B * T || !contiguous(outputs[1]))
            return STZS_ESHAPE;
        a.dsum = (float*)outputs[1].data;
    }
    a.ldl = lg.stride[1];
    a.bsl = lg.stride[0];
    a.B = B;
    a.T = T;
    a.nbins = (int)lg.shape[2];
    return stzs_durations(&a, stream);
}

// ---- a7
extern "C" size_t stzs_length_regulate_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t*) {
    return (inputs && n_in >= 1) ? rupz((size_t)inputs[0].shape[0] * 4, 256) : 0;
}
extern "C" int stzs_length_regulate(STZS_GENERIC_ARGS) {
    (void)p;
    if (!inputs || !outputs || n_in < 1 || n_out < 1) return STZS_EINVAL;
    const stzs_tensor_t &d = inputs[0], &idx = outputs[0];
    if (!d.data || !idx.data || !workspace) return STZS_EINVAL;
    if (d.dtype != STZS_I32 || idx.dtype != STZS_I32) return STZS_EDTYPE;
    if (d.ndim != 2 || idx.ndim != 2 || d.shape[0] != idx.shape[0] || !contiguous(d) || !contiguous(idx))
        return STZS_ESHAPE;
    if (ws_bytes < stzs_length_regulate_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    stzs_align_args a;
    memset(&a, 0, sizeof a);
    a.dur = (const int32_t*)d.data;
    a.idx = (int32_t*)idx.data;
    a.total = (int32_t*)workspace;
    a.B = (int)d.shape[0];
    a.T = (int)d.shape[1];
    a.T40 = (int)idx.shape[1];
    return stzs_alignment(&a, stream);
}

// ---- a10
extern "C" size_t stzs_sine_gen_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || n_in < 1 || !p) return 0;
    return rupz((size_t)inputs[0].shape[0] * p->i[3] * inputs[0].shape[1] * 4, 256);
}
extern "C" int stzs_sine_gen(STZS_GENERIC_ARGS) {
    if (!inputs || !outputs || !p || n_in < 3 || n_out < 1 || !workspace) return STZS_EINVAL;
    const stzs_tensor_t &F0 = inputs[0], &mw = inputs[1], &sd = inputs[2], &har = outputs[0];
    if (!F0.data || !mw.data || !sd.data || !har.data) return STZS_EINVAL;
    if (F0.dtype != STZS_F32 || mw.dtype != STZS_F32 || sd.dtype != STZS_I32) return STZS_EDTYPE;
    const int hop = p->i[0], n_fft = p->i[1], hop_s = p->i[2], nh = p->i[3];
    if (F0.ndim != 2 || F0.stride[1] != 1 || hop <= 0 || hop_s <= 0 || nh <= 0 || numel(mw) < nh + 1 ||
        numel(sd) < F0.shape[0])
        return STZS_ESHAPE;
    const int B = (int)F0.shape[0], T80 = (int)F0.shape[1];
    const int64_t Tf = (int64_t)T80 * hop / hop_s + 1;
    if (!act3(har, har.dtype) || har.shape[0] != B || har.shape[1] != Tf || har.shape[2] < n_fft + 2) return STZS_ESHAPE;
    if (ws_bytes < stzs_sine_gen_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    stzs_source_args a;
    memset(&a, 0, sizeof a);
    a.f0 = (const float*)F0.data;
    a.seeds = (const uint32_t*)sd.data;
    a.merge_w = (const float*)mw.data;
    a.prefix = (float*)workspace;
    a.har = har.data;
    a.ldf = F0.stride[0];
    a.ldh = har.stride[1];
    a.bsh = har.stride[0];
    a.B = B;
    a.T80 = T80;
    a.hop = hop;
    a.n_fft = n_fft;
    a.hop_s = hop_s;
    a.nh = nh;
    a.sr = p->f[0];
    a.sine_amp = p->f[1];
    a.noise_std = p->f[2];
    a.voiced_thr = p->f[3];
    a.har_dtype = har.dtype;
    return stzs_harmonic_source(&a, stream);
}

// ---- a13
extern "C" size_t stzs_conv_post_istft_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || n_in < 1 || !p) return 0;
    return rupz((size_t)inputs[0].shape[0] * inputs[0].shape[1] * rup(p->i[0] + 2, 8) * 4, 256);
}
extern "C" int stzs_conv_post_istft(STZS_GENERIC_ARGS) {
    if (!inputs || !outputs || !p || n_in < 3 || n_out < 1 || !workspace) return STZS_EINVAL;
    const stzs_tensor_t &x = inputs[0], &w = inputs[1], &b = inputs[2], &wav = outputs[0];
    if (!act3(x, STZS_BF16) || !w.data || !b.data || !wav.data) return STZS_EINVAL;
    const int n_fft = p->i[0], hop_s = p->i[1], Co = n_fft + 2, Ci = (int)x.shape[2];
    const int B = (int)x.shape[0], Tf = (int)x.shape[1];
    if (n_fft <= 0 || hop_s <= 0 || wav.dtype != STZS_F32 || wav.ndim != 2 || wav.shape[0] != B ||
        wav.shape[1] != (int64_t)(Tf - 1) * hop_s || wav.stride[1] != 1 || numel(b) < Co)
        return STZS_ESHAPE;
    if (ws_bytes < stzs_conv_post_istft_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    const int ldp = rup(Co, 8);
    stzs_conv_args a = conv_base();
    conv_weights(a, w, (const float*)b.data, Co, Ci, 7, 0, Ci % 128 == 0 && Co <= 32 ? STZS_PACK_NARROW32 : STZS_PACK_KSTEP);
    a.x = x.data;
    a.y = workspace;
    a.ldx = x.stride[1];
    a.bsx = x.stride[0];
    a.ldy = ldp;
    a.bsy = (int64_t)Tf * ldp;
    a.B = B;
    a.T_in = a.T_out = Tf;
    a.pad = 3;
    a.out_dtype = STZS_F32;
    a.pro_act = STZS_ACT_LEAKY;
    a.pro_slope = p->f[0];
    STZS_CHECK(stzs_conv1d(&a, stream));
    stzs_istft_args q;
    memset(&q, 0, sizeof q);
    q.post = (const float*)workspace;
    q.wav = (float*)wav.data;
    q.ldp = ldp;
    q.bsp = (int64_t)Tf * ldp;
    q.bsw = wav.stride[0];
    q.B = B;
    q.Tf = Tf;
    q.n_fft = n_fft;
    q.hop_s = hop_s;
    return stzs_istft(&q, stream);
}

// ---- a5 / a8
extern "C" size_t stzs_bilstm_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || n_in < 1 || !p) return 0;
    const size_t B = inputs[0].shape[0], T = inputs[0].shape[1], H = p->i[0];
    // [LSTM counters 4096 | exchange slab | gate projections]
    return 4096 + rupz(stzs_lstm_workspace((int)B, (int)H, 2), 256) + rupz(B * T * 8 * H * 4, 256);
}
extern "C" int stzs_bilstm(STZS_GENERIC_ARGS) {
    if (!inputs || !outputs || !p || n_in < 4 || n_out < 1 || !workspace) return STZS_EINVAL;
    const stzs_tensor_t &x = inputs[0], &wih = inputs[1], &bias = inputs[2], &whh = inputs[3], &y = outputs[0];
    if (!act3(x, STZS_BF16) || !wih.data || !bias.data || !whh.data || !act3(y, STZS_BF16)) return STZS_EINVAL;
    const int H = p->i[0], B = (int)x.shape[0], T = (int)x.shape[1], In = (int)x.shape[2];
    if (H <= 0 || H % 32 || H > 256 || y.shape[0] != B || y.shape[1] != T || y.shape[2] < 2 * H || numel(bias) < 8 * H)
        return STZS_ESHAPE;
    if (ws_bytes < stzs_bilstm_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    Carve c(workspace);
    void* sync = c.take(4096);
    void* xchg = c.take(stzs_lstm_workspace(B, H, 2));
    float* gx = (float*)c.take((size_t)B * T * 8 * H * 4);
    // the exchange state lives in the caller's (possibly reused, possibly dirtied) scratch: reset it first
    STZS_CHECK(stzs_lstm_state_reset(sync, xchg, stream));
    stzs_conv_args a = conv_base();
    conv_weights(a, wih, (const float*)bias.data, 8 * H, In, 1, 0, STZS_PACK_KSTEP);
    a.x = x.data;
    a.y = gx;
    a.ldx = x.stride[1];
    a.bsx = x.stride[0];
    a.ldy = 8 * H;
    a.bsy = (int64_t)T * 8 * H;
    a.B = B;
    a.T_in = a.T_out = T;
    a.out_dtype = STZS_F32;
    if (x.stride[1] >= a.ci_pad) a.flags |= STZS_CONV_A_DMA;
    STZS_CHECK(stzs_conv1d(&a, stream));
    stzs_lstm_args l;
    memset(&l, 0, sizeof l);
    l.gx = gx;
    l.whhT = whh.data;
    l.y = y.data;
    l.xchg = xchg;
    l.sync = sync;
    l.ldg = 8 * H;
    l.bsg = (int64_t)T * 8 * H;
    l.ldy = y.stride[1];
    l.bsy = y.stride[0];
    l.B = B;
    l.T = T;
    l.H = H;
    l.ndir = 2;
    l.status = (n_out > 1 && outputs[1].data) ? (uint32_t*)outputs[1].data : nullptr;
    return stzs_lstm(&l, stream);
}

// ---- a11
extern "C" size_t stzs_conv_transpose_up_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || n_in < 1 || !p) return 0;
    const size_t Tn = (size_t)inputs[0].shape[1] * p->i[0] + (p->i[1] ? 1 : 0);
    return rupz((size_t)inputs[0].shape[0] * Tn * rup(p->i[6], 8) * 2, 256);
}
extern "C" int stzs_conv_transpose_up(STZS_GENERIC_ARGS) {
    if (!inputs || !outputs || !p || n_in < 6 || n_out < 1 || !workspace) return STZS_EINVAL;
    const stzs_tensor_t &x = inputs[0], &har = inputs[1], &wu = inputs[2], &bu = inputs[3], &wn = inputs[4],
                        &bn = inputs[5], &y = outputs[0];
    if (!act3(x, STZS_BF16) || !act3(har, STZS_BF16) || !act3(y, STZS_BF16) || !wu.data || !bu.data || !wn.data ||
        !bn.data)
        return STZS_EINVAL;
    const int r = p->i[0], last = p->i[1] != 0, nk = p->i[2], nstride = p->i[3], npad = p->i[4], hc = p->i[5],
              Co = p->i[6];
    const int B = (int)x.shape[0], T = (int)x.shape[1], Cin = (int)x.shape[2];
    const int Tn = T * r + (last ? 1 : 0);
    if (r <= 0 || nk <= 0 || nstride <= 0 || hc <= 0 || hc > har.shape[2] || Co <= 0 || y.shape[0] != B ||
        y.shape[1] != Tn || y.shape[2] < Co || har.shape[0] != B || numel(bu) < Co || numel(bn) < Co)
        return STZS_ESHAPE;
    if (ws_bytes < stzs_conv_transpose_up_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    const int ldsrc = rup(Co, 8);
    bf16_t* xsrc = (bf16_t*)workspace;
    // the noise conv of the harmonic features, written at the up-sampled rate
    stzs_conv_args n = conv_base();
    conv_weights(n, wn, (const float*)bn.data, Co, hc, nk, 0, STZS_PACK_KSTEP);
    n.x = har.data;
    n.y = xsrc;
    n.ldx = har.stride[1];
    n.bsx = har.stride[0];
    n.ldy = ldsrc;
    n.bsy = (int64_t)Tn * ldsrc;
    n.B = B;
    n.T_in = (int)har.shape[1];
    n.stride = nstride;
    n.pad = npad;
    n.T_out = Tn;
    if (nk == 1 && nstride == 1 && npad == 0 && har.stride[1] >= n.ci_pad) n.flags |= STZS_CONV_A_DMA;
    STZS_CHECK(stzs_conv1d(&n, stream));
    // LeakyReLU + polyphase ConvTranspose1d (+ ReflectionPad(1,0)) + the noise conv as the residual
    stzs_conv_args a = conv_base();
    conv_weights(a, wu, (const float*)bu.data, Co, Cin, 2, r,
                 (Cin % 128 == 0 && Co % 16 == 0) ? STZS_PACK_LANE16 : STZS_PACK_KSTEP);
    a.x = x.data;
    a.y = y.data;
    a.ldx = x.stride[1];
    a.bsx = x.stride[0];
    a.ldy = y.stride[1];
    a.bsy = y.stride[0];
    a.B = B;
    a.T_in = T;
    a.T_out = T + 1;
    a.pad = 1;
    a.ups_pad = (2 * r - r) / 2;
    a.T_final = T * r;
    a.refl = last;
    a.pro_act = STZS_ACT_LEAKY;
    a.pro_slope = p->f[0];
    a.res = xsrc;
    a.ldr = ldsrc;
    a.bsr = (int64_t)Tn * ldsrc;
    return stzs_conv1d(&a, stream);
}

// ---- a12
namespace {
struct MrfWs {
    size_t act, slab, stat, stats_ws;
};
MrfWs mrf_ws(int B, int T, int C) {
    const int Cc = rup(C, 8), ntile = (T + STZS_CONV_STAT_ROWS - 1) / STZS_CONV_STAT_ROWS;
    return MrfWs{rupz((size_t)B * T * C * 2, 256), rupz((size_t)B * ntile * Cc * 2 * 4, 256),
                 rupz((size_t)B * Cc * 4, 256), rupz(stzs_chan_stats_workspace(B, T, Cc), 256)};
}
}  // namespace

extern "C" size_t stzs_mrf_resblock_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || n_in < 1 || !p) return 0;
    const MrfWs w = mrf_ws((int)inputs[0].shape[0], (int)inputs[0].shape[1], (int)inputs[0].shape[2]);
    return 3 * w.act + w.slab + 8 * w.stat + w.stats_ws;  // bufA, bufB, t1 | slab | 4 x (mean, rstd) | x statistics
}
extern "C" int stzs_mrf_resblock(STZS_GENERIC_ARGS) {
    if (!inputs || !outputs || !p || n_in < 2 || n_out < 1 || !workspace) return STZS_EINVAL;
    const int C = p->i[0], nk = p->i[7], nd = p->i[8], form = p->i[9];
    if (nk < 1 || nk > 3 || nd < 1 || nd > 3) return STZS_ESHAPE;
    if (n_in != 2 + 6 * nk * nd) return STZS_EINVAL;
    const stzs_tensor_t &x = inputs[0], &gb = inputs[1], &yo = outputs[0];
    if (!act3(x, STZS_BF16) || !act3(yo, STZS_BF16) || !gb.data || gb.dtype != STZS_F32) return STZS_EINVAL;
    const int B = (int)x.shape[0], T = (int)x.shape[1];
    {  // no in-place form: y is written while later resblocks still read x (and its statistics describe x)
        const char *x0 = (const char*)x.data, *x1 = x0 + ((B - 1) * x.stride[0] + (T - 1) * x.stride[1] + C) * 2;
        const char *y0 = (const char*)yo.data, *y1 = y0 + ((B - 1) * yo.stride[0] + (T - 1) * yo.stride[1] + C) * 2;
        if (y0 < x1 && x0 < y1) return STZS_EINVAL;
    }
    if (x.shape[2] != C || C % 8 || yo.shape[0] != B || yo.shape[1] != T || yo.shape[2] < C || gb.ndim != 2 ||
        gb.shape[0] != B || gb.shape[1] < (int64_t)nk * nd * 4 * C)
        return STZS_ESHAPE;
    for (int i = 2; i < n_in; ++i)
        if (!inputs[i].data) return STZS_EINVAL;
    if (ws_bytes < stzs_mrf_resblock_workspace(inputs, n_in, p)) return STZS_ESHAPE;
    const MrfWs w = mrf_ws(B, T, C);
    Carve cv(workspace);
    bf16_t* buf[3] = {(bf16_t*)cv.take(w.act), (bf16_t*)cv.take(w.act), (bf16_t*)cv.take(w.act)};  // A, B, t1
    void* slab = cv.take(w.slab);
    float* st[8];
    for (int i = 0; i < 8; ++i) st[i] = (float*)cv.take(w.stat);
    void* sws = cv.take(w.stats_ws);
    const int Cc = rup(C, 8);
    const int64_t gbs = gb.stride[0];
    const float* G = (const float*)gb.data;
    // statistics of the stage input
    stzs_stats_args sa;
    memset(&sa, 0, sizeof sa);
    sa.x = x.data;
    sa.mean = st[0];
    sa.rstd = st[1];
    sa.partial = sws;
    sa.ld = x.stride[1];
    sa.bs = x.stride[0];
    sa.stat_bs = Cc;
    sa.B = B;
    sa.T = T;
    sa.C = Cc;
    sa.dtype = STZS_BF16;
    sa.eps = 1e-5f;
    STZS_CHECK(stzs_chan_stats(&sa, stream));
    auto finalize = [&](float* mean, float* rstd) {
        stzs_stats_args f;
        memset(&f, 0, sizeof f);
        f.mean = mean;
        f.rstd = rstd;
        f.partial = slab;
        f.stat_bs = Cc;
        f.B = B;
        f.T = T;
        f.C = Cc;
        f.eps = 1e-5f;
        return stzs_chan_stats_final(&f, STZS_CONV_STAT_ROWS, stream);
    };
    struct View {
        const void* p;
        int64_t ld, bs;
    };
    const View X{x.data, x.stride[1], x.stride[0]}, Y{yo.data, yo.stride[1], yo.stride[0]};
    const View A{buf[0], C, (int64_t)T * C}, Bv{buf[1], C, (int64_t)T * C}, T1{buf[2], C, (int64_t)T * C};
    for (int j = 0; j < nk; ++j) {
        const int k = p->i[1 + j];
        View cur = X;
        float *cm = st[0], *cr = st[1];
        for (int m = 0; m < nd; ++m) {
            const int dil = p->i[4 + m], L = j * nd + m;
            const stzs_tensor_t* in = inputs + 2 + 6 * L;  // c1 w, c1 b, alpha1, c2 w, c2 b, alpha2
            // c1: AdaIN(n1) + Snake(alpha1) -> dilated conv -> t1 (+ its statistics)
            stzs_conv_args a = conv_base();
            conv_weights(a, in[0], (const float*)in[1].data, C, C, k, 0, form);
            a.x = cur.p;
            a.ldx = cur.ld;
            a.bsx = cur.bs;
            a.y = (void*)T1.p;
            a.ldy = T1.ld;
            a.bsy = T1.bs;
            a.B = B;
            a.T_in = a.T_out = T;
            a.dil = dil;
            a.pad = dil * (k - 1) / 2;
            a.pro_mode = STZS_PRO_ADAIN;
            a.pro_mean = cm;
            a.pro_rstd = cr;
            a.stat_bs = Cc;
            a.pro_gb = G + (int64_t)L * 4 * C;
            a.gb_bs = gbs;
            a.gb_beta_off = C;
            a.pro_act = STZS_ACT_SNAKE;
            a.pro_alpha = (const float*)in[2].data;
            a.stat_part = slab;
            a.stat_ld = Cc;
            STZS_CHECK(stzs_conv1d(&a, stream));
            STZS_CHECK(finalize(st[2], st[3]));
            // c2: AdaIN(n2) + Snake(alpha2) -> conv -> + cur (the last layer: / nk, accumulated into y)
            const bool last = m == nd - 1;
            const View out = last ? Y : (cur.p == A.p ? Bv : A);
            stzs_conv_args b = conv_base();
            conv_weights(b, in[3], (const float*)in[4].data, C, C, k, 0, form);
            b.x = T1.p;
            b.ldx = T1.ld;
            b.bsx = T1.bs;
            b.y = (void*)out.p;
            b.ldy = out.ld;
            b.bsy = out.bs;
            b.B = B;
            b.T_in = b.T_out = T;
            b.pad = (k - 1) / 2;
            b.pro_mode = STZS_PRO_ADAIN;
            b.pro_mean = st[2];
            b.pro_rstd = st[3];
            b.stat_bs = Cc;
            b.pro_gb = G + (int64_t)L * 4 * C + 2 * C;
            b.gb_bs = gbs;
            b.gb_beta_off = C;
            b.pro_act = STZS_ACT_SNAKE;
            b.pro_alpha = (const float*)in[5].data;
            b.res = cur.p;
            b.ldr = cur.ld;
            b.bsr = cur.bs;
            b.alpha = last ? 1.f / nk : 1.f;
            b.beta = 1.f;
            if (last && j > 0) {
                b.acc_in = Y.p;
                b.lda = Y.ld;
                b.bsa = Y.bs;
            }
            if (!last) {
                b.stat_part = slab;
                b.stat_ld = Cc;
            }
            STZS_CHECK(stzs_conv1d(&b, stream));
            if (!last) {
                float* nm = st[4 + 2 * (m & 1)];
                float* nr = st[5 + 2 * (m & 1)];
                STZS_CHECK(finalize(nm, nr));
                cm = nm;
                cr = nr;
                cur = out;
            }
        }
    }
    return STZS_OK;
}
