// Composite §8(b) operators of the generic tensor-descriptor C-ABI (include/stzs.h): a2 denoiser_fwd, a9
// decoder_pre, a8 f0n_predictor -- the three hot-path rows whose weights are dozens of packed tensors.  Each one is
// the engine's launch sequence (stzs/engine.py denoiser_prepare + denoiser_step, decoder_pre + blk,
// f0n_predictor) restated in native host code over the per-kernel entry points, with the same kernel choices and
// arguments, so its results are bit-identical to the engine path (tests/test_gpu_abi_generic.py), and a C / C++
// host can run one full NFE, the decoder front blocks or the prosody curves without Python.
//
// Every operator is written ONCE as a function over a Ctx: in the dry pass (the *_workspace query) the Ctx only
// carves the workspace and launches nothing; in the real pass it carves the same pieces and launches.  The
// workspace is caller-owned scratch with no required contents: buffers whose padding channels a kernel reads are
// zeroed here, and the LSTM exchange state is reset on entry (stzs_lstm_state_reset).
// The per-input order of each operator is the enum in include/stzs.h (STZS_DN_*, STZS_DP_*, STZS_FN_*).
#include <math.h>

#include "abi_util.hpp"

using namespace stzs_abi;

namespace {

inline int esz(int dt) { return dt == STZS_F32 ? 4 : (dt == STZS_BF16 ? 2 : (dt == STZS_F8 ? 1 : 4)); }

// channels-last activation view: element (b, t, c) at base + (b * bs + t * ld + c0 + c) * esz
struct Act {
    char* base = nullptr;
    int64_t ld = 0, bs = 0;
    int B = 0, T = 0, C = 0, c0 = 0, dt = STZS_BF16;
    void* ptr() const { return base ? base + (size_t)c0 * esz(dt) : nullptr; }
    Act sl(int c, int n) const {
        Act a = *this;
        a.c0 += c;
        a.C = n;
        return a;
    }
};
inline Act act_of(const stzs_tensor_t& t) {
    Act a;
    a.base = (char*)t.data;
    a.B = (int)t.shape[0];
    a.T = (int)t.shape[1];
    a.C = (int)t.shape[2];
    a.ld = t.stride[1];
    a.bs = t.stride[0];
    a.dt = t.dtype;
    return a;
}

struct Stats {
    float* mean;
    float* rstd;
    int64_t stat_bs;
};
struct Pro {  // AdaIN prologue: InstanceNorm statistics + gamma | beta rows (gamma at gb, beta at gb + beta_off)
    Stats st;
    const float* gb;
    int64_t gb_bs, beta_off;
};

struct ConvOpt {
    int T_out = -1, pad = 0, dil = 1, stride = 1;
    const Pro* pro = nullptr;
    int pro_act = STZS_ACT_NONE;
    float pro_slope = 0.f, cscale = 1.f;
    const Act* res = nullptr;
    int res_tdiv = 1;
    const Act* acc = nullptr;
    float alpha = 1.f, beta = 0.f;
    const float* gate = nullptr;
    int64_t gate_bs = 0;
    int epi_act = STZS_ACT_NONE;
    float epi_slope = 0.f;
    Stats* stats_out = nullptr;  // fused InstanceNorm statistics of the stored output
    bool rows = false;           // per-utterance linear: the whole-chip small-M form when K allows (rows_ok)
};

// the engine's rule for its per-utterance linears (stzs/engine.py _rows_z): one K slice, every wave the same
// K-step count
bool rows_ok(int ci_pad) {
    const int nk = ci_pad / 32;
    return ci_pad % 32 == 0 && nk % 4 == 0 && (nk / 4 == 1 || nk / 4 == 2 || nk / 4 == 4 || nk / 4 == 8 || nk / 4 == 16);
}

// a packed conv / linear: weights (STZS_PACK_* form), fp32 bias (or none)
struct CW {
    const stzs_tensor_t* w;
    const stzs_tensor_t* b;
    int Co, Ci, ks, form;
};
// the engine's form rule for the k3 AdaIN-block convs (stzs/weights.py pack_blk): the register-direct form for
// 128-channel chunks and Co % 32 == 0, the LDS-ring MRF form for Co % 16 == 0, else the general one
inline int blk_form(int Co, int Ci) {
    return (Ci > 64 && Co % 32 == 0) ? STZS_PACK_FRAG32 : (Ci > 64 && Co % 16 == 0) ? STZS_PACK_LANE16 : STZS_PACK_KSTEP;
}
// ... and for the blocks' 1x1 shortcut (r06): the register-direct form under the same condition, else the K-step one
inline int sc_form(int Co, int Ci) { return (Ci > 64 && Co % 32 == 0) ? STZS_PACK_FRAG32 : STZS_PACK_KSTEP; }

struct Ctx {
    Carve cv;
    bool dry;
    void* stream;
    explicit Ctx(void* ws, bool dry_, void* s) : cv(dry_ ? nullptr : ws), dry(dry_), stream(s) {}
    void* take(size_t n) { return cv.take(n); }
    float* f32(size_t n) { return (float*)take(n * 4); }
    // a channels-last buffer [B, T, rup(C, 8)]; zeroed when it has padding channels (a conv's 16-B staging reads a
    // partly valid 8-channel vector whole and weights it by zero-padded weights: garbage there would be NaN * 0)
    // or when the caller asks (buffers only partly written by their producers)
    int act(Act& a, int B, int T, int C, int dt, bool zero = false) {
        a = Act();
        a.B = B;
        a.T = T;
        a.C = C;
        a.dt = dt;
        a.ld = rup(C, 8);
        a.bs = (int64_t)T * a.ld;
        const size_t n = (size_t)B * a.bs * esz(dt);
        a.base = (char*)take(n);
        if (!dry && (zero || a.ld != C) && hipMemsetAsync(a.base, 0, n, reinterpret_cast<hipStream_t>(stream)) != hipSuccess)
            return STZS_EHIP;
        return STZS_OK;
    }
    size_t used() const { return cv.off; }
};

#define CK(x)                          \
    do {                               \
        const int rc__ = (x);          \
        if (rc__ != STZS_OK) return rc__; \
    } while (0)

// InstanceNorm statistics over time of x's channels (stzs_chan_stats), the engine's stats()
int stats(Ctx& c, const Act& x, Stats& st) {
    const int Cc = rup(x.C, 8);
    st.mean = c.f32((size_t)x.B * Cc);
    st.rstd = c.f32((size_t)x.B * Cc);
    st.stat_bs = Cc;
    void* ws = c.take(stzs_chan_stats_workspace(x.B, x.T, Cc) + 4);
    if (c.dry) return STZS_OK;
    stzs_stats_args a;
    memset(&a, 0, sizeof a);
    a.x = x.ptr();
    a.mean = st.mean;
    a.rstd = st.rstd;
    a.partial = ws;
    a.ld = x.ld;
    a.bs = x.bs;
    a.stat_bs = Cc;
    a.B = x.B;
    a.T = x.T;
    a.C = Cc;
    a.dtype = x.dt;
    a.eps = 1e-5f;
    return stzs_chan_stats(&a, c.stream);
}

// the engine's conv(): argument fill, LDS-DMA flag rule, optional fused statistics + finalize
int conv(Ctx& c, const CW& w, const Act& x, const Act& y, const ConvOpt& o = ConvOpt()) {
    stzs_conv_args a = conv_base();
    conv_weights(a, *w.w, w.b ? (const float*)w.b->data : nullptr, w.Co, w.Ci, w.ks, 0, w.form);
    a.x = x.ptr();
    a.y = y.ptr();
    a.ldx = x.ld;
    a.bsx = x.bs;
    a.ldy = y.ld;
    a.bsy = y.bs;
    a.B = x.B;
    a.T_in = x.T;
    a.dil = o.dil;
    a.stride = o.stride;
    a.pad = o.pad;
    a.T_out = o.T_out >= 0 ? o.T_out : (x.T + 2 * o.pad - o.dil * (w.ks - 1) - 1) / o.stride + 1;
    a.in_dtype = x.dt;
    a.out_dtype = y.dt;
    if (o.pro) {
        a.pro_mode = STZS_PRO_ADAIN;
        a.pro_mean = o.pro->st.mean;
        a.pro_rstd = o.pro->st.rstd;
        a.stat_bs = o.pro->st.stat_bs;
        a.pro_gb = o.pro->gb;
        a.gb_bs = o.pro->gb_bs;
        a.gb_beta_off = o.pro->beta_off;
    }
    a.pro_act = o.pro_act;
    a.pro_slope = o.pro_slope;
    a.pro_cscale = o.cscale;
    if (o.res) {
        a.res = o.res->ptr();
        a.ldr = o.res->ld;
        a.bsr = (o.res->B > 1 || o.res->B == y.B) ? o.res->bs : 0;
    }
    a.res_tdiv = o.res_tdiv;
    if (o.acc) {
        a.acc_in = o.acc->ptr();
        a.lda = o.acc->ld;
        a.bsa = o.acc->bs;
    }
    a.gate = o.gate;
    a.gate_bs = o.gate_bs;
    a.alpha = o.alpha;
    a.beta = o.beta;
    a.epi_act = o.epi_act;
    a.epi_slope = o.epi_slope;
    if (w.ks == 1 && o.stride == 1 && o.pad == 0 && !o.pro && o.pro_act == STZS_ACT_NONE && o.cscale == 1.f &&
        (x.dt == STZS_BF16 || x.dt == STZS_F8) && x.c0 + a.ci_pad <= x.ld && a.T_out == x.T && w.form == STZS_PACK_KSTEP)
        a.flags |= STZS_CONV_A_DMA;
    if (o.rows && rows_ok(a.ci_pad) && w.ks == 1 && w.form == STZS_PACK_KSTEP && !o.pro && !o.stats_out &&
        (x.dt == STZS_F32 || (x.dt == STZS_BF16 && o.cscale == 1.f)) && x.c0 + a.ci_pad <= x.ld && a.T_out == x.T)
        a.flags = (a.flags & ~STZS_CONV_A_DMA) | STZS_CONV_ROWS;
    float* slab = nullptr;
    int Cc = 0;
    if (o.stats_out) {
        Cc = rup(w.Co, 8);
        const int ntile = (a.T_out + STZS_CONV_STAT_ROWS - 1) / STZS_CONV_STAT_ROWS;
        slab = c.f32((size_t)y.B * ntile * Cc * 2);
        a.stat_part = slab;
        a.stat_ld = Cc;
        o.stats_out->mean = c.f32((size_t)y.B * Cc);
        o.stats_out->rstd = c.f32((size_t)y.B * Cc);
        o.stats_out->stat_bs = Cc;
    }
    if (c.dry) return STZS_OK;
    CK(stzs_conv1d(&a, c.stream));
    if (!o.stats_out) return STZS_OK;
    stzs_stats_args s;
    memset(&s, 0, sizeof s);
    s.mean = o.stats_out->mean;
    s.rstd = o.stats_out->rstd;
    s.partial = slab;
    s.stat_bs = Cc;
    s.B = y.B;
    s.T = a.T_out;
    s.C = Cc;
    s.eps = 1e-5f;
    return stzs_chan_stats_final(&s, STZS_CONV_STAT_ROWS, c.stream);
}

int mean_rows(Ctx& c, const stzs_tensor_t& x, int c0, int C, float*& y) {
    y = c.f32((size_t)x.shape[0] * C);
    if (c.dry) return STZS_OK;
    return stzs_mean_rows((const float*)x.data, y, (int)x.shape[0], (int)x.shape[1], x.stride[1], x.stride[0], c0, C, C,
                          c.stream);
}

int copy2d(Ctx& c, const void* x, int64_t ldx, int64_t bsx, int in_dt, void* y, int64_t ldy, int64_t bsy, int out_dt,
           int B, int R, int C) {
    if (c.dry) return STZS_OK;
    stzs_copy_args a;
    memset(&a, 0, sizeof a);
    a.x = x;
    a.y = y;
    a.ldx = ldx;
    a.bsx = bsx;
    a.ldy = ldy;
    a.bsy = bsy;
    a.B = B;
    a.R = R;
    a.C = C;
    a.in_dtype = in_dt;
    a.out_dtype = out_dt;
    return stzs_copy2d(&a, c.stream);
}

// AdainResBlk1d (stzs/engine.py blk): out = (conv2(lrelu(AdaIN2(conv1(up(lrelu(AdaIN1(x))))))) + sc(x)) / sqrt 2
struct BlkIn {
    const stzs_tensor_t* t;  // 7 tensors: conv1 w, conv1 b, conv2 w, conv2 b, sc w (data NULL: none), pool w, pool b
    int din, dout;
    bool up;
};
int blk(Ctx& c, const BlkIn& bw, const Act& x, const Act& out, const float* gb, int64_t gbs, int off1, int off2) {
    const int B = x.B, T = x.T, dt = x.dt;
    Stats s1, s2;
    CK(stats(c, x, s1));
    const int To = bw.up ? 2 * T : T;
    Act r;
    CK(c.act(r, B, To, bw.dout, dt));
    const CW c1{&bw.t[0], &bw.t[1], bw.dout, bw.din, 3, blk_form(bw.dout, bw.din)};
    const CW c2{&bw.t[2], &bw.t[3], bw.dout, bw.dout, 3, blk_form(bw.dout, bw.dout)};
    if (bw.up) {
        Act u;
        CK(c.act(u, B, To, bw.din, dt));
        if (!c.dry) {
            stzs_dwup_args d;
            memset(&d, 0, sizeof d);
            d.x = x.ptr();
            d.y = u.ptr();
            d.mean = s1.mean;
            d.rstd = s1.rstd;
            d.gb = gb + off1;
            d.w = (const float*)bw.t[5].data;
            d.wb = (const float*)bw.t[6].data;
            d.ldx = x.ld;
            d.bsx = x.bs;
            d.ldy = u.ld;
            d.bsy = u.bs;
            d.stat_bs = s1.stat_bs;
            d.gb_bs = gbs;
            d.gb_beta_off = bw.din;
            d.B = B;
            d.T = T;
            d.C = bw.din;
            d.slope = 0.2f;
            d.dtype = dt;
            CK(stzs_adain_dwup(&d, c.stream));
        }
        ConvOpt o;
        o.pad = 1;
        o.stats_out = &s2;
        CK(conv(c, c1, u, r, o));
    } else {
        const Pro p1{s1, gb + off1, gbs, bw.din};
        ConvOpt o;
        o.pad = 1;
        o.pro = &p1;
        o.pro_act = STZS_ACT_LEAKY;
        o.pro_slope = 0.2f;
        o.stats_out = &s2;
        CK(conv(c, c1, x, r, o));
    }
    Act res = x;
    if (bw.t[4].data) {
        Act scb;
        CK(c.act(scb, B, T, bw.dout, dt));
        CK(conv(c, CW{&bw.t[4], nullptr, bw.dout, bw.din, 1, sc_form(bw.dout, bw.din)}, x, scb));
        res = scb;
    }
    const Pro p2{s2, gb + off2, gbs, bw.dout};
    ConvOpt o;
    o.pad = 1;
    o.pro = &p2;
    o.pro_act = STZS_ACT_LEAKY;
    o.pro_slope = 0.2f;
    o.res = &res;
    o.res_tdiv = bw.up ? 2 : 1;
    o.alpha = 1.f / sqrtf(2.f);
    return conv(c, c2, r, out, o);
}

// BiLSTM of the packed model (input projection on MFMA + the exchange recurrence), state reset on entry
int bilstm(Ctx& c, const Act& x, const stzs_tensor_t& wih, const stzs_tensor_t& bias, const stzs_tensor_t& whh, int H,
           const Act& y, uint32_t* status) {
    void* sync = c.take(4096);
    void* xchg = c.take(stzs_lstm_workspace(x.B, H, 2));
    Act gx;
    CK(c.act(gx, x.B, x.T, 8 * H, STZS_F32));
    CK(conv(c, CW{&wih, &bias, 8 * H, x.C, 1, STZS_PACK_KSTEP}, x, gx));
    if (c.dry) return STZS_OK;
    CK(stzs_lstm_state_reset(sync, xchg, c.stream));
    stzs_lstm_args l;
    memset(&l, 0, sizeof l);
    l.gx = (const float*)gx.ptr();
    l.whhT = whh.data;
    l.y = y.ptr();
    l.xchg = xchg;
    l.sync = sync;
    l.ldg = gx.ld;
    l.bsg = gx.bs;
    l.ldy = y.ld;
    l.bsy = y.bs;
    l.B = x.B;
    l.T = x.T;
    l.H = H;
    l.ndir = 2;
    l.status = status;
    return stzs_lstm(&l, c.stream);
}

// the AdaIN norm-group linear of a stage: gamma | beta of every norm from the pooled style vector
int norm_gb(Ctx& c, const stzs_tensor_t& w, const stzs_tensor_t& b, const float* pooled, int B, int style, int total,
            float*& gb) {
    gb = c.f32((size_t)B * total);
    Act x, y;
    x.base = (char*)pooled;
    x.B = B;
    x.T = 1;
    x.C = style;
    x.ld = style;
    x.bs = style;
    x.dt = STZS_F32;
    y.base = (char*)gb;
    y.B = B;
    y.T = 1;
    y.C = total;
    y.ld = total;
    y.bs = total;
    y.dt = STZS_F32;
    ConvOpt o;
    o.rows = true;
    return conv(c, CW{&w, &b, total, style, 1, STZS_PACK_KSTEP}, x, y, o);
}

// ---------------------------------------------------------------------------------------------- a2 denoiser_fwd
// sigma-embedding Fourier features, computed on the host exactly as stzs/engine.py fourier_features (float64 math,
// one rounding to fp32) and written by a kernel that takes them by value (graph-capturable, no host buffer)
struct Four {
    float v[256];
};
__global__ void four_kernel(const Four f, float* out, int n) {
    const int i = threadIdx.x;
    if (i < n) out[i] = f.v[i];
}

int denoiser(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t* out, int n_out, const stzs_params_t* p) {
    if (n_in < STZS_DN_NIN_BASE || n_out < 1) return STZS_EINVAL;
    const int cfg = p->i[0] != 0, NL = p->i[1], heads = p->i[2], d = p->i[3], ffn = p->i[4], nf = p->i[5];
    const float sigma = p->f[0], sd = p->f[1];
    if (NL <= 0 || heads <= 0 || d <= 0 || d % heads || ffn <= 0 || nf <= 0 || nf > 256 || nf % 2 || !(sigma > 0.f))
        return STZS_ESHAPE;
    if (n_in != STZS_DN_NIN_BASE + STZS_DN_PER_LAYER * NL) return STZS_EINVAL;
    const stzs_tensor_t &X = in[STZS_DN_X], &Ht = in[STZS_DN_HTXT], &Pm = in[STZS_DN_PROMPT], &D = out[0];
    if (X.dtype != STZS_F32 || X.ndim != 3 || !contiguous(X) || !act3(Ht, STZS_BF16) || Pm.dtype != STZS_F32 ||
        Pm.ndim != 3 || !contiguous(Pm) || D.dtype != STZS_F32 || !contiguous(D))
        return STZS_EDTYPE;
    const int R = (int)X.shape[0], Ls = (int)X.shape[1], cd = (int)X.shape[2];
    const int B = (int)Ht.shape[0], T = (int)Ht.shape[1], dtx = (int)Ht.shape[2];
    if (R != (cfg ? 2 * B : B) || Pm.shape[0] != B || Pm.shape[1] != Ls || Pm.shape[2] != cd || numel(D) != numel(X))
        return STZS_ESHAPE;
    for (int i = 0; i < n_in; ++i)
        if (!in[i].data && i != STZS_DN_CTX_NULL && i != STZS_DN_POOL_NULL) return STZS_EINVAL;
    if (cfg && (!in[STZS_DN_CTX_NULL].data || !in[STZS_DN_POOL_NULL].data)) return STZS_EINVAL;
    const int Lc = T + Ls;
    auto W = [&](int wi, int Co, int Ci) { return CW{&in[wi], &in[wi + 1], Co, Ci, 1, STZS_PACK_KSTEP}; };
    // ---- step-invariant context (denoiser_prepare, one sigma) ----
    Act ctx;
    CK(c.act(ctx, R, Lc, d, STZS_BF16, true));
    Act ht = act_of(Ht);
    auto rows_of = [&](const Act& base, int b0, int nb, int t0, int C) {  // rows [t0, ...) of utterances [b0, b0 + nb)
        Act y = base;
        y.base = base.base + ((size_t)b0 * base.bs + (size_t)t0 * base.ld) * esz(base.dt);
        y.B = nb;
        y.C = C;
        return y;
    };
    ConvOpt oT;
    oT.T_out = T;
    CK(conv(c, W(STZS_DN_CTX_TXT_W, d, dtx), ht, rows_of(ctx, 0, B, 0, d), oT));
    Act pa;
    pa.base = (char*)Pm.data;
    pa.B = B;
    pa.T = Ls;
    pa.C = cd;
    pa.ld = cd;
    pa.bs = (int64_t)Ls * cd;
    pa.dt = STZS_F32;
    ConvOpt oP;
    oP.T_out = Ls;
    CK(conv(c, W(STZS_DN_CTX_PRM_W, d, cd), pa, rows_of(ctx, 0, B, T, d), oP));
    if (cfg) {
        CK(conv(c, W(STZS_DN_CTX_TXT_W, d, dtx), ht, rows_of(ctx, B, B, 0, d), oT));
        Act dst = rows_of(ctx, B, B, T, d);
        CK(copy2d(c, in[STZS_DN_CTX_NULL].data, d, 0, STZS_BF16, dst.ptr(), ctx.ld, ctx.bs, STZS_BF16, B, Ls, d));
    }
    float* pm;
    CK(mean_rows(c, Pm, 0, cd, pm));
    float* pool = c.f32((size_t)R * d);
    {
        Act x, y;
        x.base = (char*)pm;
        x.B = B;
        x.T = 1;
        x.C = cd;
        x.ld = cd;
        x.bs = cd;
        x.dt = STZS_F32;
        y.base = (char*)pool;
        y.B = B;
        y.T = 1;
        y.C = d;
        y.ld = d;
        y.bs = d;
        y.dt = STZS_F32;
        ConvOpt o;
        o.rows = true;
        CK(conv(c, W(STZS_DN_POOL_W, d, cd), x, y, o));
        if (cfg) CK(copy2d(c, in[STZS_DN_POOL_NULL].data, d, 0, STZS_F32, pool + (size_t)B * d, d, d, STZS_F32, B, 1, d));
    }
    Act kv[16];
    if (NL > 16) return STZS_ESHAPE;
    for (int l = 0; l < NL; ++l) {
        CK(c.act(kv[l], R, Lc, 2 * d, STZS_BF16));
        CK(conv(c, W(STZS_DN_NIN_BASE + STZS_DN_PER_LAYER * l + STZS_DN_L_KV_W, 2 * d, d), ctx, kv[l]));
    }
    // sigma embedding: EDM c_noise = log(sigma) / 4 -> Fourier features -> MLP (SiLU) -> temb
    const double sg = (double)sigma;
    const double c_in = 1.0 / sqrt(sg * sg + (double)sd * sd), c_skip = (double)sd * sd / (sg * sg + (double)sd * sd),
                 c_out = sg * sd / sqrt(sg * sg + (double)sd * sd), c_noise = log(sg) / 4.0;
    Act four, t0, temb;
    CK(c.act(four, 1, 1, nf, STZS_F32));
    CK(c.act(t0, 1, 1, d, STZS_F32));
    CK(c.act(temb, 1, 1, d, STZS_F32));
    if (!c.dry) {
        Four f;
        const int half = nf / 2;
        for (int j = 0; j < half; ++j) {
            const double fr = exp(-log(10000.0) * (double)j / (double)half);
            const double arg = 1000.0 * c_noise * fr;
            f.v[j] = (float)cos(arg);
            f.v[half + j] = (float)sin(arg);
        }
        hipLaunchKernelGGL(four_kernel, dim3(1), dim3(256), 0, reinterpret_cast<hipStream_t>(c.stream), f,
                           (float*)four.ptr(), nf);
        if (hipGetLastError() != hipSuccess) return STZS_EHIP;
    }
    {
        ConvOpt o;
        o.epi_act = STZS_ACT_SILU;
        o.rows = true;
        CK(conv(c, W(STZS_DN_T0_W, d, nf), four, t0, o));
        ConvOpt o1;
        o1.rows = true;
        CK(conv(c, W(STZS_DN_T1_W, d, d), t0, temb, o1));
    }
    Act cb, mod, fmod;
    CK(c.act(cb, R, 1, d, STZS_BF16));
    CK(c.act(mod, R, 1, 6 * d, STZS_F32));
    CK(c.act(fmod, R, 1, 2 * d, STZS_F32));
    float* modx = c.f32((size_t)NL * R * 6 * d);
    float* fmodx = c.f32((size_t)R * 2 * d);
    if (!c.dry) CK(stzs_dn_cond_steps(pool, (const float*)temb.ptr(), cb.ptr(), R, d, 1, c.stream));
    {
        Act cbr = cb, modr = mod, fmodr = fmod;  // [R, 1, C] -> the engine's [R rows, 1] views
        CK(conv(c, W(STZS_DN_ADA_W, 6 * d, d), cbr, modr));
        CK(conv(c, W(STZS_DN_FINAL_ADA_W, 2 * d, d), cbr, fmodr));
    }
    if (!c.dry) {
        CK(stzs_adaln_expand((const float*)mod.ptr(), (const float*)in[STZS_DN_ADA_TABLE].data, modx, R, d, 6, NL,
                             0b010010u, c.stream));
        CK(stzs_adaln_expand((const float*)fmod.ptr(), nullptr, fmodx, R, d, 2, 1, 0b10u, c.stream));
    }
    // ---- one NFE (denoiser_step) ----
    Act h, an, qkv, o, q, ff;
    CK(c.act(h, R, Ls, d, STZS_F32));
    CK(c.act(an, R, Ls, d, STZS_BF16));
    CK(c.act(qkv, R, Ls, 3 * d, STZS_BF16));
    CK(c.act(o, R, Ls, d, STZS_BF16));
    CK(c.act(q, R, Ls, d, STZS_BF16));
    CK(c.act(ff, R, Ls, ffn, STZS_BF16));
    Act xa;
    xa.base = (char*)X.data;
    xa.B = R;
    xa.T = Ls;
    xa.C = cd;
    xa.ld = cd;
    xa.bs = (int64_t)Ls * cd;
    xa.dt = STZS_F32;
    Act pos;
    pos.base = (char*)in[STZS_DN_POS].data;
    pos.B = 1;
    pos.T = Ls;
    pos.C = d;
    pos.ld = d;
    pos.bs = (int64_t)Ls * d;
    pos.dt = STZS_F32;
    {
        ConvOpt oi;
        oi.cscale = (float)c_in;
        oi.res = &pos;
        CK(conv(c, W(STZS_DN_IN_W, d, cd), xa, h, oi));
    }
    auto ln = [&](const float* G, int64_t gs, const float* Bt, int64_t bs, int gdiv) -> int {
        if (c.dry) return STZS_OK;
        stzs_rowln_args a;
        memset(&a, 0, sizeof a);
        a.x = h.ptr();
        a.y = an.ptr();
        a.G = G;
        a.Bt = Bt;
        a.ldx = h.ld;
        a.ldy = an.ld;
        a.gs = gs;
        a.bs = bs;
        a.R = R * Ls;
        a.C = d;
        a.gdiv = gdiv;
        a.in_dtype = STZS_F32;
        a.out_dtype = STZS_BF16;
        a.act = STZS_ACT_NONE;
        a.gadd = 0.f;
        a.eps = 1e-5f;
        return stzs_row_layernorm(&a, c.stream);
    };
    auto attn = [&](const Act& qa, const Act& ka, const Act& va, const Act& oa) -> int {
        if (c.dry) return STZS_OK;
        stzs_attn_args a;
        memset(&a, 0, sizeof a);
        a.q = qa.ptr();
        a.k = ka.ptr();
        a.v = va.ptr();
        a.o = oa.ptr();
        a.ldq = qa.ld;
        a.ldk = ka.ld;
        a.ldv = va.ld;
        a.ldo = oa.ld;
        a.bsq = qa.bs;
        a.bsk = ka.bs;
        a.bsv = va.bs;
        a.bso = oa.bs;
        a.R = qa.B;
        a.Lq = qa.T;
        a.Lk = ka.T;
        a.heads = heads;
        a.dh = d / heads;
        return stzs_attention(&a, c.stream);
    };
    CK(ln(modx + d, 6 * d, modx, 6 * d, Ls));  // layer 0's adaLN-modulated LayerNorm 1
    for (int l = 0; l < NL; ++l) {
        const int base = STZS_DN_NIN_BASE + STZS_DN_PER_LAYER * l;
        const float* mb = modx + (size_t)l * R * 6 * d;
        CK(conv(c, W(base + STZS_DN_L_QKV_W, 3 * d, d), an, qkv));
        CK(attn(qkv.sl(0, d), qkv.sl(d, d), qkv.sl(2 * d, d), o));
        ConvOpt oo;
        oo.res = &h;
        oo.gate = mb + 2 * d;
        oo.gate_bs = 6 * d;
        CK(conv(c, W(base + STZS_DN_L_O_W, d, d), o, h, oo));
        CK(ln((const float*)in[base + STZS_DN_L_LN_G].data, 0, (const float*)in[base + STZS_DN_L_LN_B].data, 0, 1));
        CK(conv(c, W(base + STZS_DN_L_Q_W, d, d), an, q));
        CK(attn(q, kv[l].sl(0, d), kv[l].sl(d, d), o));
        ConvOpt oc;
        oc.res = &h;
        CK(conv(c, W(base + STZS_DN_L_CO_W, d, d), o, h, oc));
        CK(ln(mb + 4 * d, 6 * d, mb + 3 * d, 6 * d, Ls));
        ConvOpt of;
        of.epi_act = STZS_ACT_GELU;
        CK(conv(c, W(base + STZS_DN_L_FF1_W, ffn, d), an, ff, of));
        ConvOpt o2;
        o2.res = &h;
        o2.gate = mb + 5 * d;
        o2.gate_bs = 6 * d;
        CK(conv(c, W(base + STZS_DN_L_FF2_W, d, ffn), ff, h, o2));
        if (l + 1 < NL) {
            const float* mn = modx + (size_t)(l + 1) * R * 6 * d;
            CK(ln(mn + d, 6 * d, mn, 6 * d, Ls));
        } else {
            CK(ln(fmodx + d, 2 * d, fmodx, 2 * d, Ls));  // the final adaLN
        }
    }
    Act Dy;
    Dy.base = (char*)D.data;
    Dy.B = R;
    Dy.T = Ls;
    Dy.C = cd;
    Dy.ld = cd;
    Dy.bs = (int64_t)Ls * cd;
    Dy.dt = STZS_F32;
    ConvOpt ot;
    ot.alpha = (float)c_out;
    ot.acc = &xa;
    ot.beta = (float)c_skip;
    return conv(c, W(STZS_DN_OUT_W, cd, d), an, Dy, ot);
}

// ---------------------------------------------------------------------------------------------- a9 decoder_pre
int decoder_pre(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t* out, int n_out, const stzs_params_t* p) {
    if (n_in != STZS_DP_NIN || n_out < 1) return STZS_EINVAL;
    const int denc = p->i[0], dres = p->i[1], dout = p->i[2], sty = p->i[3], total = p->i[4];
    const stzs_tensor_t &Asr = in[STZS_DP_ASR], &F0 = in[STZS_DP_F0], &Nn = in[STZS_DP_N], &Cd = in[STZS_DP_CODES];
    if (!act3(Asr, STZS_BF16) || F0.dtype != STZS_F32 || Nn.dtype != STZS_F32 || Cd.dtype != STZS_F32 ||
        !act3(out[0], STZS_BF16))
        return STZS_EDTYPE;
    const int B = (int)Asr.shape[0], T40 = (int)Asr.shape[1], dtx = (int)Asr.shape[2], T80 = 2 * T40;
    if (denc <= 0 || dres <= 0 || dout <= 0 || sty <= 0 || sty > Cd.shape[2] || F0.ndim != 2 || F0.shape[0] != B ||
        F0.shape[1] != T80 || F0.stride[1] != 1 || Nn.ndim != 2 || Nn.shape[0] != B || Nn.shape[1] != T80 ||
        Nn.stride[1] != 1 || Nn.stride[0] != F0.stride[0] || Cd.shape[0] != B || Cd.ndim != 3 ||
        out[0].shape[0] != B || out[0].shape[1] != T80 || out[0].shape[2] < dout)
        return STZS_ESHAPE;
    for (int i = 0; i < n_in; ++i)  // the sc / pool tensors of a block may be absent (data NULL)
        if (!in[i].data && !(i >= STZS_DP_BLK0 && (i - STZS_DP_BLK0) % 7 >= 4)) return STZS_EINVAL;
    const int dcat = denc + 2 + dres;
    // per block (encode, decode0..3): din, dout, up; the norm group holds norm1 (2 din), norm2 (2 dout) of each
    const int din_[5] = {dtx + 2, dcat, dcat, dcat, dcat}, dout_[5] = {denc, denc, denc, denc, dout};
    int off[5][2], o_ = 0;
    for (int j = 0; j < 5; ++j) {
        off[j][0] = o_;
        o_ += 2 * din_[j];
        off[j][1] = o_;
        o_ += 2 * dout_[j];
    }
    if (total < o_) return STZS_ESHAPE;
    float* sa;
    CK(mean_rows(c, Cd, 0, sty, sa));
    float* gb;
    CK(norm_gb(c, in[STZS_DP_NORM_W], in[STZS_DP_NORM_B], sa, B, sty, total, gb));
    Act enc;
    CK(c.act(enc, B, T40, dtx + 2, STZS_BF16, true));
    CK(copy2d(c, Asr.data, Asr.stride[1], Asr.stride[0], STZS_BF16, enc.ptr(), enc.ld, enc.bs, STZS_BF16, B, T40, dtx));
    Act cats[2];
    CK(c.act(cats[0], B, T40, dcat, STZS_BF16, true));
    CK(c.act(cats[1], B, T40, dcat, STZS_BF16, true));
    const int cF = denc + dres, cN = cF + 1;
    for (int j = 0; j < 2; ++j) {
        if (!c.dry) {
            stzs_f0n_args a;
            memset(&a, 0, sizeof a);
            a.f0 = (const float*)F0.data;
            a.n = (const float*)Nn.data;
            a.wf = (const float*)in[STZS_DP_F0CONV].data;
            a.wn = (const float*)in[STZS_DP_NCONV].data;
            a.y0 = cats[j].ptr();
            a.y1 = j == 0 ? enc.ptr() : nullptr;
            a.ldf = F0.stride[0];
            a.ldy0 = cats[j].ld;
            a.bsy0 = cats[j].bs;
            a.ldy1 = enc.ld;
            a.bsy1 = enc.bs;
            a.B = B;
            a.T80 = T80;
            a.cf0 = cF;
            a.cn0 = cN;
            a.cf1 = dtx;
            a.cn1 = dtx + 1;
            a.dtype = STZS_BF16;
            CK(stzs_f0n_down(&a, c.stream));
        }
        CK(conv(c, CW{&in[STZS_DP_ASR_RES_W], &in[STZS_DP_ASR_RES_W + 1], dres, dtx, 1, STZS_PACK_KSTEP},
                enc.sl(0, dtx), cats[j].sl(denc, dres)));
    }
    auto bk = [&](int j) { return BlkIn{in + STZS_DP_BLK0 + 7 * j, din_[j], dout_[j], j == 4}; };
    CK(blk(c, bk(0), enc.sl(0, dtx + 2), cats[0].sl(0, denc), gb, total, off[0][0], off[0][1]));
    int src = 0;
    for (int i = 1; i <= 3; ++i) {
        CK(blk(c, bk(i), cats[src].sl(0, dcat), cats[1 - src].sl(0, denc), gb, total, off[i][0], off[i][1]));
        src = 1 - src;
    }
    Act g = act_of(out[0]);
    g.C = dout;
    return blk(c, bk(4), cats[src].sl(0, dcat), g, gb, total, off[4][0], off[4][1]);
}

// ---------------------------------------------------------------------------------------------- a8 f0n_predictor
int f0n(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t* out, int n_out, const stzs_params_t* p) {
    if (n_in != STZS_FN_NIN || n_out < 2) return STZS_EINVAL;
    const int H = p->i[0], c0 = p->i[1], c1 = p->i[2], c2 = p->i[3], sc0 = p->i[4], spr = p->i[5], total = p->i[6];
    const stzs_tensor_t &En = in[STZS_FN_EN], &Cd = in[STZS_FN_CODES];
    if (!act3(En, STZS_BF16) || Cd.dtype != STZS_F32 || out[0].dtype != STZS_F32 || out[1].dtype != STZS_F32)
        return STZS_EDTYPE;
    const int B = (int)En.shape[0], T40 = (int)En.shape[1], T80 = 2 * T40;
    if (H <= 0 || c0 <= 0 || c1 <= 0 || c2 <= 0 || spr <= 0 || Cd.ndim != 3 || Cd.shape[0] != B ||
        sc0 + spr > Cd.shape[2] || out[0].ndim != 2 || out[0].shape[0] != B || out[0].shape[1] != T80 ||
        !contiguous(out[0]) || out[1].ndim != 2 || out[1].shape[0] != B || out[1].shape[1] != T80 || !contiguous(out[1]))
        return STZS_ESHAPE;
    for (int i = 0; i < n_in; ++i) {
        const int r = (i - STZS_FN_BR0) % STZS_FN_PER_BRANCH;
        const bool optional = i >= STZS_FN_BR0 && r < 21 && (r % 7 >= 4);  // sc / pool tensors
        if (!in[i].data && !optional) return STZS_EINVAL;
    }
    uint32_t* status = (n_out > 2 && out[2].data) ? (uint32_t*)out[2].data : nullptr;
    const int hid = 2 * H;
    Act xs;
    CK(c.act(xs, B, T40, hid, STZS_BF16));
    CK(bilstm(c, act_of(En), in[STZS_FN_LSTM_IH], in[STZS_FN_LSTM_BIAS], in[STZS_FN_LSTM_WHH], H, xs, status));
    float* sg;
    CK(mean_rows(c, Cd, sc0, spr, sg));
    float* gb;
    CK(norm_gb(c, in[STZS_FN_NORM_W], in[STZS_FN_NORM_B], sg, B, spr, total, gb));
    const int din_[3] = {hid, c0, c1}, dout_[3] = {c0, c1, c2};
    int o_ = 0;
    for (int br = 0; br < 2; ++br) {
        const stzs_tensor_t* bt = in + STZS_FN_BR0 + STZS_FN_PER_BRANCH * br;
        Act y[3];
        CK(c.act(y[0], B, T40, c0, STZS_BF16));
        CK(c.act(y[1], B, T80, c1, STZS_BF16));
        CK(c.act(y[2], B, T80, c2, STZS_BF16));
        Act x = xs;
        for (int j = 0; j < 3; ++j) {
            const int off1 = o_, off2 = o_ + 2 * din_[j];
            o_ += 2 * din_[j] + 2 * dout_[j];
            CK(blk(c, BlkIn{bt + 7 * j, din_[j], dout_[j], j == 1}, x, y[j], gb, total, off1, off2));
            x = y[j];
        }
        Act f;
        f.base = (char*)out[br].data;
        f.B = B;
        f.T = T80;
        f.C = 1;
        f.ld = 1;
        f.bs = out[br].stride[0];
        f.dt = STZS_F32;
        CK(conv(c, CW{&bt[21], &bt[22], 1, c2, 1, STZS_PACK_KSTEP}, y[2], f));
    }
    return o_ > total ? STZS_ESHAPE : STZS_OK;
}

template <typename F>
int run(F fn, const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
        void* workspace, size_t ws_bytes, void* stream) {
    if (!inputs || !outputs || !p) return STZS_EINVAL;
    {  // the dry pass sizes the workspace and checks every argument before anything is launched
        Ctx dry(nullptr, true, stream);
        CK(fn(dry, inputs, n_in, outputs, n_out, p));
        if (!workspace || ws_bytes < dry.used()) return STZS_ESHAPE;
    }
    Ctx c(workspace, false, stream);
    return fn(c, inputs, n_in, outputs, n_out, p);
}

}  // namespace

// The workspace queries run the operator's dry pass over the inputs alone (outputs do not change the carve).
namespace {
int dn_q(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t*, int, const stzs_params_t* p) {
    // mirror of denoiser() without output checks: the carve depends on inputs and params only
    stzs_tensor_t D;
    memset(&D, 0, sizeof D);
    D = in[STZS_DN_X];
    return denoiser(c, in, n_in, &D, 1, p);
}
int dp_q(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t*, int, const stzs_params_t* p) {
    stzs_tensor_t g;
    memset(&g, 0, sizeof g);
    g.dtype = STZS_BF16;
    g.ndim = 3;
    g.shape[0] = in[STZS_DP_ASR].shape[0];
    g.shape[1] = 2 * in[STZS_DP_ASR].shape[1];
    g.shape[2] = p->i[2];
    g.stride[2] = 1;
    g.stride[1] = g.shape[2];
    g.stride[0] = g.shape[1] * g.shape[2];
    g.data = (void*)16;  // never dereferenced by the dry pass
    return decoder_pre(c, in, n_in, &g, 1, p);
}
int fn_q(Ctx& c, const stzs_tensor_t* in, int n_in, stzs_tensor_t*, int, const stzs_params_t* p) {
    stzs_tensor_t o[2];
    memset(o, 0, sizeof o);
    for (int k = 0; k < 2; ++k) {
        o[k].dtype = STZS_F32;
        o[k].ndim = 2;
        o[k].shape[0] = in[STZS_FN_EN].shape[0];
        o[k].shape[1] = 2 * in[STZS_FN_EN].shape[1];
        o[k].stride[1] = 1;
        o[k].stride[0] = o[k].shape[1];
        o[k].data = (void*)16;
    }
    return f0n(c, in, n_in, o, 2, p);
}
}  // namespace

extern "C" size_t stzs_denoiser_fwd_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || !p || n_in < STZS_DN_NIN_BASE) return 0;
    Ctx dry(nullptr, true, nullptr);
    return dn_q(dry, inputs, n_in, nullptr, 0, p) == STZS_OK ? dry.used() : 0;
}
extern "C" int stzs_denoiser_fwd(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                                 const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream) {
    return run(denoiser, inputs, n_in, outputs, n_out, p, workspace, ws_bytes, stream);
}
extern "C" size_t stzs_decoder_pre_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || !p || n_in != STZS_DP_NIN) return 0;
    Ctx dry(nullptr, true, nullptr);
    return dp_q(dry, inputs, n_in, nullptr, 0, p) == STZS_OK ? dry.used() : 0;
}
extern "C" int stzs_decoder_pre(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                                const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream) {
    return run(decoder_pre, inputs, n_in, outputs, n_out, p, workspace, ws_bytes, stream);
}
extern "C" size_t stzs_f0n_predictor_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p) {
    if (!inputs || !p || n_in != STZS_FN_NIN) return 0;
    Ctx dry(nullptr, true, nullptr);
    return fn_q(dry, inputs, n_in, nullptr, 0, p) == STZS_OK ? dry.used() : 0;
}
extern "C" int stzs_f0n_predictor(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                                  const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream) {
    return run(f0n, inputs, n_in, outputs, n_out, p, workspace, ws_bytes, stream);
}
