/*
 * libstzs_hip.so — C-ABI of the MI355X-native StyleTTS-ZS synthesis hot path (gfx950).
 *
 * The upstream reference exposes NO interface for this path: `/root/reference/README.md:15-16`
 * reads "## Inference / ### Under construction".  The entry points below are the operator
 * boundary pinned by SURVEY.md §8(b) (L1 "torch ops" -> this C-ABI), one per hot-path function
 * of SURVEY.md §8(a); each declaration names the row it implements.  INTEGRATION.md shows the
 * ctypes binding (stzs/_lib.py) a maintainer would add on the reference side.
 *
 * Contract:
 *   - plain pointers + element strides, no framework types; every tensor is caller-owned device
 *     memory (the library never allocates on the hot path);
 *   - channels-last ("NTC") activations: element (b, t, c) at b*bs + t*ld + c;
 *   - every call is asynchronous on `stream` (a hipStream_t passed as void*), never syncs the
 *     host, and is safe to capture into a hipGraph;
 *   - returns STZS_OK (0) or a negative code; no exception crosses the ABI; stzs_strerror()
 *     names it.  Shape/dtype violations are rejected before any launch.
 */
#ifndef STZS_H
#define STZS_H

#include <stddef.h>
#include <stdint.h>

#ifdef __cplusplus
extern "C" {
#endif

#define STZS_OK 0
#define STZS_EINVAL (-1)  /* null pointer / bad enum / misaligned */
#define STZS_ESHAPE (-2)  /* shape or stride violation */
#define STZS_EDTYPE (-3)  /* unsupported dtype combination */
#define STZS_EHIP (-4)    /* HIP runtime error on launch */

enum { STZS_F32 = 0, STZS_BF16 = 1, STZS_I32 = 2, STZS_F8 = 3 /* OCP e4m3fn (gfx950), with a row scale */ };
enum { STZS_ACT_NONE = 0, STZS_ACT_LEAKY = 1, STZS_ACT_SNAKE = 2, STZS_ACT_GELU = 3, STZS_ACT_SILU = 4 };
enum { STZS_PRO_NONE = 0, STZS_PRO_ADAIN = 1 };
/* stzs_conv_args.flags: the caller guarantees that for a ks=1 bf16 linear every input row can be
 * read over [0, ci_pad) channels (row padding inside the buffer) -> A streams by LDS-DMA */
#define STZS_CONV_A_DMA 8

/* ---- library ---- */
int stzs_init(int device);
const char* stzs_strerror(int code);
int stzs_version(void);

/* ---- §8(a) a2/a9/a11/a12/a13-conv: the universal MFMA conv1d / linear -------------------
 * y[b, t, co] = epi( sum_{k, ci} W[k, co, ci] * pro(x)[b, t*stride + k*dil - pad, ci] )
 *   pro(x) = act_pro(x * sc[b,ci] + sh[b,ci]);  NONE: sc = pro_cscale, sh = 0;
 *            ADAIN: sc = (1 + gamma) * rstd, sh = beta - mean * sc   (AdaIN1d, InstanceNorm)
 *   epi(v) = ((act_epi(v + bias) * gate[b,co] + res[b, t/res_tdiv, co]) * alpha) + beta * acc_in
 * Weights are pre-packed bf16 [ks][co_pad][ci_pad] (stzs/weights.py).  ups > 0 selects the
 * polyphase ConvTranspose1d form (ks = 2, pad = 1, co = ups * Co): output row q, phase p lands at
 * t = q*ups + p - ups_pad (+refl, with row 1 mirrored to row 0 for ReflectionPad(1,0)).
 * Replaces: the decoder/predictor convs and every denoiser linear (SURVEY §8(a) a2,a9,a11,a12). */
typedef struct stzs_conv_args {
    const void* x;
    const void* w;
    const float* bias;
    void* y;
    const void* res;
    const void* acc_in;
    const float* gate;
    const float* pro_mean;
    const float* pro_rstd;
    const float* pro_gb;
    const float* pro_alpha;
    int64_t ldx, bsx, ldy, bsy, ldr, bsr, lda, bsa;
    int64_t gate_bs, stat_bs, gb_bs, gb_beta_off;
    int32_t B, T_in, T_out, Ci, Co, ks, dil, stride, pad;
    int32_t ci_pad, co_pad, cic;
    int32_t ups, ups_pad, T_final, refl, res_tdiv;
    int32_t in_dtype, out_dtype;
    int32_t pro_mode, pro_act, epi_act, flags;
    float pro_cscale, pro_slope, epi_slope, alpha, beta, pad_f;
    /* optional fused InstanceNorm statistics of the STORED output (after rounding to out_dtype):
     * per (utterance b, STZS_CONV_STAT_ROWS-row chunk, channel c < Co) the fp32 (sum, sumsq) at
     * stat_part[((b * nch + chunk) * stat_ld + c) * 2 + {0,1}], nch = ceil(T_out / 64) -- the
     * partial layout of stzs_chan_stats; finish with stzs_chan_stats_final(chunk_rows = 64).
     * Plain (non-ConvTranspose, non-linear) convs only; NULL = off. */
    void* stat_part;
    int64_t stat_ld;
    /* fp8 linears (configs[4] denoiser, in_dtype = STZS_F8): x rows are e4m3fn codes with one fp32
     * scale per flat row (x_scale[b * T_in + t], e.g. from stzs_row_layernorm / stzs_quant_rows), the
     * weights an e4m3fn K-step stream [co_pad/128][ci_pad/64][128][64] (stzs/weights.py pack_conv_f8)
     * with one fp32 scale per output column (w_scale[co_pad]); acc * x_scale * w_scale enters the
     * usual epilogue.  Plain linears only (ks = 1, flags STZS_CONV_A_DMA); NULL otherwise. */
    const float* x_scale;
    const float* w_scale;
    /* in-launch split-K for bf16 linears (the LDS-DMA GEMM path: ks = 1, STZS_CONV_A_DMA, bf16 x, not fp8):
     * splitk in {0, 1} = off, {2, 4} = the ci_pad / 32 K-steps (a multiple of splitk) of every 64-row x
     * 128-column output tile are split over splitk workgroups (grid z).  Each writes its fp32 partial tile to
     * splitk_ws with write-through stores and takes a ticket on splitk_ctr[tile]; the last arriver reads the
     * splitk slabs back and sums them in slice order 0, 1, ... (the result depends neither on the arrival order
     * nor on the row count: batch-invariant) and runs the usual epilogue.  splitk_ws: 16-B aligned,
     * stzs_conv_splitk_workspace() bytes; splitk_ctr: one uint32 per tile, ZERO before the first launch (every
     * launch leaves them zero).  Used for the batch-1 denoiser linears, whose 8-32 output tiles would otherwise
     * stream all of K through 8-32 CUs (configs[1]).
     * Also on the generic bf16 conv (conv_mfma: k >= 1, no W_* / A_DMA / ROWS flag): splitk in 2..16 (at most the
     * chunk count) splits the n = ci_pad / cic input-channel chunks, slice z taking chunks [z n / splitk,
     * (z+1) n / splitk); each 128-row x 128-column tile (per utterance) sums its slices the same way (with one
     * chunk per slice, the DEEP form: a second launch splitk_epi combines the slices -- same output bits).  splitk_ws:
     * B * ceil(T_out / 128) * (co_pad / 128) * splitk * 65536 bytes, splitk_ctr: one zeroed uint32 per tile.  Used
     * for the batch-1 text-encoder k5 convs (4 tiles x 80 K-steps otherwise) and the batch-1 decoder / predictor
     * AdaIN-block convs (16 tiles x 108 K-steps for a decoder conv1). */
    void* splitk_ws;
    unsigned int* splitk_ctr;
    int32_t splitk;
    int32_t pad_sk;
    /* optional (the generic conv path only -- no STZS_CONV_W_* / A_DMA / ROWS flag): the AdaIN prologue's
     * statistics straight from InstanceNorm partials instead of pro_mean / pro_rstd.  When pro_part != NULL,
     * mean and rstd of (utterance b, channel c) are computed in the prologue from the fp32 (sum, sumsq) pairs
     * pro_part[((b * pro_nch + k) * pro_ld + c) * 2 + {0, 1}], k < pro_nch <= 8 (the layout of
     * stzs_chan_stats_partial and of the conv's own fused statistics), over pro_T input rows with pro_eps,
     * in fp64 in the order of stzs_chan_stats_final -- the same bits as finalising first (one launch less). */
    const float* pro_part;
    int64_t pro_ld;
    int32_t pro_nch, pro_T;
    float pro_eps, pad_pp;
} stzs_conv_args;
/* split-K workspace of a linear over `rows` flat rows: fp32 slab bytes; the tile (= counter) count is
 * bytes / (splitk * 32768).  0 for a bad argument. */
size_t stzs_conv_splitk_workspace(int64_t rows, int32_t co_pad, int32_t splitk);
#define STZS_CONV_STAT_ROWS 64
/* flags bit: weights packed with the 16-lane channel permutation of the MRF kernel (stzs/weights.py
 * pack_conv(lane16=True)): inside each 128-column tile, packed row wc*64 + nt*16 + g*4 + r holds
 * output channel wc*64 + g*16 + nt*4 + r.  Selects the MRF conv (csrc/mrf.hip): AdaIN + Snake / LeakyReLU
 * prologue, bf16 in/out, Ci % 128 == 0, Co % 16 == 0, stride 1, no gate/ups/epilogue activation. */
#define STZS_CONV_W_LANE16 16
/* flags bit: narrow weights (Co <= 32) packed as [NK][32][32] K-steps with packed row nt*16 + g*4 + r
 * holding output channel g*8 + nt*4 + r (stzs/weights.py pack_conv(narrow32=True)).  Selects the
 * narrow conv of csrc/mrf.hip: 128-channel chunks, bf16 in, fp32 out, LeakyReLU / identity prologue
 * (no AdaIN), bias, alpha; no residual / gate / statistics.  (conv_post: 128 -> 22 channels) */
#define STZS_CONV_W_NARROW32 32
/* flags bit: PRECISE (parity) mode -- fp32 weights packed [co_pad/128][ci_pad/32][ks][128 co][32 ci]
 * (stzs/weights.py kstep_stream_f32, cic = 32) and fp32 operands on v_mfma_f32_16x16x4_f32 (exact fp32
 * products, fp32 accumulate), libm-accurate prologue activations; bf16|f32 in, bf16|f32 out, every
 * conv feature except the fp8 path.  Used by StyleTTSZS(precise_decoder=True) to meet the north-star
 * mel-L1 <= 1e-3 on the decoder (bf16 weight rounding alone costs ~1.3e-2). */
#define STZS_CONV_W_F32 64
/* flags bit (diagnostic): keep the dispatcher's linear workgroup order on the LANE16 / NARROW32 kernels and the
 * LDS-DMA linear GEMM instead of the XCD-aware remap (neighbouring tiles on one L2); results are identical
 * either way. */
#define STZS_CONV_LINEAR_IDS 128
/* flags bit: weights packed in MFMA fragment order for the register-direct MRF conv (csrc/mrfv.hip,
 * stzs/weights.py pack_conv(frag32=True)): [co_pad/128][ci_pad/128][ks][4 k-steps][4 waves][2][64 lanes][8]
 * bf16, packed row w*32 + nt*16 + g*4 + r of a 128-column tile holding output channel w*32 + g*8 + nt*4 + r.
 * Same prologue / epilogue contract as STZS_CONV_W_LANE16 with ks in {3, 7, 11} (Snake) or ks = 3
 * (LeakyReLU / identity), Co % 8 == 0; bit-identical results, no weight ring and no K-loop barrier. */
#define STZS_CONV_W_FRAG32 256
/* (512: formerly STZS_CONV_MRF_PIPE, the persistent k3 MRF form of rounds 2-4 -- removed in round 5, no end-to-end
 * gain; the bit stays unused) */
/* flags: PRECISE split-operand form (csrc/conv.hip conv_x3).  w = two bf16 K-step streams (hi = bf16(w),
 * then lo = bf16(w - hi)), each [co_pad/128][ci_pad/32 * ks][128][32] in the STZS_PACK_KSTEP swizzle with
 * cic = 32 (stzs/weights.py kstep_stream_x3); activations are split the same way when staged, and every
 * product is ah*bh + ah*bl + al*bh on bf16 MFMA with fp32 accumulation (~fp32 accuracy at ~3x bf16 work).
 * Requires cic = 32; any in/out dtype; the accurate (libm) prologue activations. */
#define STZS_CONV_W_X3 1024
/* flags bit: SMALL-M linear on the whole chip (csrc/rows.hip; the batch-1 denoiser linears): bf16 (or fp32, scaled by
 * pro_cscale and rounded to bf16) x rows, STZS_PACK_KSTEP weights; every workgroup owns 16 output columns, all rows of
 * a 64/128-row block and 1/Z of K, operands loaded straight into MFMA fragments.  splitk = Z in {0, 1} (off) or any Z
 * with ci_pad / 32 = 4 Z {1, 2, 4, 8, 16}: the Z slices hand their fp32 partials to the tile's last arriver through
 * splitk_ws (stzs_conv_rows_workspace bytes: the larger of this layout and stzs_ln_linear's K-slice layout) and
 * splitk_ctr (one zeroed uint32 per tile, left zeroed).  Epilogue:
 * bias, epi_act NONE | GELU | SILU, FLAT gate, residual, alpha, beta * acc_in.  The per-element summation order depends on
 * K and Z only (batch-invariant).  Replaces gemm_glds for 100-row linears whose 8-32 tiles would stream all of K
 * through 8-32 CUs (SURVEY §8(a) a2 at B = 1). */
#define STZS_CONV_ROWS 2048
/* flags bit (with STZS_CONV_W_FRAG32 and ups > 0, refl in {0, 1}, Co % 128 == 0): the polyphase ConvTranspose with
 * the generator's 1x1 noise conv fused as ONE extra K-step per 128-column tile (stzs/weights.py pack_ups_noise):
 * res = the harmonic-source rows [B, T_final + refl, >= 32] bf16 (ldr / bsr; channels past the noise conv's input
 * width are zero), the weight stream holds (K-steps of the ConvTranspose + 1) per tile, bias = ConvTranspose bias +
 * noise bias, gate = the noise conv's weights fp32 [Co][32] (the ReflectionPad(1,0) row: its ConvTranspose value is
 * output row 2's, its noise term row 0's).  y[t] = convT(x)[t] + noise(har)[t] without the noise conv's output. */
#define STZS_CONV_UPS_NOISE 4096
/* flags bit (FRAG32 weights, Snake prologue, ci_pad > 128, co_pad % 256 == 0): keep the register-direct MRF conv at
 * 128 output channels per workgroup instead of its default wide form (256 per workgroup: every staged input row
 * transformed once per 256 channels instead of once per 128).  Bit-identical either way; an A/B switch. */
#define STZS_CONV_MRFV_NARROW 8192
/* flags: PRECISE register-direct form of the FRAG32 convs (csrc/mrfx.hip): the split-operand arithmetic of
 * STZS_CONV_W_X3 (w * z = wl * zh + wh * zl + wh * zh, fp32 accumulate) with the data movement of STZS_CONV_W_FRAG32.
 * w = per 32-wide K-step (loop order [co_pad/128][ci_pad/128][ks][4]) the hi then the lo fragment block
 * [2][4 waves][2][64 lanes][8] bf16 of the STZS_CONV_W_FRAG32 layout (same frag32 row permutation; stzs/weights.py
 * frag32x3_stream, STZS_PACK_FRAG32X3).  cic = 128, ks in {3, 7, 11} (Snake) or 3 (LeakyReLU / identity, no
 * accumulate input), stride 1, fp32 x / y / res / acc_in (32-B aligned rows), Co % 8 == 0; the InstanceNorm
 * statistics are those of the stored fp32 values. */
#define STZS_CONV_W_FRAG32X3 16384
/* flags bit (FRAG32 weights, Snake prologue): keep the register-direct MRF conv's 128-row time tiles where its
 * launcher would take 64-row tiles (grids of fewer than two 128-row tiles per CU, e.g. batch 1).  Bit-identical either
 * way (same staged operands, K order and 64-row statistics chunks); an A/B switch. */
#define STZS_CONV_MRFV_T128 32768
/* flags bit (conv_mfma split-K with one input-channel chunk per slice): keep the 3-slot weight ring instead of the
 * DEEP form (every K-step of the slice in its own LDS slot, all issued at entry).  Bit-identical; an A/B switch. */
#define STZS_CONV_RING 65536
/* flags bit (with the DEEP split-K form): combine the slices in the tile's last-arriving workgroup (one workgroup reads
 * every other slice's 64-KB fp32 slab) instead of the second launch splitk_epi (8 workgroups per tile).  Outputs are
 * bit-identical; the fused statistics partials differ in fp32 association only.  An A/B switch. */
#define STZS_CONV_SK_TICKET 131072
/* bytes of splitk_ws for a K-sliced small-M linear over `rows` rows, Co columns, kgroups slices: covers both the
 * csrc/rows.hip form (STZS_CONV_ROWS) and the 16-row K-slice form of stzs_ln_linear (ln = NULL, splitk in {2, 4}) */
size_t stzs_conv_rows_workspace(int64_t rows, int32_t Co, int32_t kgroups);
int stzs_conv1d(const stzs_conv_args* a, void* stream);
/* n in 1..3 independent stzs_conv1d problems (no one reads another's output) in as few launches as the library can:
 * the k3 / k7 / k11 convs of one generator MRF layer (a[0..2]: STZS_CONV_W_FRAG32, ks 3, 7, 11, Snake AdaIN prologue,
 * no acc_in, alpha 1, same B / T_out / Ci / Co / ci_pad / co_pad, all with or all without a residual, small grids --
 * each taking the 64-row tiles on its own, e.g. batch 1) run as ONE launch whose workgroups execute each problem's own
 * kernel body; two generic-path bf16 convs that would each take the DEEP split-K form with its combine launch (splitk
 * = ci_pad / cic, same shape / slice count / prologue activation: the prosody predictor's F0 and N branches at batch 1,
 * each with its OWN splitk_ws) share one conv launch and one combine launch; anything else runs one stzs_conv1d after
 * the other.  Outputs (and fused statistics partials) are bit-identical to n stzs_conv1d calls either way.  Returns 1
 * when the problems shared their launches, n when they ran one after the other, or a negative STZS_E* code (from the
 * first failing problem's checks; the problems before it have been launched).  (r06: no reference counterpart -- the
 * reference runs these convs one at a time) */
int stzs_conv1d_group(const stzs_conv_args* a, int n, void* stream);

/* ---- InstanceNorm statistics over time, per (b, c): mean and 1/sqrt(var + eps) -----------
 * x [B, T, ld] (bf16|f32), channels [0, C).  `partial` is caller workspace of
 * stzs_chan_stats_workspace(B, T, C) bytes.  (SURVEY §8(a) a9/a12 AdaIN statistics) */
typedef struct stzs_stats_args {
    const void* x;
    float* mean;
    float* rstd;
    void* partial;
    int64_t ld, bs, stat_bs;
    int32_t B, T, C, dtype;
    float eps, pad_f;
} stzs_stats_args;
size_t stzs_chan_stats_workspace(int B, int T, int C);
int stzs_chan_stats(const stzs_stats_args* a, void* stream);
/* pass 1 of stzs_chan_stats alone: the fp32 (sum, sumsq) partials of every 256-row chunk into a->partial
 * ([B][ceil(T / 256)][C][2]; mean / rstd not written, may be NULL) -- for a consumer that finalises them itself
 * (stzs_conv_args.pro_part) or a later stzs_chan_stats_final(a, 256). */
int stzs_chan_stats_partial(const stzs_stats_args* a, void* stream);
/* second pass only: mean / rstd from a partial slab already holding ceil(T / chunk_rows) chunks
 * (written by stzs_conv1d's stat_part epilogue with chunk_rows = STZS_CONV_STAT_ROWS); x unused. */
int stzs_chan_stats_final(const stzs_stats_args* a, int chunk_rows, void* stream);
/* n in 1..3 stzs_chan_stats_final problems (same chunk_rows) in ONE launch; each mean / rstd bit-identical to its own
 * stzs_chan_stats_final call.  (r06: the three MRF resblocks' statistics at batch 1, beside stzs_conv1d_group) */
int stzs_chan_stats_final_group(const stzs_stats_args* a, int n, int chunk_rows, void* stream);

/* ---- row LayerNorm + modulation (+activation), one wave per row -------------------------
 * y[r, c] = act((x - mu_r) * rstd_r * (gadd + G[(r/gdiv)*gs + c]) + Bt[(r/gdiv)*bs + c])
 * (AdaLN / adaLN-single modulate / affine LayerNorm) */
typedef struct stzs_rowln_args {
    const void* x;
    void* y;
    const float* G;
    const float* Bt;
    int64_t ldx, ldy, gs, bs;
    int32_t R, C, gdiv, in_dtype, out_dtype, act;
    float gadd, eps, slope, pad_f;
    /* out_dtype = STZS_F8: y holds e4m3fn codes of y / y_scale[r], y_scale[r] the power-of-two row
     * scale of stzs_quant_rows */
    float* y_scale;
} stzs_rowln_args;
int stzs_row_layernorm(const stzs_rowln_args* a, void* stream);
/* the LayerNorm that feeds a small-M linear, fused into it (csrc/lnrows.hip; the configs[1] batch-1 denoiser's
 * adaLN / affine LayerNorms, each read by one linear): y = epilogue(A W^T) with A = the bf16 rows stzs_row_layernorm(ln)
 * would store (its statistics summed per 16-lane group: within one bf16 ulp; ln->y is not written).  a: a linear
 * (ks 1, no prologue, no residual / gate / split-K / fp8) on STZS_PACK_KSTEP bf16 weights with Ci = ci_pad = ln->C in
 * {128, 256, 512}; a->x unused, ln->R = B * T_in rows of ln->x (f32 | bf16), ln->out_dtype = STZS_BF16, ln->act
 * NONE.  Epilogue: bias, epi_act NONE | GELU | SILU, alpha, beta * acc_in; y bf16 | f32.  Per output element one
 * sequential K chain (batch-invariant).
 * ln = NULL: the plain small-M linear on 16-row workgroups of 16 columns (64 with K slices; A = the x rows: bf16, or fp32 scaled
 * by pro_cscale and rounded to bf16; ci_pad / 32 in {4, 8, 16, 32, 64}; x 16-B aligned, ldx / bsx multiples of 8;
 * epilogue adds the FLAT gate and the residual).  splitk = Z in {2, 4} with ci_pad / 32 / Z in {4, 8, 16}: K slices
 * handed to each tile's last arriver through splitk_ws (stzs_conv_rows_workspace(rows, Co, Z) bytes suffice) and
 * splitk_ctr (zeroed uint32 tickets, left zero), summed in slice order. */
int stzs_ln_linear(const stzs_conv_args* a, const stzs_rowln_args* ln, void* stream);

/* per-row fp8 quantisation with a power-of-two row scale (exact scaling, as MX block scales):
 * scale[r] = 2^k_r, the smallest power of two with amax_r / 2^k_r <= 448 (1 for an all-zero row),
 * y[r, c] = e4m3fn_rne(x[r, c] / scale[r]); x bf16 [R, ldx], C % 8 == 0, C <= 2048, ldy % 16 == 0.
 * (configs[4]: attention outputs and the FFN hidden rows entering the fp8 denoiser linears) */
typedef struct stzs_quant_args {
    const void* x;
    void* y;
    float* scale;
    int64_t ldx, ldy;
    int32_t R, C;
} stzs_quant_args;
int stzs_quant_rows(const stzs_quant_args* a, void* stream);

/* ---- multi-head attention, softmax(q k^T / sqrt(dh)) v, rows independent ----------------
 * q [R, Lq, ldq], k/v [R, Lk, ldk/ldv], o [R, Lq, ldo]; bf16 (precise = 0, MFMA flash kernel) or fp32
 * (precise = 1: split-operand bf16x3 products on the same MFMAs, libm expf -- the precise mode); heads x dh = D.
 * (denoiser self-attention over L_s codes, cross-attention to context) */
typedef struct stzs_attn_args {
    const void* q;
    const void* k;
    const void* v;
    void* o;
    int64_t ldq, ldk, ldv, ldo, bsq, bsk, bsv, bso;
    int32_t R, Lq, Lk, heads, dh, precise;
} stzs_attn_args;
int stzs_attention(const stzs_attn_args* a, void* stream);

/* ---- LSTM recurrence (input projection done by stzs_conv1d) -----------------------------
 * gx [B, T, ldg] f32 holds x W_ih^T + b_ih + b_hh for both directions (fwd 4H | rev 4H, gate
 * order i,f,g,o); whhT = W_hh^T as bf16 16x16x32 B fragments [2][4H/16][H/32][64][8]
 * (stzs/weights.py lstm_frags); H % 32 == 0, H <= 256; h written bf16 to y[b, t, dir*H + j].
 * Launches H/32 x ndir x ceil(B/64) co-resident workgroups that exchange h_t every step through
 * `xchg` (write-through stores + agent-scope arrival counters in `sync`); spins are bounded and a
 * timeout ORs STZS_STATUS_LSTM_TIMEOUT into `*status` (and the last word of `sync`) instead of hanging.
 * (DurationEncoder BiLSTMs, duration LSTM, shared LSTM) */
typedef struct stzs_lstm_args {
    const float* gx;
    const void* whhT;
    void* y;
    void* xchg;  /* workspace: stzs_lstm_workspace(B, H, ndir) bytes, zero-initialised once */
    void* sync;  /* workspace: 4096 bytes of arrival counters, zero-initialised ONCE by the caller; every call
                  * leaves them zeroed (its last workgroup resets them), so no per-call memset is needed.
                  * Calls sharing one sync buffer must be stream-ordered. */
    int64_t ldg, bsg, ldy, bsy;
    int32_t B, T, H, ndir;
    /* optional caller-owned status word: a spin that times out ORs STZS_STATUS_LSTM_TIMEOUT into it (the
     * h-states of that call are then wrong).  Never cleared by the library, so one word can collect the
     * status of every launch of a captured graph; the caller reads it after the work (StyleTTSZS raises). */
    uint32_t* status;
    uint32_t spin_limit; /* polls before a spin times out; 0 = default (1 << 22). Tests force small values. */
    /* 1 = PRECISE split-operand mode: whhT holds the hi fragments of both directions followed by the lo ones
     * (stzs/weights.py pack_lstm(x3=True)), h is exchanged as hi | lo bf16, the gates use libm expf / tanhf
     * and y is fp32 [b, t, dir*H + j].  0 = bf16 h / bf16 y. */
    uint32_t precise;
} stzs_lstm_args;
#define STZS_STATUS_LSTM_TIMEOUT 1u
size_t stzs_lstm_workspace(int B, int H, int ndir);
int stzs_lstm(const stzs_lstm_args* a, void* stream);
/* two INDEPENDENT recurrences in one launch (side by side on the chip, whatever a graph runtime does with
 * concurrent branches): same B, H, ndir and precise (one kernel shape), each with its own gx / weights / T / y and
 * its OWN xchg workspace and sync block (a->xchg != b->xchg, a->sync != b->sync, else STZS_EINVAL); each output is
 * the same bits as its own stzs_lstm call.  STZS_ESHAPE when the shapes differ.  Where the two grids together
 * would exceed one workgroup per CU (e.g. B > 128 at H = 256) the two recurrences are launched one after the other on
 * the stream instead -- same bits, no error.  (Replaces two back-to-back stzs_lstm calls -- the duration LSTM and the shared F0/N LSTM
 * of ProsodyPredictor when the durations are given) */
int stzs_lstm_pair(const stzs_lstm_args* a, const stzs_lstm_args* b, void* stream);
/* zero an LSTM's exchange state -- the 4096-B `sync` block and the granule region at the start of `xchg` (may be
 * NULL) -- with a tiny kernel of agent-scope atomic stores (graph-replay coherent, unlike a memset node).  For
 * callers that keep that state in scratch memory shared with other work (the generic stzs_bilstm does this
 * before every recurrence). */
int stzs_lstm_state_reset(void* sync, void* xchg, void* stream);

/* ---- predictor glue ---- */
/* per-token style: linear resample of codes[:, :, c0:c0+Cs] (L_s rows) to T rows (F.interpolate
 * linear, align_corners=False) into y[b, t, yc0 + c], plus copy of h[b, t, 0:Ch] to y[..., 0:Ch] */
typedef struct stzs_prprep_args {
    const float* codes;
    const void* h;
    void* y;
    int64_t ldc, bsc, ldh, bsh, ldy, bsy;
    int32_t B, L, T, c0, Cs, Ch, yc0, f32; /* f32 = 1: h and y fp32 (precise mode), 0: bf16 */
} stzs_prprep_args;
int stzs_predictor_prep(const stzs_prprep_args* a, void* stream);

/* durations: round(sum_j sigmoid(logit_j)) (serial fp32 sum), clamp >= 1; override if given */
typedef struct stzs_dur_args {
    const float* logits;
    const int32_t* override_dur;
    int32_t* dur;
    float* dsum;
    int64_t ldl, bsl;
    int32_t B, T, nbins, pad_i;
} stzs_dur_args;
int stzs_durations(const stzs_dur_args* a, void* stream);

/* alignment: exclusive scan of dur -> token index per aligned frame idx[b, f], f < T40;
 * frames beyond sum(dur) get -1; total[b] = sum(dur). */
typedef struct stzs_align_args {
    const int32_t* dur;
    int32_t* idx;
    int32_t* total;
    int32_t B, T, T40, pad_i;
} stzs_align_args;
int stzs_alignment(const stzs_align_args* a, void* stream);

/* row gather: y[b, f, yc0 + c] = x[b, idx[b, f], xc0 + c] for c < C (C % 8 == 0); idx<0 -> 0 */
typedef struct stzs_gather_args {
    const void* x;
    const int32_t* idx;
    void* y;
    int64_t ldx, bsx, ldy, bsy;
    int32_t B, Tsrc, Tdst, C, xc0, yc0, dtype, pad_i;
} stzs_gather_args;
int stzs_gather_rows(const stzs_gather_args* a, void* stream);

/* AdaIN + LeakyReLU(0.2) + depthwise ConvTranspose1d(k3, s2, p1, op1): [B,T,C] -> [B,2T,C] */
typedef struct stzs_dwup_args {
    const void* x;
    void* y;
    const float* mean;
    const float* rstd;
    const float* gb;
    const float* w;   /* [C][3] */
    const float* wb;  /* [C] */
    int64_t ldx, bsx, ldy, bsy, stat_bs, gb_bs, gb_beta_off;
    int32_t B, T, C, dtype; /* dtype of x and y: STZS_BF16 | STZS_F32 */
    float slope, pad_f;
} stzs_dwup_args;
int stzs_adain_dwup(const stzs_dwup_args* a, void* stream);

/* Conv1d(1,1,k3,s2,p1) on F0 and N [B, T80] f32 -> bf16 channels of up to two destinations */
typedef struct stzs_f0n_args {
    const float* f0;
    const float* n;
    const float* wf; /* 4 floats: w0 w1 w2 bias */
    const float* wn;
    void* y0;
    void* y1;
    int64_t ldf, ldy0, bsy0, ldy1, bsy1;
    int32_t B, T80, cf0, cn0, cf1, cn1;
    int32_t dtype, pad_i; /* dtype of y0 / y1: STZS_BF16 | STZS_F32 */
} stzs_f0n_args;
int stzs_f0n_down(const stzs_f0n_args* a, void* stream);

/* ---- decoder source + iSTFT ---- */
/* harmonic source (SineGen, counter-RNG noise, Linear(9->1)+tanh) and its n_fft STFT
 * (real | imag) -> har [B, Tf, ldh] bf16, Tf = T80*hop/hop_s + 1.  `prefix` is caller workspace
 * [B][nh][T80] f32 (frame-rate phase prefix, computed in fp64 and wrapped every frame). */
typedef struct stzs_source_args {
    const float* f0;
    const uint32_t* seeds;
    const float* merge_w; /* nh weights + 1 bias */
    float* prefix;
    void* har;
    int64_t ldf, ldh, bsh;
    int32_t B, T80, hop, n_fft, hop_s, nh;
    float sr, sine_amp, noise_std, voiced_thr;
    int32_t har_dtype, pad_i; /* dtype of har: STZS_BF16 | STZS_F32 */
} stzs_source_args;
int stzs_harmonic_source(const stzs_source_args* a, void* stream);

/* iSTFT: post [B, Tf, ldp] f32 (n_bins log-mag | n_bins phase-arg) -> wav [B, (Tf-1)*hop_s]
 * spec = exp(m) * exp(i sin(p)); hann window, center=True, window-square normalisation */
typedef struct stzs_istft_args {
    const float* post;
    float* wav;
    int64_t ldp, bsp, bsw;
    int32_t B, Tf, n_fft, hop_s;
} stzs_istft_args;
int stzs_istft(const stzs_istft_args* a, void* stream);

/* streaming iSTFT (SURVEY §8(a) a14, configs[4] long-form): the frames of one chunk [f0, f0 + Fc)
 * emit every output sample whose overlapping frames are all known; the `halo` (= ceil(n_fft/hop_s)
 * - 1, 3 at 20/5) raw frame rows before the chunk are carried in a caller-owned tail
 * [B][halo][ldt] f32 (ldt >= n_fft + 2): tail_in holds frames f0-halo .. f0-1 (unused at f0 = 0),
 * tail_out receives frames f0+Fc-halo .. f0+Fc-1 (must not alias tail_in: ping-pong two buffers).
 * The chunk writes samples n in [n0, n1) (stzs_istft_stream_span) to wav[b*bsw + n - n0]; the
 * final chunk also emits the trailing samples up to (f0 + Fc - 1) * hop_s.  Concatenated chunks
 * are bit-identical to stzs_istft over the whole utterance (same kernel, same summation order). */
typedef struct stzs_istft_stream_args {
    const float* post;     /* chunk frames: row j = frame f0 + j, [B, Fc, ldp] */
    const float* tail_in;
    float* tail_out;
    float* wav;
    int64_t ldp, bsp, bsw, ldt;
    int32_t B, f0, Fc, final_chunk, n_fft, hop_s;
} stzs_istft_stream_args;
int stzs_istft_stream(const stzs_istft_stream_args* a, void* stream);
/* -> halo (>= 0) or a negative error; [*n0, *n1) = output samples of the chunk */
int stzs_istft_stream_span(int f0, int Fc, int final_chunk, int n_fft, int hop_s, int64_t* n0, int64_t* n1);

/* ---- reference-prompt front end (csrc/frontend.hip) -------------------------
 * log-mel of the 3-s reference = stzs_stft_frames -> stzs_conv1d (bf16 DFT GEMM against the cos | -sin
 * basis, fp32 out) -> stzs_log_mel; the prompt encoder's k5 convs run on stzs_conv1d, its adaptive
 * average pooling on stzs_pool_rows. */
/* y[b, t, m] = bf16(window[m] * x[reflect(t * hop + (n_fft - win) / 2 + m - n_fft / 2)]) for m < win,
 * 0 for win <= m < ldy: the windowed STFT frames of torch.stft(center=True, pad_mode="reflect") */
typedef struct stzs_frames_args {
    const float* wav;      /* [B, ldw] f32, N samples each */
    const float* window;   /* [win] f32 (periodic Hann) */
    void* y;               /* [B, F, ldy] bf16, F = N / hop + 1 */
    int64_t ldw, ldy, bsy;
    int32_t B, N, F, n_fft, win, hop;
} stzs_frames_args;
int stzs_stft_frames(const stzs_frames_args* a, void* stream);
/* y[b, t, m] = log(max(sum_{k0 <= k < k1} fb[m][k] (re_k^2 + im_k^2), 1e-5)), [k0, k1) = ranges[m] */
typedef struct stzs_logmel_args {
    const float* spec;     /* [B, F, lds] f32: nbin real parts | nbin imaginary parts */
    const float* fb;       /* [n_mels][nbin] f32 mel filterbank */
    const int32_t* ranges; /* [n_mels][2] nonzero bin range of each filter */
    void* y;               /* [B, F, ldy] bf16 | f32 */
    int64_t lds, bss, ldy, bsy;
    int32_t B, F, nbin, n_mels, out_dtype, pad_i;
} stzs_logmel_args;
int stzs_log_mel(const stzs_logmel_args* a, void* stream);
/* adaptive average pooling over time: y[b, i, c] = mean_{floor(iT/L) <= t < ceil((i+1)T/L)} x[b, t, c] */
typedef struct stzs_pool_args {
    const void* x;
    void* y;
    int64_t ldx, bsx, ldy, bsy;
    int32_t B, T, L, C, in_dtype, out_dtype;
} stzs_pool_args;
int stzs_pool_rows(const stzs_pool_args* a, void* stream);

/* ---- discrete style codes (README.md:5 "fixed-length time-varying discrete style codes") ----
 * product vector quantiser over rows of C = G * dg fp32 values: group g of row r takes the codebook entry
 *   k* = argmin_k d_k,  d_k = sum_{j < dg} (x[r, g*dg + j] - cb[g][k][j])^2
 * accumulated serially over j with separately rounded IEEE sub / mul / add (no FMA contraction), the first
 * minimum winning a tie -- so the indices are bit-exact against the oracle (oracle/stzs_ref.py quantize_codes).
 * idx[r * ldi + g] = k*, y[r * ldy + g*dg + j] = cb[g][k*][j] (dequantised codes; y may alias x when ldy == ldx).
 * lookup != 0: idx is an INPUT (teacher-forced discrete codes, clamped to [0, K)), only y is written and x is
 * unused.  dg in {4, 8, 16}. */
typedef struct stzs_vq_args {
    const float* x;
    const float* codebook; /* [G][K][dg] fp32 */
    int32_t* idx;
    float* y;
    int64_t ldx, ldi, ldy;
    int32_t R, G, K, dg, lookup, pad_i;
} stzs_vq_args;
int stzs_code_quantize(const stzs_vq_args* a, void* stream);

/* ---- sampler glue ---- */
/* c[r, j] = silu(pool[r, j] + temb[j]) -> bf16 */
int stzs_dn_cond(const float* pool, const float* temb, void* c, int R, int D, void* stream);
/* the same for every sampler step at once: c[s][r][j] = silu(pool[r][j] + temb[s][j]), s < steps (the
 * step-invariant conditioning of a whole sampling run in one launch instead of one per NFE) */
int stzs_dn_cond_steps(const float* pool, const float* temb, void* c, int R, int D, int steps, void* stream);
/* precise mode: the same with fp32 c */
int stzs_dn_cond_steps_f32(const float* pool, const float* temb, float* c, int R, int D, int steps, void* stream);
/* out[l][r][j] = mod[r][j] + (table ? table[l][j] : 0) + ((j / D) in scale_mask ? 1 : 0) */
int stzs_adaln_expand(const float* mod, const float* table, float* out, int R, int D, int nchunk,
                      int nlayers, unsigned scale_mask, void* stream);
/* fused CFG combine + Euler step on the duplicated state x [R, N] (R = B or 2B):
 * Dg = cfg ? D_u + s (D_c - D_u) : D_c ;  x <- x + dsig (x - Dg) / s0 (both halves),
 * dsig = sigma_{i+1} - sigma_i rounded once from fp64 on the host */
int stzs_cfg_euler(float* x, const float* D, int B, int N, int cfg, float scale, float s0,
                   float dsig, void* stream);
/* x[r, :] = eps[b, :] * sigma for both halves (state init) */
int stzs_state_init(float* x, const float* eps, int B, int N, int cfg, float sigma, void* stream);
/* y[b, c] = mean_l x[b, l, c0 + c]  (pooled style / prompt vectors), f32 */
int stzs_mean_rows(const float* x, float* y, int B, int L, int64_t ldx, int64_t bsx, int c0,
                   int C, int64_t ldy, void* stream);
/* generic strided 2-D copy with dtype conversion: R rows x C cols (row r of batch b) */
typedef struct stzs_copy_args {
    const void* x;
    void* y;
    int64_t ldx, bsx, ldy, bsy;
    int32_t B, R, C, in_dtype, out_dtype, pad_i;
} stzs_copy_args;
int stzs_copy2d(const stzs_copy_args* a, void* stream);
/* token embedding gather: y[b, t, :] = emb[tok[b, t], :] (f32 table -> bf16 rows) */
int stzs_embed(const int32_t* tok, const float* emb, void* y, int B, int T, int D, int64_t ldy,
               void* stream);
/* precise mode: fp32 embedding rows */
int stzs_embed_f32(const int32_t* tok, const float* emb, float* y, int B, int T, int D, int64_t ldy, void* stream);

/* ======================================================================================================
 * Generic tensor-descriptor entry points (SURVEY.md §8(b) "C-ABI"): one per hot-path operator of §8(a),
 *   int    stzs_<op>(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
 *                    const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
 *   size_t stzs_<op>_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
 * composed in native host code (csrc/abi.hip) over the per-kernel entry points above.  Tensors are caller-owned
 * device memory described by (data, dtype, ndim, shape, stride in ELEMENTS); activations are channels-last
 * [B, T, C] with stride[2] == 1 (the row pitch stride[1] may exceed C).  The workspace is caller-owned device
 * scratch of at least the queried size (ws_bytes is checked), with no required contents: it may be shared by
 * consecutive operators on one stream (the ops holding LSTM exchange state in it reset that state on entry).
 * Aliasing: outputs must not overlap inputs unless an operator says otherwise (cfg_euler_step allows y == x;
 * mrf_resblock rejects overlap with STZS_EINVAL).  Weights are the packed layouts
 * produced by stzs_pack_conv / stzs_pack_lstm below (host memory; the caller copies them to the device).
 * The denoiser, decoder pre-blocks and F0/N predictor (a2, a9, a8) compose dozens of weight tensors: their input
 * lists follow the STZS_DN_* / STZS_DP_* / STZS_FN_* enums at the end of this header.
 * ====================================================================================================== */
typedef struct stzs_tensor_t {
    void* data;
    int32_t dtype; /* STZS_F32 | STZS_BF16 | STZS_I32 | STZS_F8 */
    int32_t ndim;  /* <= 4 */
    int64_t shape[4];
    int64_t stride[4]; /* elements */
} stzs_tensor_t;
typedef struct stzs_params_t {
    int32_t i[16];
    float f[8];
} stzs_params_t;

/* packed weight forms (host-side packers; stzs/weights.py pack_conv restated in C++) */
enum { STZS_PACK_KSTEP = 0, STZS_PACK_LANE16 = 1, STZS_PACK_FRAG32 = 2, STZS_PACK_NARROW32 = 3,
       STZS_PACK_X3 = 4 /* precise mode: hi | lo split streams, 32-channel K-steps (STZS_CONV_W_X3) */,
       STZS_PACK_FRAG32X3 = 5 /* precise mode, register-direct: hi | lo FRAG32 blocks per K-step (STZS_CONV_W_FRAG32X3) */ };
/* bytes of the packed bf16 form of a Conv1d weight [Co][Ci][ks] (ups = 0) or ConvTranspose1d weight [Ci][Co][2 ups]
 * (ups > 0, polyphase); 0 if the form does not apply to the shape */
size_t stzs_pack_conv_size(int Co, int Ci, int ks, int ups, int form);
/* w fp32 (host), packed bf16 (host, stzs_pack_conv_size bytes); returns STZS_OK / STZS_ESHAPE / STZS_EINVAL */
int stzs_pack_conv(const float* w, int Co, int Ci, int ks, int ups, int form, void* packed);
/* LSTM of input width In, hidden H: W_ih (fwd | rev) as ONE KSTEP linear [8H][In] (bytes stzs_pack_conv_size(8H, In,
 * 1, 0, KSTEP)) + its bias b_ih + b_hh [8H] fp32, and W_hh^T MFMA fragments (2 * 4H * H bf16).  Torch gate order
 * i, f, g, o; w_* fp32 host arrays in torch.nn.LSTM layout. */
int stzs_pack_lstm(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, const float* w_ih_rev,
                   const float* w_hh_rev, const float* b_ih_rev, const float* b_hh_rev, int In, int H, void* ih_packed,
                   float* ih_bias, void* whh_frags);
/* the precise-mode LSTM (stzs_lstm_args.precise = 1): W_ih in the STZS_PACK_X3 form (stzs_pack_conv_size(8H, In, 1,
 * 0, STZS_PACK_X3) bytes), the bias as above, and the hi fragments of both directions followed by the lo ones
 * (2 * 2 * 4H * H bf16) */
int stzs_pack_lstm_x3(const float* w_ih, const float* w_hh, const float* b_ih, const float* b_hh, const float* w_ih_rev,
                      const float* w_hh_rev, const float* b_ih_rev, const float* b_hh_rev, int In, int H,
                      void* ih_packed, float* ih_bias, void* whh_frags);

/* a3  cfg_euler_step: in {x f32 [R, N], D f32 [R, N]} -> out {x' f32 [R, N]};
 *     i[0] = cfg (R = 2B, conditional rows first), f[0] = scale, f[1] = sigma, f[2] = sigma_next */
int stzs_cfg_euler_step(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                        const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_cfg_euler_step_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a6  duration_head: in {logits f32 [B, T, nbins]} -> out {dur i32 [B, T] (, dsum f32 [B, T])} */
int stzs_duration_head(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                       const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_duration_head_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a7  length_regulate: in {dur i32 [B, T]} -> out {idx i32 [B, T40]} (T40 = outputs[0].shape[1]) */
int stzs_length_regulate(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                         const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_length_regulate_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a10 sine_gen: in {F0 f32 [B, T80], merge f32 [nh + 1], seeds i32 [B]} -> out {har bf16|f32 [B, Tf, >= n_fft + 2]};
 *     i[0] = hop, i[1] = n_fft, i[2] = hop_s, i[3] = nh; f[0] = sr, f[1] = sine_amp, f[2] = noise_std,
 *     f[3] = voiced_threshold.  Tf = T80 hop / hop_s + 1 */
int stzs_sine_gen(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
                  void* workspace, size_t ws_bytes, void* stream);
size_t stzs_sine_gen_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a13 conv_post_istft: in {x bf16 [B, Tf, Ci], w (packed NARROW32 if Ci % 128 == 0 else KSTEP, Co = n_fft + 2,
 *     ks = 7), bias f32 [Co]} -> out {wav f32 [B, (Tf - 1) hop_s]}; i[0] = n_fft, i[1] = hop_s; f[0] = LeakyReLU slope */
int stzs_conv_post_istft(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                         const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_conv_post_istft_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a5/a8 bilstm: in {x bf16 [B, T, In], ih packed (stzs_pack_lstm), ih_bias f32 [8H], whh frags} -> out {y bf16
 *     [B, T, >= 2H] (, status i32 [1]: OR-ed STZS_STATUS_LSTM_TIMEOUT)}; i[0] = H */
int stzs_bilstm(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
                void* workspace, size_t ws_bytes, void* stream);
size_t stzs_bilstm_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a11 conv_transpose_up: in {x bf16 [B, T, Cin], har bf16 [B, Tf, >= har_ch], ups w (packed LANE16 if Cin % 128 == 0
 *     and Co % 16 == 0 else KSTEP; ConvTranspose1d [Cin][Co][2r]), ups bias f32 [Co], noise w (KSTEP,
 *     [Co][har_ch][nk]), noise bias f32 [Co]} -> out {y bf16 [B, T r + last, >= Co]};
 *     i[0] = r, i[1] = last stage (ReflectionPad(1,0) + 1 row), i[2] = noise kernel nk, i[3] = noise stride,
 *     i[4] = noise pad, i[5] = har_ch, i[6] = Co; f[0] = LeakyReLU slope (0.1) */
int stzs_conv_transpose_up(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                           const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_conv_transpose_up_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);
/* a12 mrf_resblock: the MRF of one generator stage, nk resblocks (kernels i[1..nk]) x nd dilations (i[4..3+nd]),
 *     averaged: in {x bf16 [B, T, C], gb f32 [B, nk * nd * 4C] (per resblock layer (j, m): gamma1 | beta1 | gamma2 |
 *     beta2, C each), then per layer (j, m) in order: c1 w, c1 bias, alpha1 f32 [C], c2 w, c2 bias, alpha2} ->
 *     out {y bf16 [B, T, C]}; i[0] = C, i[1..3] = resblock kernels, i[4..6] = dilations, i[7] = nk, i[8] = nd,
 *     i[9] = weight form (STZS_PACK_FRAG32 | LANE16 | KSTEP) */
int stzs_mrf_resblock(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out,
                      const stzs_params_t* p, void* workspace, size_t ws_bytes, void* stream);
size_t stzs_mrf_resblock_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);

/* ---- composite operators (csrc/abi_ops.hip): the engine's launch sequences in native host code, bit-identical to
 * stzs/engine.py; bf16 activations (the precise mode stays on the Python engine).  Inputs in the enum order below;
 * "w" = a packed STZS_PACK_KSTEP linear (AdaIN-block k3 convs: STZS_PACK_LANE16 when Ci > 64 and Co % 16 == 0),
 * "b" = its fp32 bias.  Workspace: the operator's own query (a dry pass of the same code). */

/* a2 denoiser_fwd: ONE EDM-preconditioned denoiser evaluation D(x, sigma) = c_skip x + c_out F(c_in x, sigma) with
 *     classifier-free-guidance rows: in {x f32 [R, L_s, code] (R = 2B with cfg: conditional rows, then null-prompt
 *     rows), h_txt bf16 [B, T, d_txt], prompt f32 [B, L_s, code], then the weights below} -> out {D f32 [R, L_s, code]};
 *     i[0] = cfg, i[1] = layers, i[2] = heads, i[3] = d, i[4] = ffn width, i[5] = Fourier features (<= 256);
 *     f[0] = sigma, f[1] = sigma_data.  (stzs/engine.py denoiser_prepare + denoiser_step) */
enum {
    STZS_DN_X = 0, STZS_DN_HTXT, STZS_DN_PROMPT,
    STZS_DN_IN_W, STZS_DN_IN_B, STZS_DN_POS /* f32 [L_s, d] */,
    STZS_DN_T0_W, STZS_DN_T0_B, STZS_DN_T1_W, STZS_DN_T1_B,
    STZS_DN_POOL_W, STZS_DN_POOL_B, STZS_DN_CTX_TXT_W, STZS_DN_CTX_TXT_B, STZS_DN_CTX_PRM_W, STZS_DN_CTX_PRM_B,
    STZS_DN_ADA_W, STZS_DN_ADA_B, STZS_DN_ADA_TABLE /* f32 [layers, 6d] */, STZS_DN_FINAL_ADA_W, STZS_DN_FINAL_ADA_B,
    STZS_DN_OUT_W, STZS_DN_OUT_B,
    STZS_DN_CTX_NULL /* bf16 [L_s, d]: null-prompt context rows (cfg) */, STZS_DN_POOL_NULL /* f32 [d] (cfg) */,
    STZS_DN_NIN_BASE /* then per layer l, at STZS_DN_NIN_BASE + STZS_DN_PER_LAYER * l: */
};
enum {
    STZS_DN_L_QKV_W = 0, STZS_DN_L_QKV_B, STZS_DN_L_O_W, STZS_DN_L_O_B, STZS_DN_L_Q_W, STZS_DN_L_Q_B,
    STZS_DN_L_KV_W, STZS_DN_L_KV_B, STZS_DN_L_CO_W, STZS_DN_L_CO_B, STZS_DN_L_FF1_W, STZS_DN_L_FF1_B,
    STZS_DN_L_FF2_W, STZS_DN_L_FF2_B, STZS_DN_L_LN_G /* f32 [d] */, STZS_DN_L_LN_B, STZS_DN_PER_LAYER
};
int stzs_denoiser_fwd(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
                      void* workspace, size_t ws_bytes, void* stream);
size_t stzs_denoiser_fwd_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);

/* a9 decoder_pre: in {asr bf16 [B, T40, d_txt] (aligned text features), F0 f32 [B, T80], N f32 [B, T80] (same row
 *     stride), codes f32 [B, L_s, code], F0 conv f32 [4] (w0 w1 w2 bias), N conv f32 [4], asr_res w, b, AdaIN norm
 *     group w [total x style_ac], b, then 5 blocks (encode, decode0..3) x 7: conv1 w, conv1 b, conv2 w, conv2 b,
 *     sc w (data NULL when din == dout), pool w f32 [din x 3], pool b f32 [din] (decode3 only, else NULL)} ->
 *     [the block convs packed STZS_PACK_FRAG32 when din > 64 and Co % 32 == 0 (conv1, conv2 and the 1x1 shortcut),
 *     else conv1 / conv2 STZS_PACK_LANE16 when Co % 16 == 0 and STZS_PACK_KSTEP otherwise -- stzs/weights.py pack_blk]
 *     out {generator input bf16 [B, T80, >= dec_out]}; i[0] = dec_enc, i[1] = dec_asr_res, i[2] = dec_out,
 *     i[3] = style_ac (acoustic code channels pooled for AdaIN), i[4] = columns of the norm group (its first ones:
 *     norm1 | norm2 gamma-beta of the 5 blocks in order).  (stzs/engine.py decoder_pre) */
enum {
    STZS_DP_ASR = 0, STZS_DP_F0, STZS_DP_N, STZS_DP_CODES, STZS_DP_F0CONV, STZS_DP_NCONV, STZS_DP_ASR_RES_W,
    STZS_DP_ASR_RES_B, STZS_DP_NORM_W, STZS_DP_NORM_B, STZS_DP_BLK0, STZS_DP_NIN = STZS_DP_BLK0 + 35
};
int stzs_decoder_pre(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
                     void* workspace, size_t ws_bytes, void* stream);
size_t stzs_decoder_pre_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);

/* a8 f0n_predictor: in {en bf16 [B, T40, pr_in] (aligned predictor features), codes f32 [B, L_s, code], shared BiLSTM
 *     (stzs_pack_lstm: ih packed, ih bias, W_hh^T fragments), AdaIN norm group w [total x style_pr], b, then per
 *     branch (F0, N) 3 blocks x 7 tensors (as decoder_pre; block 1 up-samples x2) + projection w, b (Co = 1)} ->
 *     out {F0 f32 [B, T80], N f32 [B, T80] (, status i32 [1]: OR-ed STZS_STATUS_LSTM_TIMEOUT)}; i[0] = LSTM hidden H,
 *     i[1..3] = branch widths c0, c1, c2, i[4] = first prosodic code channel, i[5] = prosodic channels, i[6] = norm
 *     group columns.  (stzs/engine.py f0n_predictor) */
enum {
    STZS_FN_EN = 0, STZS_FN_CODES, STZS_FN_LSTM_IH, STZS_FN_LSTM_BIAS, STZS_FN_LSTM_WHH, STZS_FN_NORM_W, STZS_FN_NORM_B,
    STZS_FN_BR0, STZS_FN_PER_BRANCH = 23, STZS_FN_NIN = STZS_FN_BR0 + 2 * 23
};
int stzs_f0n_predictor(const stzs_tensor_t* inputs, int n_in, stzs_tensor_t* outputs, int n_out, const stzs_params_t* p,
                       void* workspace, size_t ws_bytes, void* stream);
size_t stzs_f0n_predictor_workspace(const stzs_tensor_t* inputs, int n_in, const stzs_params_t* p);

#ifdef __cplusplus
}
#endif
#endif /* STZS_H */
