/* stzs_fused.h -- fused small-M linears of the batch-1 denoiser (SURVEY.md §8(a) a2 at B = 1, configs[1]).
 *
 * At batch 1 a denoiser evaluation is ~70 dependent launches of a few microseconds each; a graph-replayed
 * dependent launch costs ~5.7 us on MI355X, so the launch count, not the arithmetic, sets the
 * latency.  These entry points run the whole-chip small-M linear of STZS_CONV_ROWS (csrc/rows.hip) with the
 * operation that CONSUMES its output folded into the same launch, handed over inside the launch by the
 * last-arriver pattern (no spinning, no co-residency assumption):
 *
 *   STZS_FUSE_LN    the LayerNorm of the output rows (stzs_row_layernorm semantics, `ln`): the output is stored
 *                   write-through (sc1); every 16-row block has a counter, the block's last-arriving column tile
 *                   normalises its 16 rows (sc1 loads) and writes ln.y.  Replaces stzs_conv1d + stzs_row_layernorm
 *                   (the residual linears sa_o / ca_o / ff2 and the input projection of the denoiser).
 *   STZS_FUSE_ATTN  the multi-head attention whose q (and k / v, if they lie in y) are this linear's output
 *                   (stzs_attention semantics, `attn`, bf16, dh = 64): every (utterance, head) has a counter over
 *                   the column tiles of that head and the row blocks of that utterance; its last arriver runs the
 *                   flash unit of that head (sc1 loads) and writes attn.o.  Replaces stzs_conv1d +
 *                   stzs_attention: the qkv linear + self-attention, the cross-attention query linear +
 *                   cross-attention.
 *   STZS_FUSE_CFG   the classifier-free-guidance combine + Euler step of the sampler state (stzs_cfg_euler
 *                   semantics, `cfg_*`) on the denoiser output D = y: every 16-column tile has a counter over the row
 *                   blocks, its last arriver updates the state x for its columns (D by sc1 loads).  Replaces
 *                   stzs_conv1d + stzs_cfg_euler for the denoiser's output projection.
 *
 * Results are bit-identical to the unfused pair (same per-element arithmetic: the linear's K order depends on K
 * and the split only, the LayerNorm / attention code is the same device code).  Counters: `ctr` holds
 * stzs_rows_fuse_counters() uint32 words, ZERO before the first launch; every launch leaves them zero.
 */
#ifndef STZS_FUSED_H
#define STZS_FUSED_H
#include "stzs.h"
#ifdef __cplusplus
extern "C" {
#endif

#define STZS_FUSE_LN 1
#define STZS_FUSE_ATTN 2
#define STZS_FUSE_CFG 3

typedef struct stzs_rows_fuse {
    int32_t mode;           /* STZS_FUSE_LN | STZS_FUSE_ATTN */
    int32_t pad0;
    unsigned int* ctr;      /* hand-off counters (see above) */
    /* STZS_FUSE_LN: x == the linear's y (fp32, rows flat: bsy == T_in * ldy or B == 1), ldx == ldy,
     * R == B * T_in, C == Co <= 2048, out_dtype BF16, in_dtype F32 */
    stzs_rowln_args ln;
    /* STZS_FUSE_ATTN: bf16, precise 0, dh 64, q == y (+ 0), R == B, Lq == T_in, Co % (heads * dh) == 0;
     * k / v may point into y (the qkv linear) or at tensors written by earlier launches */
    stzs_attn_args attn;
    /* STZS_FUSE_CFG: y = D fp32 [R, T_in, Co] flat (ldy == Co, bsy == T_in * Co), R == 2 cfg_B (cfg_on) or cfg_B;
     * cfg_x = the state [R, T_in * Co] fp32 (x of stzs_cfg_euler), updated in place for rows < cfg_B and copied to
     * rows cfg_B + b when cfg_on; scale / sigma / dsig as stzs_cfg_euler's s / s0 / dsig */
    float* cfg_x;
    int32_t cfg_B, cfg_on;
    float cfg_scale, cfg_sigma, cfg_dsig, cfg_pad;
} stzs_rows_fuse;

/* counter words a fused launch of `a` needs (0 for a bad argument) */
size_t stzs_rows_fuse_counters(const stzs_conv_args* a, const stzs_rows_fuse* f);
/* the STZS_CONV_ROWS linear `a` (its contract, include/stzs.h) + the fused consumer `f` in ONE launch */
int stzs_conv_rows_fused(const stzs_conv_args* a, const stzs_rows_fuse* f, void* stream);

#ifdef __cplusplus
}
#endif
#endif
