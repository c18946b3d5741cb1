// stzs_conv1d entry (include/stzs.h): argument checks shared by every conv form, then the
// register-direct MRF conv (csrc/mrfv.hip) for STZS_CONV_W_FRAG32 weights, the general dispatcher
// (csrc/conv.hip) for everything else.  Kept in its own translation unit so that adding a kernel
// form does not rebuild conv.hip.
#include "common.hpp"

int stzs_conv1d_core(const stzs_conv_args* a, void* stream);           // csrc/conv.hip
int stzs_mrfv_conv_launch(const stzs_conv_args& a, hipStream_t s);    // csrc/mrfv.hip
int stzs_rows_gemm_launch(const stzs_conv_args& a, hipStream_t s);    // csrc/rows.hip
int stzs_mrfx_conv_launch(const stzs_conv_args& a, hipStream_t s);    // csrc/mrfx.hip

int stzs_mrfv_trio_launch(const stzs_conv_args* a, hipStream_t s);   // csrc/mrfv.hip
int stzs_conv_pair_launch(const stzs_conv_args* a, hipStream_t s);    // csrc/conv.hip

namespace {

// stzs_conv1d's argument checks for STZS_CONV_W_FRAG32 weights (the register-direct conv)
int frag32_checks(const stzs_conv_args* a) {
    if (!a->x || !a->w || !a->y) return STZS_EINVAL;
    if (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_A_DMA)) return STZS_EINVAL;
    if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0 || a->dil <= 0) return STZS_ESHAPE;
    if (a->ci_pad < a->Ci || a->co_pad < a->Co) return STZS_ESHAPE;
    if (a->ldx % 8 || a->bsx % 8 || a->ldx < ((a->Ci + 7) / 8) * 8) return STZS_ESHAPE;
    if (!stzs_aligned(a->x, 16) || !stzs_aligned(a->w, 16) || !stzs_aligned(a->y, 16)) return STZS_EINVAL;
    if (a->pro_mode == STZS_PRO_ADAIN && (!a->pro_mean || !a->pro_rstd || !a->pro_gb)) return STZS_EINVAL;
    if (a->in_dtype == STZS_F8 || a->x_scale) return STZS_EDTYPE;
    if (a->splitk > 1) return STZS_EINVAL;
    if (a->stat_part && !stzs_aligned(a->stat_part, 8)) return STZS_EINVAL;
    return STZS_OK;
}

}  // namespace

extern "C" int stzs_conv1d_group(const stzs_conv_args* a, int n, void* stream) {
    if (!a || n < 1 || n > 3) return STZS_EINVAL;
    if (n == 3 && !a[0].pro_part && !a[1].pro_part && !a[2].pro_part && (a[0].flags & STZS_CONV_W_FRAG32) &&
        (a[1].flags & STZS_CONV_W_FRAG32) && (a[2].flags & STZS_CONV_W_FRAG32) && !(a[0].flags & STZS_CONV_W_FRAG32X3) &&
        !(a[1].flags & STZS_CONV_W_FRAG32X3) && !(a[2].flags & STZS_CONV_W_FRAG32X3) && a[0].ups <= 0 && a[1].ups <= 0 &&
        a[2].ups <= 0 && frag32_checks(&a[0]) == STZS_OK && frag32_checks(&a[1]) == STZS_OK &&
        frag32_checks(&a[2]) == STZS_OK) {
        const int rc = stzs_mrfv_trio_launch(a, reinterpret_cast<hipStream_t>(stream));
        if (rc == STZS_OK) return 1;
        if (rc != STZS_ESHAPE) return rc;
    }
    if (n == 2 && !a[0].pro_part == !a[1].pro_part) {  // (pro_part: both or neither, as the body reads it uniformly)
        const int rc = stzs_conv_pair_launch(a, reinterpret_cast<hipStream_t>(stream));
        if (rc == STZS_OK) return 1;
        if (rc != STZS_ESHAPE) return rc;
    }
    for (int i = 0; i < n; ++i) {  // one after the other (the same results)
        const int rc = stzs_conv1d(&a[i], stream);
        if (rc != STZS_OK) return rc;
    }
    return n;
}

extern "C" int stzs_conv1d(const stzs_conv_args* a, void* stream) {
    // prologue statistics from partials (pro_part): the generic conv path only (csrc/conv.hip checks the rest)
    if (a && a->pro_part && (a->flags & (STZS_CONV_W_FRAG32X3 | STZS_CONV_W_FRAG32 | STZS_CONV_ROWS))) return STZS_EINVAL;
    if (a && (a->flags & STZS_CONV_W_FRAG32X3)) {  // the precise register-direct form
        if (!a->x || !a->w || !a->y) return STZS_EINVAL;
        if (a->flags & (STZS_CONV_W_LANE16 | STZS_CONV_W_NARROW32 | STZS_CONV_W_F32 | STZS_CONV_W_X3 | STZS_CONV_A_DMA |
                        STZS_CONV_W_FRAG32 | STZS_CONV_ROWS | STZS_CONV_UPS_NOISE))
            return STZS_EINVAL;
        if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0 || a->dil <= 0) return STZS_ESHAPE;
        if (a->ci_pad < a->Ci || a->co_pad < a->Co || a->ldx < ((a->Ci + 7) / 8) * 8) return STZS_ESHAPE;
        if (!stzs_aligned(a->w, 16)) return STZS_EINVAL;
        if (a->pro_mode == STZS_PRO_ADAIN && (!a->pro_mean || !a->pro_rstd || !a->pro_gb)) return STZS_EINVAL;
        if (a->in_dtype == STZS_F8 || a->x_scale) return STZS_EDTYPE;
        if (a->splitk > 1) return STZS_EINVAL;
        if (a->stat_part && !stzs_aligned(a->stat_part, 8)) return STZS_EINVAL;
        return stzs_mrfx_conv_launch(*a, reinterpret_cast<hipStream_t>(stream));
    }
    if (a && (a->flags & STZS_CONV_W_FRAG32)) {
        const int rc = frag32_checks(a);
        if (rc != STZS_OK) return rc;
        return stzs_mrfv_conv_launch(*a, reinterpret_cast<hipStream_t>(stream));
    }
    if (a && (a->flags & STZS_CONV_ROWS)) {
        if (!a->x || !a->w || !a->y) return STZS_EINVAL;
        if (a->B <= 0 || a->T_in <= 0 || a->T_out <= 0 || a->Ci <= 0 || a->Co <= 0) return STZS_ESHAPE;
        if (a->ci_pad < a->Ci || a->co_pad < a->Co || a->co_pad % 128) return STZS_ESHAPE;
        if (a->ldx % 8 || a->bsx % 8) return STZS_ESHAPE;
        if (!stzs_aligned(a->x, 16) || !stzs_aligned(a->w, 16)) return STZS_EINVAL;
        if (a->res && a->res_tdiv != 1) return STZS_EINVAL;  // the residual row is the output row (rows.hip)
        return stzs_rows_gemm_launch(*a, reinterpret_cast<hipStream_t>(stream));
    }
    return stzs_conv1d_core(a, stream);
}
