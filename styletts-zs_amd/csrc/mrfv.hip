// The MRF conv, register-direct weight form: the launcher (stzs_mrfv_conv_launch) and the
// multi-chunk instances -- the wide stage-0 forms and the decoder / predictor AdaIN-block k3 convs.  The kernel template
// and its design notes: csrc/mrfv_kernel.hpp; the single-chunk stage-1 instances: csrc/mrfv_n1.hip.
#include "mrfv_kernel.hpp"

namespace {

template <int PACT, bool HR, bool HA>
void (*pick(int ks, bool one, bool al, bool wide, bool t64))(stzs_conv_args) {
    if (wide) return al ? pick_ks<PACT, HR, HA, 0, true, 2>(ks) : pick_ks<PACT, HR, HA, 0, false, 2>(ks);
    static_assert(PACT == STZS_ACT_SNAKE, "the single-chunk forms are the Snake (MRF) convs");
    if (one) return stzs_mrfv_pick_n1(ks, HR, HA, al, t64);  // (csrc/mrfv_n1.hip)
    if (t64)  // (64-row tiles: the Snake forms of small grids)
        return al ? pick_ks<PACT, HR, HA, 0, true, 1, 64>(ks) : pick_ks<PACT, HR, HA, 0, false, 1, 64>(ks);
    return al ? pick_ks<PACT, HR, HA, 0, true>(ks) : pick_ks<PACT, HR, HA, 0, false>(ks);
}

}  // namespace

int stzs_ups_conv_launch(const stzs_conv_args& a, hipStream_t s);   // csrc/ups.hip (polyphase ConvTranspose)

namespace {

// the launcher's shape checks (beyond stzs_conv1d's own)
int mrfv_shape(const stzs_conv_args& a) {
    const int rows_in = 128 + (a.ks - 1) * a.dil;
    if (a.stride != 1 || a.cic != 128 || a.ci_pad % 128 || a.Co % 8 || a.co_pad % BCO || rows_in > 16 * sb_rows(a.ks) ||
        a.in_dtype != STZS_BF16 || a.out_dtype != STZS_BF16 || a.gate || a.epi_act != STZS_ACT_NONE || a.ups ||
        a.refl || a.ldy % 8 || a.bsy % 8 || (a.res && (a.ldr % 8 || a.bsr % 8 || a.res_tdiv <= 0)) ||
        (a.acc_in && (a.lda % 8 || a.bsa % 8)) || (a.stat_part && a.stat_ld < a.Co))
        return STZS_ESHAPE;
    if (a.pro_act == STZS_ACT_SNAKE && !a.pro_alpha) return STZS_EINVAL;
    if (a.pro_act == STZS_ACT_SNAKE && a.res && a.res_tdiv != 1) return STZS_ESHAPE;  // (TD1 in the kernel)
    return STZS_OK;
}

// the Snake forms' tile choice: the wide form (256 output channels per workgroup) for multi-chunk Snake convs whose wide
// grid still gives every CU two workgroups (at batch 1 a stage-0 conv has 32 row tiles: the narrow form's 64 workgroups
// finish sooner), unless STZS_CONV_MRFV_NARROW; else 64-row tiles where the narrow 128-row grid would not give every CU
// two workgroups (batch 1: a stage-1 conv is 188 tiles, a stage-0 conv 64), unless STZS_CONV_MRFV_T128.  Every form is
// bit-identical, so the choice never changes a result.
void snake_form(const stzs_conv_args& a, bool& wide, bool& t64) {
    const long wide_tiles = (long)a.B * ((a.T_out + 127) / 128) * (a.co_pad / (2 * BCO));
    wide = a.pro_act == STZS_ACT_SNAKE && a.ci_pad > 128 && a.co_pad % (2 * BCO) == 0 && wide_tiles >= 512 &&
           !(a.flags & STZS_CONV_MRFV_NARROW);
    const long tiles128 = (long)a.B * ((a.T_out + 127) / 128) * (a.co_pad / BCO);
    const int rows64 = 64 + (a.ks - 1) * a.dil;
    t64 = !wide && a.pro_act == STZS_ACT_SNAKE && tiles128 < 2 * stzs_cu_count() &&
          rows64 <= 16 * (a.ks == 3 ? sb_rows64(3) : a.ks == 7 ? sb_rows64(7) : sb_rows64(11)) &&
          !(a.flags & STZS_CONV_MRFV_T128);
}

}  // namespace

// (r06) the k3 / k7 / k11 convs of one MRF layer in one launch (mrfv_trio, csrc/mrfv_kernel.hpp): STZS_ESHAPE unless
// a[0..2] have ks 3, 7, 11, the Snake prologue, no accumulate input, alpha 1, the same B / T_out / Ci / Co / padding
// and residual-ness, and each would take the narrow 64-row form on its own (the small grids of batch 1).  The caller
// (stzs_conv1d_group) has run stzs_conv1d's argument checks on each.
__attribute__((visibility("hidden"))) int stzs_mrfv_trio_launch(const stzs_conv_args* a, hipStream_t s) {
    static const int KS[3] = {3, 7, 11};
    size_t lds = 0;
    for (int i = 0; i < 3; ++i) {
        const stzs_conv_args& b = a[i];
        const int rc = mrfv_shape(b);
        if (rc != STZS_OK) return rc;
        bool wide, t64;
        snake_form(b, wide, t64);
        if (b.ks != KS[i] || b.pro_act != STZS_ACT_SNAKE || b.acc_in || b.alpha != 1.f || !t64 || wide ||
            b.B != a[0].B || b.T_out != a[0].T_out || b.Ci != a[0].Ci || b.Co != a[0].Co || b.ci_pad != a[0].ci_pad ||
            b.co_pad != a[0].co_pad || (b.res != nullptr) != (a[0].res != nullptr))
            return STZS_ESHAPE;
        const size_t l = mrfv_lds(64 + (b.ks - 1) * b.dil);
        lds = l > lds ? l : lds;
    }
    const bool R = a[0].res != nullptr;
    void (*k)(stzs_conv_args, stzs_conv_args, stzs_conv_args) =
        a[0].ci_pad == 128 ? stzs_mrfv_trio_pick_n1(R) : (R ? mrfv_trio<true, 0, 64> : mrfv_trio<false, 0, 64>);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    dim3 grid((unsigned)a[0].B * (unsigned)((a[0].T_out + 63) / 64), a[0].co_pad / BCO, 3);
    hipLaunchKernelGGL(k, grid, dim3(NTH), lds, s, a[0], a[1], a[2]);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

// internal entry used by stzs_conv1d for STZS_CONV_W_FRAG32 weights
__attribute__((visibility("hidden"))) int stzs_mrfv_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    if (a.ups > 0) return stzs_ups_conv_launch(a, s);
    {
        const int rc = mrfv_shape(a);
        if (rc != STZS_OK) return rc;
    }
    void (*k)(stzs_conv_args) = nullptr;
    const bool R = a.res != nullptr, A = a.acc_in != nullptr;
    bool blk_wide = false, blk_t64 = false;
    bool wide, t64;
    snake_form(a, wide, t64);
    const long wide_tiles = (long)a.B * ((a.T_out + 127) / 128) * (a.co_pad / (2 * BCO));
    const long tiles128 = (long)a.B * ((a.T_out + 127) / 128) * (a.co_pad / BCO);
    if (a.pro_act == STZS_ACT_SNAKE) {
        const bool one = a.ci_pad == 128;
        const bool al = a.alpha != 1.f;
        k = R ? (A ? pick<STZS_ACT_SNAKE, true, true>(a.ks, one, al, wide, t64) : pick<STZS_ACT_SNAKE, true, false>(a.ks, one, al, wide, t64))
              : (A ? pick<STZS_ACT_SNAKE, false, true>(a.ks, one, al, wide, t64) : pick<STZS_ACT_SNAKE, false, false>(a.ks, one, al, wide, t64));
    } else if (!A && a.ks == 1 && a.pro_act == STZS_ACT_NONE && a.pro_mode == STZS_PRO_NONE && !a.stat_part) {
        // (r06) the AdaIN blocks' 1x1 shortcut convs (1090 -> 1024 at the decoder): the block convs' data movement with
        // one tap -- as a FLAT LDS-DMA GEMM they ran at 0.11 of their roofline, streaming A and B tiles through LDS
        blk_wide = a.ci_pad > 128 && a.co_pad % (2 * BCO) == 0 && wide_tiles >= 2 * stzs_cu_count() &&
                   !(a.flags & STZS_CONV_MRFV_NARROW);
        blk_t64 = !blk_wide && tiles128 < 4 * stzs_cu_count() && !(a.flags & STZS_CONV_MRFV_T128);
        k = blk_wide ? (R ? mrfv_conv<STZS_ACT_NONE, true, false, 1, 0, true, 2> : mrfv_conv<STZS_ACT_NONE, false, false, 1, 0, true, 2>)
          : blk_t64 ? (R ? mrfv_conv<STZS_ACT_NONE, true, false, 1, 0, true, 1, 64> : mrfv_conv<STZS_ACT_NONE, false, false, 1, 0, true, 1, 64>)
                     : (R ? mrfv_conv<STZS_ACT_NONE, true, false, 1, 0, true> : mrfv_conv<STZS_ACT_NONE, false, false, 1, 0, true>);
    } else if (!A && a.ks == 3) {  // the AdaIN residual blocks of the decoder / prosody predictor
        // (r05) the wide form here too where the wide grid gives every CU two workgroups (a decoder conv at 64
        // utterances: 512 wide tiles): each 9-chunk input row staged once per 256 output channels instead of per 128 --
        // 111 -> 88 us per 1024-channel decoder conv at B = 64; at 32 utterances (256 wide tiles) the narrow form is as
        // fast (56.4 vs 57.5 us), so it stays there (`tools/blk_probe.py` FRAG32=1).  Bit-identical.
        blk_wide = a.ci_pad > 128 && a.co_pad % (2 * BCO) == 0 && wide_tiles >= 2 * stzs_cu_count() &&
                   !(a.flags & STZS_CONV_MRFV_NARROW);
        // 64-row tiles for the narrow block convs below 4 128-row tiles per CU (a decoder conv at 32 utterances: 512
        // tiles; 57.1 -> 55.2 us, the predictor's 256-channel convs 24.4 -> 21.8): more, shorter workgroups per CU
        // hide more of each input chunk's staging latency.  Bit-identical; STZS_MRFV_T64_BLK=N sets the threshold
        // (0: off), STZS_CONV_MRFV_T128 keeps 128 rows.
        static const int t64_blk = [] {
            const char* e = getenv("STZS_MRFV_T64_BLK");
            return e ? atoi(e) : 4;
        }();
        blk_t64 = !blk_wide && t64_blk > 0 && tiles128 < t64_blk * stzs_cu_count() && !(a.flags & STZS_CONV_MRFV_T128);
        if (a.pro_act == STZS_ACT_LEAKY)
            k = blk_wide ? (R ? mrfv_conv<STZS_ACT_LEAKY, true, false, 3, 0, true, 2> : mrfv_conv<STZS_ACT_LEAKY, false, false, 3, 0, true, 2>)
              : blk_t64 ? (R ? mrfv_conv<STZS_ACT_LEAKY, true, false, 3, 0, true, 1, 64> : mrfv_conv<STZS_ACT_LEAKY, false, false, 3, 0, true, 1, 64>)
                         : (R ? mrfv_conv<STZS_ACT_LEAKY, true, false, 3, 0, true> : mrfv_conv<STZS_ACT_LEAKY, false, false, 3, 0, true>);
        else if (a.pro_act == STZS_ACT_NONE)
            k = blk_wide ? (R ? mrfv_conv<STZS_ACT_NONE, true, false, 3, 0, true, 2> : mrfv_conv<STZS_ACT_NONE, false, false, 3, 0, true, 2>)
              : blk_t64 ? (R ? mrfv_conv<STZS_ACT_NONE, true, false, 3, 0, true, 1, 64> : mrfv_conv<STZS_ACT_NONE, false, false, 3, 0, true, 1, 64>)
                         : (R ? mrfv_conv<STZS_ACT_NONE, true, false, 3, 0, true> : mrfv_conv<STZS_ACT_NONE, false, false, 3, 0, true>);
    }
    if (!k) return STZS_ESHAPE;
    const int BTk = (t64 || blk_t64) ? 64 : 128;
    const size_t ldsk = mrfv_lds(BTk + (a.ks - 1) * a.dil);
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)ldsk);
    dim3 grid((unsigned)a.B * (unsigned)((a.T_out + BTk - 1) / BTk), a.co_pad / (wide || blk_wide ? 2 * BCO : BCO));
    hipLaunchKernelGGL(k, grid, dim3(NTH), ldsk, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
