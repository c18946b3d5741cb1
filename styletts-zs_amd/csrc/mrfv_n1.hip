// The stage-1 generator MRF convs (single 128-channel input chunk, Snake prologue): the NCH = 1
// instances of csrc/mrfv_kernel.hpp, in a translation unit of their own so they are built without packed-fp32 VALU ops
// (styletts-zs_amd/build.py FILE_FLAGS): same arithmetic per lane (v_pk_fma_f32 is two fmas), so bit-identical.
#include "mrfv_kernel.hpp"

mrfv_kfn stzs_mrfv_pick_n1(int ks, bool hr, bool ha, bool al, bool t64) {
#define STZS_N1(HR, HA) \
    if (hr == HR && ha == HA) { \
        if (t64) return al ? pick_ks<STZS_ACT_SNAKE, HR, HA, 1, true, 1, 64>(ks) : pick_ks<STZS_ACT_SNAKE, HR, HA, 1, false, 1, 64>(ks); \
        return al ? pick_ks<STZS_ACT_SNAKE, HR, HA, 1, true>(ks) : pick_ks<STZS_ACT_SNAKE, HR, HA, 1, false>(ks); \
    }
    STZS_N1(false, false)
    STZS_N1(true, false)
    STZS_N1(false, true)
    STZS_N1(true, true)
#undef STZS_N1
    return nullptr;
}
