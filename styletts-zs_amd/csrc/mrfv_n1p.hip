// The stage-1 generator MRF convs as tile runs (mrfv_kernel.hpp PT): one workgroup per run of consecutive 128-row
// tiles of one utterance, the next tile's rows loaded under the current tile's K loop.  Built like csrc/mrfv_n1.hip
// (no packed-fp32 VALU ops, styletts-zs_amd/build.py FILE_FLAGS); bit-identical to the one-tile forms.
#include "mrfv_kernel.hpp"

mrfv_kfn stzs_mrfv_pick_n1_run(int ks, bool hr, bool ha, bool al) {
#define STZS_N1P(HR, HA) \
    if (hr == HR && ha == HA) \
        return al ? pick_ks<STZS_ACT_SNAKE, HR, HA, 1, true, 1, 128, true>(ks) : pick_ks<STZS_ACT_SNAKE, HR, HA, 1, false, 1, 128, true>(ks);
    STZS_N1P(false, false)
    STZS_N1P(true, false)
    STZS_N1P(false, true)
    STZS_N1P(true, true)
#undef STZS_N1P
    return nullptr;
}
