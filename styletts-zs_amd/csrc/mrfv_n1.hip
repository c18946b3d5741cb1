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

mrfv_trio_kfn stzs_mrfv_trio_pick_n1(bool hr) { return hr ? mrfv_trio<true, 1, 64> : mrfv_trio<false, 1, 64>; }

#ifdef STZS_MRFV_PROF
// (probe build only) the stage-1 instances' phase stamps -> host; zero: clear them after the copy
extern "C" int stzs_mrfv_prof_read(unsigned long long* host, size_t n, int zero) {
    void* p = nullptr;
    if (hipGetSymbolAddress(&p, HIP_SYMBOL(g_mprof)) != hipSuccess) return -1;
    if (hipDeviceSynchronize() != hipSuccess) return -1;
    if (host && hipMemcpy(host, p, n * 8, hipMemcpyDeviceToHost) != hipSuccess) return -1;
    if (zero && hipMemset(p, 0, sizeof(unsigned long long) * 8 * 16384) != hipSuccess) return -1;
    return 0;
}
#endif
