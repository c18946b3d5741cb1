// Host shim for the two-shard root-cause bisection (tools/pk_bisect.py): loads one code-object
// variant of csrc/source.hip (tools/probe/pk_variants.py) with hipModuleLoad and launches it exactly as
// stzs_harmonic_source does (same grid, block, dynamic LDS), so an engine twin can swap only this kernel.
#include <hip/hip_runtime.h>
#include "stzs.h"

static hipModule_t mod;
static hipFunction_t f_prefix, f_stft;

extern "C" int shim_load(const char* path) {
    if (hipModuleLoad(&mod, path) != hipSuccess) return -1;
    if (hipModuleGetFunction(&f_prefix, mod, "_ZN12_GLOBAL__N_119phase_prefix_kernelE16stzs_source_args") != hipSuccess)
        return -2;
    if (hipModuleGetFunction(&f_stft, mod, "_ZN12_GLOBAL__N_118source_stft_kernelILi20EEEv16stzs_source_args") !=
        hipSuccess)
        return -3;
    return 0;
}

extern "C" int shim_harmonic_source(const stzs_source_args* a, void* stream) {
    if (!f_stft || a->n_fft != 20) return STZS_EINVAL;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    stzs_source_args arg = *a;
    void* params[] = {&arg};
    if (hipModuleLaunchKernel(f_prefix, a->B * a->nh, 1, 1, 256, 1, 1, 0, s, params, nullptr) != hipSuccess)
        return STZS_EHIP;
    const int FB = 256;
    const int N = a->T80 * a->hop, Tf = N / a->hop_s + 1, NS = a->hop_s * (FB - 1) + a->n_fft, KW = 8;
    const size_t lds = (size_t)(NS + 3 * a->n_fft) * 4 + (size_t)a->nh * (8 + 4 + 2 * KW * 4);
    if (hipModuleLaunchKernel(f_stft, (Tf + FB - 1) / FB, a->B, 1, 256, 1, 1, (unsigned)lds, s, params, nullptr) !=
        hipSuccess)
        return STZS_EHIP;
    return STZS_OK;
}
