// Harmonic source of the iSTFT decoder: NSF SineGen from F0, counter-RNG
// noise, Linear(9->1) + tanh merge, and its n_fft-point STFT (real | imag) feeding noise_convs.
//
// Phase accuracy (SURVEY §7 "SineGen phase cumsum drifts in fp32"): a per-(utterance, harmonic)
// thread accumulates the frame-rate phase prefix in fp64 and wraps it every 80-fps frame; the
// in-frame phase is then prefix + (j+1) * f/sr in fp32 (|arg| < 60 cycles, so < 4e-6 cycles of
// error).  Every fp32/fp64 op that must agree bit-for-bit with the oracle uses explicit _rn
// intrinsics (no FMA contraction).  Samples are generated once per workgroup into LDS
// (reflect-padded at the ends, centre=True) and consumed by all frames that overlap them; the
// per-frame phase increments and prefixes of the few frames a workgroup spans sit in LDS.  Sine and
// the noise's Box-Muller use the hardware transcendentals (v_sin / v_cos in revolutions, v_log):
// the counter stream is the oracle's, the transform within ~1e-6 of its fp64 one.
#include "common.hpp"

namespace {

STZS_DEV uint32_t hash32(uint32_t x) {
    x ^= x >> 16;
    x *= 0x7FEB352Du;
    x ^= x >> 15;
    x *= 0x846CA68Bu;
    x ^= x >> 16;
    return x;
}
STZS_DEV uint32_t stream_key(uint32_t seed, uint32_t stream) {
    return hash32(hash32(seed + 0x9E3779B9u) ^ stream);
}
STZS_DEV float counter_normal(uint32_t key, uint32_t idx) {
    const uint32_t a = hash32(key ^ hash32(idx * 2u));
    const uint32_t b = hash32(key ^ hash32(idx * 2u + 1u));
    const double u1 = ((double)(a >> 8) + 1.0) * (1.0 / 16777216.0);
    const double u2 = (double)(b >> 8) * (1.0 / 16777216.0);
    return (float)(sqrt(-2.0 * log(u1)) * cos(6.283185307179586 * u2));
}
// the same counter pair as counter_normal, Box-Muller in fp32 hardware intrinsics (v_log_f32,
// v_sqrt_f32, v_cos_f32 in revolutions): within ~2e-6 of the fp64 transform (tests/test_gpu_ops.py).
// hi0 = hash32(2 idx), hi1 = hash32(2 idx + 1): the counter hashes do not depend on the stream key, so a sample's
// harmonics share them (the same values as counter_normal computes)
STZS_DEV float counter_normal_fast(uint32_t key, uint32_t hi0, uint32_t hi1) {
    const uint32_t a = hash32(key ^ hi0);
    const uint32_t b = hash32(key ^ hi1);
    const float u1 = ((float)(a >> 8) + 1.f) * (1.f / 16777216.f);
    const float u2 = (float)(b >> 8) * (1.f / 16777216.f);
    return __builtin_sqrtf(-1.3862943611198906f * __builtin_amdgcn_logf(u1)) * __builtin_amdgcn_cosf(u2);
}
STZS_DEV float initial_phase(uint32_t key) {
    return (float)((double)(hash32(key ^ 0xA5A5A5A5u) >> 8) * (1.0 / 16777216.0));
}

// One workgroup per (utterance, harmonic): the per-frame phase increments hop * (f0 (h + 1) / sr) -- the fp64
// division is the expensive part -- are computed for a chunk of frames by all 256 threads into LDS, then one lane
// runs the dependent chain acc = frac(acc + d_k) over the chunk.  The same fp64 operations in the same order as
// the one-thread-per-(b, h) loop it replaces (which ran 9 lanes of one wave at batch 1: 71 us), so bit-identical.
constexpr int PP_CHUNK = 1024;
__global__ __launch_bounds__(256) void phase_prefix_kernel(const stzs_source_args a) {
    __shared__ double d[PP_CHUNK];
    const int i = blockIdx.x;  // (b, h)
    const int b = i / a.nh, h = i - b * a.nh;
    const float* F = a.f0 + (long)b * a.ldf;
    float* P = a.prefix + (long)i * a.T80;
    double acc = 0.0;
    for (int k0 = 0; k0 < a.T80; k0 += PP_CHUNK) {
        const int n = min(PP_CHUNK, a.T80 - k0);
        __syncthreads();
        for (int k = threadIdx.x; k < n; k += 256) {
            const double inc = __ddiv_rn(__dmul_rn((double)F[k0 + k], (double)(h + 1)), (double)a.sr);
            d[k] = __dmul_rn((double)a.hop, inc);
        }
        __syncthreads();
        if (threadIdx.x == 0) {
            for (int k = 0; k < n; ++k) {
                P[k0 + k] = (float)acc;
                acc = __dadd_rn(acc, d[k]);
                acc = acc - floor(acc);
            }
        }
    }
}

constexpr int FB = 256;  // STFT frames per workgroup
constexpr int KW = 8;    // 80-fps frames spanned by one workgroup's samples (checked on the host)

// NFFT > 0: the transform size at compile time (twiddles and window in registers, the STFT sums fully unrolled);
// 0: any size (runtime loops over the LDS tables).  The same products summed in the same order either way.
template <int NFFT>
__global__ __launch_bounds__(256) void source_stft_kernel(const stzs_source_args a) {
    extern __shared__ float sm[];
    const int nfft = NFFT ? NFFT : a.n_fft, hs = a.hop_s, nb = nfft / 2 + 1;
    const int NS = hs * (FB - 1) + nfft;
    float* sbuf = sm;                 // NS samples
    float* twc = sbuf + NS;           // nfft cos
    float* tws = twc + nfft;          // nfft sin
    float* win = tws + nfft;          // nfft hann
    uint32_t* keys = reinterpret_cast<uint32_t*>(win + nfft);  // nh
    float* ph0 = reinterpret_cast<float*>(keys + a.nh);        // nh
    float* finc = ph0 + a.nh;                                   // [KW][nh] per-frame phase increment
    float* fpre = finc + KW * a.nh;                             // [KW][nh] per-frame phase prefix + ph0
    float* mw = fpre + KW * a.nh;                               // nh merge weights
    const int b = blockIdx.y, f0i = blockIdx.x * FB, tid = threadIdx.x;
    const int N = a.T80 * a.hop;
    const int Tf = N / hs + 1;
    if (tid < nfft) {
        const double ang = 2.0 * 3.141592653589793 * tid / nfft;
        twc[tid] = (float)cos(ang);
        tws[tid] = (float)sin(ang);
        win[tid] = (float)(0.5 - 0.5 * cos(ang));
    }
    if (tid < a.nh) {
        const uint32_t key = stream_key(a.seeds[b], (uint32_t)tid);
        keys[tid] = key;
        ph0[tid] = tid == 0 ? 0.f : initial_phase(key);
        mw[tid] = a.merge_w[tid];
    }
    __syncthreads();
    const float* F = a.f0 + (long)b * a.ldf;
    const float* P = a.prefix + (long)b * a.nh * a.T80;
    // the <= KW 80-fps frames this workgroup's samples fall in (reflection maps into them as well)
    const int nlo = max(f0i * hs - nfft / 2, 0), nhi = min(f0i * hs - nfft / 2 + NS - 1, N - 1);
    const int k_lo = nlo / a.hop, nk = nhi / a.hop - k_lo + 1;
    for (int e = tid; e < nk * a.nh; e += 256) {
        const int kk = e / a.nh, h = e - kk * a.nh, k = k_lo + kk;
        finc[kk * a.nh + h] = __fdiv_rn(__fmul_rn(F[k], (float)(h + 1)), a.sr);
        fpre[kk * a.nh + h] = __fadd_rn(P[(long)h * a.T80 + k], ph0[h]);
    }
    __syncthreads();
    const float amp = a.sine_amp, amp3 = __fdiv_rn(a.sine_amp, 3.0f);
    const float wb = a.merge_w[a.nh];
    for (int p = tid; p < NS; p += 256) {
        int n = (f0i * hs + p) - nfft / 2;  // centre=True: padded index -> signal index
        if (n < 0) n = -n;
        if (n >= N) n = 2 * (N - 1) - n;
        float v = 0.f;
        if (n >= 0 && n < N) {
            const int k = n / a.hop, kk = k - k_lo;
            const float jj = (float)(n - k * a.hop + 1);
            const bool voiced = F[k] > a.voiced_thr;
            const float uv = voiced ? 1.f : 0.f;
            const float namp = voiced ? a.noise_std : amp3;
            const float* fi = finc + kk * a.nh;
            const float* fp = fpre + kk * a.nh;
            const uint32_t hi0 = hash32((uint32_t)n * 2u), hi1 = hash32((uint32_t)n * 2u + 1u);
            float acc = 0.f;
            for (int h = 0; h < a.nh; ++h) {
                const float t = __fadd_rn(fp[h], __fmul_rn(jj, fi[h]));
                const float th = __fsub_rn(t, floorf(t));  // wrapped phase, cycles
                const float sine = amp * __builtin_amdgcn_sinf(th);
                const float z = counter_normal_fast(keys[h], hi0, hi1);
                acc = fmaf(mw[h], fmaf(sine, uv, namp * z), acc);
            }
            const float xx = acc + wb;
            v = 1.f - 2.f * __builtin_amdgcn_rcpf(1.f + __expf(2.f * xx));  // tanh
        }
        sbuf[p] = v;
    }
    __syncthreads();
    const int f = f0i + tid;
    if (tid < FB && f < Tf) {
        const float* s = sbuf + tid * hs;
        const bool f32 = a.har_dtype == STZS_F32;
        bf16_t* Hh = reinterpret_cast<bf16_t*>(a.har) + (long)b * a.bsh + (long)f * a.ldh;
        float* Hf = reinterpret_cast<float*>(a.har) + (long)b * a.bsh + (long)f * a.ldh;
        if constexpr (NFFT > 0) {
            constexpr int NB = NFFT / 2 + 1;
            float tc[NFFT], ts[NFFT], x[NFFT];
#pragma unroll
            for (int i = 0; i < NFFT; ++i) {
                tc[i] = twc[i];
                ts[i] = tws[i];
                x[i] = s[i] * win[i];
            }
            float re[NB], im[NB];
#pragma unroll
            for (int kb = 0; kb < NB; ++kb) {
                float r = 0.f, q = 0.f;
#pragma unroll
                for (int i = 0; i < NFFT; ++i) {
                    const int m = (kb * i) % NFFT;
                    r += x[i] * tc[m];
                    q -= x[i] * ts[m];
                }
                re[kb] = r;
                im[kb] = q;
            }
            if (f32) {
#pragma unroll
                for (int kb = 0; kb < NB; ++kb) {
                    Hf[kb] = re[kb];
                    Hf[NB + kb] = im[kb];
                }
            } else {
#pragma unroll
                for (int kb = 0; kb < NB; ++kb) {
                    Hh[kb] = f2bf(re[kb]);
                    Hh[NB + kb] = f2bf(im[kb]);
                }
            }
        } else {
            for (int kb = 0; kb < nb; ++kb) {
                float re = 0.f, im = 0.f;
                for (int i = 0; i < nfft; ++i) {
                    const int m = (kb * i) % nfft;
                    const float x = s[i] * win[i];
                    re += x * twc[m];
                    im -= x * tws[m];
                }
                if (f32) {
                    Hf[kb] = re;
                    Hf[nb + kb] = im;
                } else {
                    Hh[kb] = f2bf(re);
                    Hh[nb + kb] = f2bf(im);
                }
            }
        }
        for (int c = 2 * nb; c < a.ldh; ++c) {
            if (f32) Hf[c] = 0.f;
            else Hh[c] = 0;
        }
    }
}

}  // namespace

extern "C" int stzs_harmonic_source(const stzs_source_args* a, void* stream) {
    if (!a || !a->f0 || !a->seeds || !a->merge_w || !a->prefix || !a->har) return STZS_EINVAL;
    if (a->B <= 0 || a->T80 <= 0 || a->nh <= 0 || a->nh > 64 || a->n_fft <= 0 || a->n_fft > 64 || a->hop_s <= 0)
        return STZS_ESHAPE;
    if (a->ldh < 2 * (a->n_fft / 2 + 1)) return STZS_ESHAPE;
    if (a->har_dtype != STZS_BF16 && a->har_dtype != STZS_F32) return STZS_EDTYPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int n = a->B * a->nh;
    hipLaunchKernelGGL(phase_prefix_kernel, dim3(n), dim3(256), 0, s, *a);
    STZS_LAUNCH_CHECK();
    const int N = a->T80 * a->hop;
    const int Tf = N / a->hop_s + 1;
    const int NS = a->hop_s * (FB - 1) + a->n_fft;
    if (NS / a->hop + 2 > KW) return STZS_ESHAPE;
    const size_t lds = (size_t)(NS + 3 * a->n_fft) * 4 + (size_t)a->nh * (8 + 4 + 2 * KW * 4);
    if (a->n_fft == 20)
        hipLaunchKernelGGL(source_stft_kernel<20>, dim3((Tf + FB - 1) / FB, a->B), dim3(256), lds, s, *a);
    else
        hipLaunchKernelGGL(source_stft_kernel<0>, dim3((Tf + FB - 1) / FB, a->B), dim3(256), lds, s, *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
