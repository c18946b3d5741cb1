// Predictor glue kernels: per-token style resampling, the integer
// duration head, the alignment scan, the row gather (length regulator), the AdaIN + depthwise
// x2 ConvTranspose of the upsampling AdainResBlk, and the stride-2 F0/N convs of the decoder.
// All are HBM/latency-bound byte work: 16-B vector loads, no MFMA.
#include "common.hpp"

namespace {

template <typename TT>
__global__ __launch_bounds__(256) void pr_prep(const stzs_prprep_args a) {
    const int t = blockIdx.x, b = blockIdx.y, tid = threadIdx.x;
    TT* Y = reinterpret_cast<TT*>(a.y) + (long)b * a.bsy + (long)t * a.ldy;
    const TT* Hs = reinterpret_cast<const TT*>(a.h) + (long)b * a.bsh + (long)t * a.ldh;
    for (int v = tid; v < a.Ch / 8; v += 256) {
        float f[8];
        load8(Hs + v * 8, f);
        store8(Y + v * 8, f);
    }
    // torch upsample_linear1d, align_corners=False (area_pixel_compute_source_index)
    const float ratio = (float)a.L / (float)a.T;
    float src = ratio * ((float)t + 0.5f) - 0.5f;
    if (src < 0.f) src = 0.f;
    const int i0 = (int)src;
    const int i1 = i0 + (i0 < a.L - 1 ? 1 : 0);
    float l1 = src - (float)i0;
    l1 = fminf(fmaxf(l1, 0.f), 1.f);
    const float l0 = 1.f - l1;
    const float* C0 = a.codes + (long)b * a.bsc + (long)i0 * a.ldc + a.c0;
    const float* C1 = a.codes + (long)b * a.bsc + (long)i1 * a.ldc + a.c0;
    for (int c = tid; c < a.Cs; c += 256) DT<TT>::st(Y + a.yc0 + c, l0 * C0[c] + l1 * C1[c]);
}

__global__ __launch_bounds__(256) void dur_kernel(const stzs_dur_args a) {
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)a.B * a.T) return;
    const int b = (int)(i / a.T), t = (int)(i - (long)b * a.T);
    const float* L = a.logits + (long)b * a.bsl + (long)t * a.ldl;
    // 8 logits' loads in flight at a time, the sigmoids summed in bin order (as the one-load-at-a-time loop)
    float acc = 0.f;
    int j = 0;
    for (; j + 8 <= a.nbins; j += 8) {
        float v[8];
#pragma unroll
        for (int u = 0; u < 8; ++u) v[u] = L[j + u];
#pragma unroll
        for (int u = 0; u < 8; ++u) acc = __fadd_rn(acc, 1.f / (1.f + expf(-v[u])));
    }
    for (; j < a.nbins; ++j) acc = __fadd_rn(acc, 1.f / (1.f + expf(-L[j])));
    if (a.dsum) a.dsum[i] = acc;
    int d = (int)rintf(acc);
    if (d < 1) d = 1;
    a.dur[i] = a.override_dur ? a.override_dur[i] : d;
}

__global__ __launch_bounds__(256) void align_kernel(const stzs_align_args a) {
    extern __shared__ int cs[];
    const int b = blockIdx.x;
    const int32_t* D = a.dur + (long)b * a.T;
    if (threadIdx.x == 0) {
        int s = 0;
        cs[0] = 0;
        for (int i = 0; i < a.T; ++i) {
            s += D[i];
            cs[i + 1] = s;
        }
        a.total[b] = s;
    }
    __syncthreads();
    const int tot = cs[a.T];
    for (int f = threadIdx.x; f < a.T40; f += 256) {
        int out = -1;
        if (f < tot) {  // largest i with cs[i] <= f
            int lo = 0, hi = a.T - 1;
            while (lo < hi) {
                const int mid = (lo + hi + 1) >> 1;
                if (cs[mid] <= f) lo = mid; else hi = mid - 1;
            }
            out = lo;
        }
        a.idx[(long)b * a.T40 + f] = out;
    }
}

template <typename T>
__global__ __launch_bounds__(256) void gather_kernel(const stzs_gather_args a) {
    const int f = blockIdx.x, b = blockIdx.y;
    const int src = a.idx[(long)b * a.Tdst + f];
    const T* X = reinterpret_cast<const T*>(a.x) + (long)b * a.bsx + (long)(src < 0 ? 0 : src) * a.ldx + a.xc0;
    T* Y = reinterpret_cast<T*>(a.y) + (long)b * a.bsy + (long)f * a.ldy + a.yc0;
    for (int v = threadIdx.x; v < a.C / 8; v += 256) {
        float x[8];
        if (src >= 0) load8(X + v * 8, x);
        else
            for (int j = 0; j < 8; ++j) x[j] = 0.f;
        store8(Y + v * 8, x);
    }
}

template <typename T>
__global__ __launch_bounds__(256) void dwup_kernel(const stzs_dwup_args a) {
    const int to = blockIdx.x, b = blockIdx.y;
    const int m = to >> 1;
    const bool odd = to & 1;
    const T* X = reinterpret_cast<const T*>(a.x) + (long)b * a.bsx;
    T* Y = reinterpret_cast<T*>(a.y) + (long)b * a.bsy + (long)to * a.ldy;
    for (int c = threadIdx.x; c < a.C; c += 256) {
        const float mu = a.mean[(long)b * a.stat_bs + c], rs = a.rstd[(long)b * a.stat_bs + c];
        const float g = a.gb[(long)b * a.gb_bs + c], be = a.gb[(long)b * a.gb_bs + a.gb_beta_off + c];
        const float sc = (1.f + g) * rs, sh = be - mu * sc;
        float v0 = DT<T>::ld(X + (long)m * a.ldx + c) * sc + sh;
        v0 = v0 >= 0.f ? v0 : v0 * a.slope;
        float o;
        if (!odd) {
            o = v0 * a.w[c * 3 + 1];
        } else {
            float v1 = 0.f;
            if (m + 1 < a.T) {
                v1 = DT<T>::ld(X + (long)(m + 1) * a.ldx + c) * sc + sh;
                v1 = v1 >= 0.f ? v1 : v1 * a.slope;
            }
            o = v1 * a.w[c * 3 + 0] + v0 * a.w[c * 3 + 2];
        }
        DT<T>::st(Y + c, o + a.wb[c]);
    }
}

template <typename TO>
__global__ __launch_bounds__(256) void f0n_kernel(const stzs_f0n_args a) {
    const int T40 = a.T80 / 2;
    const long i = (long)blockIdx.x * 256 + threadIdx.x;
    if (i >= (long)a.B * T40) return;
    const int b = (int)(i / T40), t = (int)(i - (long)b * T40);
    const float* Fp = a.f0 + (long)b * a.ldf;
    const float* Np = a.n + (long)b * a.ldf;
    float of = a.wf[3], on = a.wn[3];
    for (int j = 0; j < 3; ++j) {
        const int s = 2 * t - 1 + j;
        if (s >= 0 && s < a.T80) {
            of += a.wf[j] * Fp[s];
            on += a.wn[j] * Np[s];
        }
    }
    TO* Y0 = reinterpret_cast<TO*>(a.y0) + (long)b * a.bsy0 + (long)t * a.ldy0;
    DT<TO>::st(Y0 + a.cf0, of);
    DT<TO>::st(Y0 + a.cn0, on);
    if (a.y1) {
        TO* Y1 = reinterpret_cast<TO*>(a.y1) + (long)b * a.bsy1 + (long)t * a.ldy1;
        DT<TO>::st(Y1 + a.cf1, of);
        DT<TO>::st(Y1 + a.cn1, on);
    }
}

}  // namespace

extern "C" int stzs_predictor_prep(const stzs_prprep_args* a, void* stream) {
    if (!a || !a->codes || !a->h || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->L <= 0 || a->Ch % 8 || a->ldh % 8 || a->ldy % 8) return STZS_ESHAPE;
    if (a->f32 > 1) return STZS_EINVAL;
    if (a->f32)
        hipLaunchKernelGGL(pr_prep<float>, dim3(a->T, a->B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *a);
    else
        hipLaunchKernelGGL(pr_prep<bf16_t>, dim3(a->T, a->B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_durations(const stzs_dur_args* a, void* stream) {
    if (!a || !a->logits || !a->dur) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->nbins <= 0) return STZS_ESHAPE;
    const long n = (long)a->B * a->T;
    hipLaunchKernelGGL(dur_kernel, dim3((unsigned)((n + 255) / 256)), dim3(256), 0,
                       reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_alignment(const stzs_align_args* a, void* stream) {
    if (!a || !a->dur || !a->idx || !a->total) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->T40 <= 0 || a->T > 16384) return STZS_ESHAPE;
    hipLaunchKernelGGL(align_kernel, dim3(a->B), dim3(256), (a->T + 1) * sizeof(int),
                       reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_gather_rows(const stzs_gather_args* a, void* stream) {
    if (!a || !a->x || !a->idx || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->Tdst <= 0 || a->C % 8 || a->xc0 % 8 || a->yc0 % 8 || a->ldx % 8 || a->ldy % 8)
        return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->dtype == STZS_BF16)
        hipLaunchKernelGGL(gather_kernel<bf16_t>, dim3(a->Tdst, a->B), dim3(256), 0, s, *a);
    else if (a->dtype == STZS_F32)
        hipLaunchKernelGGL(gather_kernel<float>, dim3(a->Tdst, a->B), dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_adain_dwup(const stzs_dwup_args* a, void* stream) {
    if (!a || !a->x || !a->y || !a->mean || !a->rstd || !a->gb || !a->w || !a->wb) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->C <= 0) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->dtype == STZS_BF16)
        hipLaunchKernelGGL(dwup_kernel<bf16_t>, dim3(2 * a->T, a->B), dim3(256), 0, s, *a);
    else if (a->dtype == STZS_F32)
        hipLaunchKernelGGL(dwup_kernel<float>, dim3(2 * a->T, a->B), dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_f0n_down(const stzs_f0n_args* a, void* stream) {
    if (!a || !a->f0 || !a->n || !a->wf || !a->wn || !a->y0) return STZS_EINVAL;
    if (a->B <= 0 || a->T80 <= 0 || a->T80 % 2) return STZS_ESHAPE;
    const long n = (long)a->B * (a->T80 / 2);
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->dtype == STZS_BF16)
        hipLaunchKernelGGL(f0n_kernel<bf16_t>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *a);
    else if (a->dtype == STZS_F32)
        hipLaunchKernelGGL(f0n_kernel<float>, dim3((unsigned)((n + 255) / 256)), dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
