// Reference-prompt front end in HIP (log-mel + prompt encoder), so that a whole
// synth() runs on libstzs_hip.so kernels only.  The oracle's restatement: oracle/stzs_ref.py prompt_encoder
// (torch.stft center=True / reflect pad, periodic Hann window of win samples centred in n_fft, power,
// HTK mel filterbank, log(clamp(., 1e-5)), two k5 convs + LeakyReLU(0.2), adaptive average pooling to L_s
// rows, projection).
//
//   stzs_stft_frames : reflect-padded, windowed frames as bf16 GEMM rows [B, F, ldy] (HBM-bound copy);
//                      the DFT itself is a bf16 MFMA GEMM through stzs_conv1d against a cos | -sin basis
//                      (stzs/weights.py dft_basis), fp32 out;
//   stzs_log_mel     : |X|^2 of the (re | im) rows, sparse mel filterbank (per-bin [k0, k1) ranges), log;
//   stzs_pool_rows   : adaptive average pooling over time (torch.nn.functional.adaptive_avg_pool1d bounds);
//   stzs_code_quantize: the discrete style codes (README.md:5) -- product VQ of the projected prompt rows.
#include "common.hpp"

namespace {

__global__ __launch_bounds__(256) void frames_kernel(const stzs_frames_args a) {
    const int t = blockIdx.x, b = blockIdx.y;
    const float* X = a.wav + (long)b * a.ldw;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y) + (long)b * a.bsy + (long)t * a.ldy;
    const int off = (a.n_fft - a.win) / 2;  // window centred in the n_fft frame
    for (int m = threadIdx.x; m < a.ldy; m += 256) {
        float v = 0.f;
        if (m < a.win) {
            long j = (long)t * a.hop + off + m - a.n_fft / 2;  // sample index before reflect padding
            if (j < 0) j = -j;
            if (j >= a.N) j = 2L * (a.N - 1) - j;
            v = a.window[m] * X[j];
        }
        Y[m] = f2bf(v);
    }
}

__global__ __launch_bounds__(256) void log_mel_kernel(const stzs_logmel_args a) {
    extern __shared__ float pw[];
    const long r = (long)blockIdx.y * a.F + blockIdx.x;  // b * F + t
    const float* S = a.spec + (long)blockIdx.y * a.bss + (long)blockIdx.x * a.lds;
    for (int k = threadIdx.x; k < a.nbin; k += 256) {
        const float re = S[k], im = S[a.nbin + k];
        pw[k] = re * re + im * im;
    }
    __syncthreads();
    for (int m = threadIdx.x; m < a.n_mels; m += 256) {
        const int k0 = a.ranges[2 * m], k1 = a.ranges[2 * m + 1];
        const float* w = a.fb + (long)m * a.nbin;
        float acc = 0.f;
        for (int k = k0; k < k1; ++k) acc = fmaf(w[k], pw[k], acc);
        const float v = logf(fmaxf(acc, 1e-5f));
        const long o = (long)blockIdx.y * a.bsy + (long)blockIdx.x * a.ldy + m;
        if (a.out_dtype == STZS_BF16) reinterpret_cast<bf16_t*>(a.y)[o] = f2bf(v);
        else reinterpret_cast<float*>(a.y)[o] = v;
    }
    (void)r;
}

template <typename TI, typename TO>
__global__ __launch_bounds__(256) void pool_kernel(const stzs_pool_args a) {
    const int i = blockIdx.x, b = blockIdx.y;
    const int s = (int)(((long)i * a.T) / a.L);
    const int e = (int)(((long)(i + 1) * a.T + a.L - 1) / a.L);
    const TI* X = reinterpret_cast<const TI*>(a.x) + (long)b * a.bsx;
    TO* Y = reinterpret_cast<TO*>(a.y) + (long)b * a.bsy + (long)i * a.ldy;
    const float inv = 1.f / (float)(e - s);
    for (int c = threadIdx.x; c < a.C; c += 256) {
        float acc = 0.f;
        for (int t = s; t < e; ++t) acc += DT<TI>::ld(X + (long)t * a.ldx + c);
        DT<TO>::st(Y + c, acc * inv);
    }
}

// One workgroup per (64 rows, group): the group's codebook (K x DG fp32, <= 64 KB) is staged in LDS once, and
// the K entries are split over the 4 waves (wave w scans [w K/4, (w+1) K/4) for its lane's row: every lane of a
// wave reads the same entry -> LDS broadcast).  The distance is summed serially with explicitly rounded sub / mul /
// add (the oracle's order); strict < keeps the first minimum inside a range, and the 4 range minima are combined
// in range order with strict <, so the result is the first global minimum -- the serial scan's, bit for bit.
// (One lane scanning all K from scalar loads was latency-bound: 52 us for the 50 x 32 (row, group) pairs of a
// batch-1 prompt.)
constexpr int VQ_WAVES = 4;
template <int DG>
__global__ __launch_bounds__(64 * VQ_WAVES) void vq_kernel(const stzs_vq_args a) {
    extern __shared__ __attribute__((aligned(16))) float cbs[];  // [K][DG], then [VQ_WAVES][64] (d, k) pairs
    const int lane = threadIdx.x & 63, w = threadIdx.x >> 6;
    const int r = blockIdx.x * 64 + lane, g = blockIdx.y;
    const float* cb = a.codebook + (long)g * a.K * DG;
    const bool row_ok = r < a.R;
    if (a.lookup) {
        if (w != 0 || !row_ok) return;  // (no barrier on this path)
        const int best = min(max(a.idx[(long)r * a.ldi + g], 0), a.K - 1);
        const float* c = cb + (long)best * DG;
        float* Y = a.y + (long)r * a.ldy + g * DG;
#pragma unroll
        for (int j = 0; j < DG; ++j) Y[j] = c[j];
        return;
    }
    for (int e = threadIdx.x; e < a.K * DG; e += 64 * VQ_WAVES) cbs[e] = cb[e];
    float x[DG];
    const float* X = a.x + (long)(row_ok ? r : 0) * a.ldx + g * DG;
#pragma unroll
    for (int j = 0; j < DG; ++j) x[j] = X[j];
    __syncthreads();
    const int per = (a.K + VQ_WAVES - 1) / VQ_WAVES;
    const int k0 = w * per, k1 = min(a.K, k0 + per);
    float bd = __builtin_inff();
    int best = k0 < k1 ? k0 : 0;
    for (int k = k0; k < k1; ++k) {
        const float* c = cbs + k * DG;
        float d = 0.f;
#pragma unroll
        for (int j = 0; j < DG; ++j) {
            const float t = __fsub_rn(x[j], c[j]);
            d = __fadd_rn(d, __fmul_rn(t, t));
        }
        if (d < bd) {
            bd = d;
            best = k;
        }
    }
    float* pd = cbs + a.K * DG;
    int* pk = reinterpret_cast<int*>(pd + VQ_WAVES * 64);
    pd[w * 64 + lane] = bd;
    pk[w * 64 + lane] = best;
    __syncthreads();
    if (w != 0 || !row_ok) return;
    float gd = pd[lane];
    int gb = pk[lane];
#pragma unroll
    for (int q = 1; q < VQ_WAVES; ++q)
        if (pd[q * 64 + lane] < gd) {
            gd = pd[q * 64 + lane];
            gb = pk[q * 64 + lane];
        }
    a.idx[(long)r * a.ldi + g] = gb;
    const float* c = cbs + gb * DG;
    float* Y = a.y + (long)r * a.ldy + g * DG;
#pragma unroll
    for (int j = 0; j < DG; ++j) Y[j] = c[j];
}

}  // namespace

extern "C" int stzs_code_quantize(const stzs_vq_args* a, void* stream) {
    if (!a || !a->codebook || !a->idx || !a->y || (!a->lookup && !a->x)) return STZS_EINVAL;
    if (a->R <= 0 || a->G <= 0 || a->K <= 0 || a->ldi < a->G || a->ldy < (long)a->G * a->dg ||
        (!a->lookup && a->ldx < (long)a->G * a->dg))
        return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g((a->R + 63) / 64, a->G);
    const size_t lds = (size_t)a->K * a->dg * 4 + VQ_WAVES * 64 * 8;
    if (lds > 64 * 1024) return STZS_ESHAPE;  // codebook of one group staged in LDS
    switch (a->dg) {
        case 4: hipLaunchKernelGGL(vq_kernel<4>, g, dim3(64 * VQ_WAVES), lds, s, *a); break;
        case 8: hipLaunchKernelGGL(vq_kernel<8>, g, dim3(64 * VQ_WAVES), lds, s, *a); break;
        case 16: hipLaunchKernelGGL(vq_kernel<16>, g, dim3(64 * VQ_WAVES), lds, s, *a); break;
        default: return STZS_ESHAPE;
    }
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_stft_frames(const stzs_frames_args* a, void* stream) {
    if (!a || !a->wav || !a->window || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->N < 2 || a->F <= 0 || a->hop <= 0 || a->win <= 0 || a->win > a->n_fft || a->ldy < a->win ||
        a->ldy % 8 || a->n_fft / 2 >= a->N)
        return STZS_ESHAPE;  // reflect padding needs N > n_fft / 2 (as torch)
    if ((long)(a->F - 1) * a->hop > (long)a->N + a->n_fft) return STZS_ESHAPE;
    hipLaunchKernelGGL(frames_kernel, dim3(a->F, a->B), dim3(256), 0, reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_log_mel(const stzs_logmel_args* a, void* stream) {
    if (!a || !a->spec || !a->y || !a->fb || !a->ranges) return STZS_EINVAL;
    if (a->B <= 0 || a->F <= 0 || a->nbin <= 0 || a->nbin > 8192 || a->n_mels <= 0 || a->lds < 2 * a->nbin ||
        a->ldy < a->n_mels)
        return STZS_ESHAPE;
    if (a->out_dtype != STZS_BF16 && a->out_dtype != STZS_F32) return STZS_EDTYPE;
    hipLaunchKernelGGL(log_mel_kernel, dim3(a->F, a->B), dim3(256), (size_t)a->nbin * 4,
                       reinterpret_cast<hipStream_t>(stream), *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

extern "C" int stzs_pool_rows(const stzs_pool_args* a, void* stream) {
    if (!a || !a->x || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->L <= 0 || a->C <= 0) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g(a->L, a->B);
    if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((pool_kernel<bf16_t, bf16_t>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_BF16 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((pool_kernel<bf16_t, float>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_F32)
        hipLaunchKernelGGL((pool_kernel<float, float>), g, dim3(256), 0, s, *a);
    else if (a->in_dtype == STZS_F32 && a->out_dtype == STZS_BF16)
        hipLaunchKernelGGL((pool_kernel<float, bf16_t>), g, dim3(256), 0, s, *a);
    else
        return STZS_EDTYPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
