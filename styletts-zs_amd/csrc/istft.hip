// iSTFT head of the decoder: spec = exp(m) * exp(i * sin(p)) per bin,
// n_fft-point irfft, periodic Hann synthesis window, overlap-add with hop_s, centre trim and the
// window-square envelope normalisation of torch.istft.  fp32 throughout.
// One workgroup per 256 frames: the 256 + 3 frame signals overlapping its output span are
// synthesised once into LDS, then each thread overlap-adds its output samples (4 frames each).
// HBM-bound: reads n_fft+2 floats per frame, writes hop_s samples per frame.
#include "common.hpp"

namespace {

constexpr int FB = 256;

template <int NFFT>
__global__ __launch_bounds__(256) void istft_kernel(const stzs_istft_args a) {
    extern __shared__ float sm[];
    constexpr int nfft = NFFT, nb = NFFT / 2 + 1;
    const int hs = a.hop_s;
    const int halo = (nfft + hs - 1) / hs - 1;  // frames before the block that reach its samples
    const int NF = FB + halo;
    float* fr = sm;                  // NF * nfft windowed frame signals
    float* twc = fr + NF * nfft;
    float* tws = twc + nfft;
    float* win = tws + nfft;
    const int b = blockIdx.y, f0i = blockIdx.x * FB, tid = threadIdx.x;
    if (tid < nfft) {
        const double ang = 2.0 * 3.141592653589793 * tid / nfft;
        twc[tid] = (float)cos(ang);
        tws[tid] = (float)sin(ang);
        win[tid] = (float)(0.5 - 0.5 * cos(ang));
    }
    __syncthreads();
    const float* Pp = a.post + (long)b * a.bsp;
    for (int q = tid; q < NF; q += 256) {
        const int f = f0i - halo + q;
        float* o = fr + q * nfft;
        if (f < 0 || f >= a.Tf) {
            for (int i = 0; i < nfft; ++i) o[i] = 0.f;
            continue;
        }
        const float* row = Pp + (long)f * a.ldp;
        float re[nb], im[nb];
#pragma unroll
        for (int k = 0; k < nb; ++k) {
            const float mag = expf(row[k]);
            const float ph = sinf(row[nb + k]);
            re[k] = mag * cosf(ph);
            im[k] = mag * sinf(ph);
        }
#pragma unroll
        for (int i = 0; i < nfft; ++i) {
            float x = re[0] + ((i & 1) ? -re[nb - 1] : re[nb - 1]);
            float acc = 0.f;
#pragma unroll
            for (int k = 1; k < nb - 1; ++k) {
                const int m = (k * i) % nfft;
                acc += re[k] * twc[m] - im[k] * tws[m];
            }
            x = (x + 2.f * acc) / (float)nfft;
            o[i] = x * win[i];
        }
    }
    __syncthreads();
    const int Nout = (a.Tf - 1) * hs;
    float* W = a.wav + (long)b * a.bsw;
    for (int s = tid; s < FB * hs; s += 256) {
        const int m = f0i * hs + s;       // padded sample index
        const int n = m - nfft / 2;       // output sample index (centre trim)
        if (n < 0 || n >= Nout) continue;
        float y = 0.f, env = 0.f;
        int fhi = m / hs;
        if (fhi > a.Tf - 1) fhi = a.Tf - 1;
        for (int f = fhi; f >= 0 && m - f * hs < nfft; --f) {
            const int i = m - f * hs;
            const int q = f - (f0i - halo);
            y += fr[q * nfft + i];
            env += win[i] * win[i];
        }
        W[n] = y / env;
    }
}

}  // namespace

extern "C" int stzs_istft(const stzs_istft_args* a, void* stream) {
    if (!a || !a->post || !a->wav) return STZS_EINVAL;
    if (a->B <= 0 || a->Tf < 2 || a->n_fft <= 0 || a->n_fft > 64 || a->n_fft % 2 || a->hop_s <= 0 ||
        a->ldp < a->n_fft + 2)
        return STZS_ESHAPE;
    const int halo = (a->n_fft + a->hop_s - 1) / a->hop_s - 1;
    const size_t lds = (size_t)((FB + halo) * a->n_fft + 3 * a->n_fft) * 4;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g((a->Tf + FB - 1) / FB, a->B);
    if (a->n_fft == 20)
        hipLaunchKernelGGL(istft_kernel<20>, g, dim3(256), lds, s, *a);
    else if (a->n_fft == 16)
        hipLaunchKernelGGL(istft_kernel<16>, g, dim3(256), lds, s, *a);
    else
        return STZS_ESHAPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
