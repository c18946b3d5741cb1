// iSTFT head of the decoder: spec = exp(m) * exp(i * sin(p)) per bin,
// n_fft-point irfft, periodic Hann synthesis window, overlap-add with hop_s, centre trim and the
// window-square envelope normalisation of torch.istft.  fp32 throughout.
//
// ONE kernel serves both the whole-utterance call (stzs_istft) and the streaming call
// (stzs_istft_stream, row a14): the whole utterance is the single chunk [0, Tf) with final = 1.  A
// chunk emits exactly the output samples whose overlapping frames are all known (padded sample m
// with m < (f0 + Fc) * hop, or every remaining sample on the final chunk); the frames before the
// chunk that still reach its samples (halo = ceil(n_fft / hop) - 1 = 3 at 20/5) come from the
// carried tail of raw frame rows.  Every sample is summed over its frames in the same (descending)
// order with the same frame synthesis code in both modes, so concatenated chunks are BIT-identical
// to the whole-utterance output (tests/test_gpu_stream.py).
//
// Work split: one workgroup per 256 - halo frames of the chunk, so the 256 frame signals overlapping its output span
// (its own + the halo) are synthesised once into LDS by the 256 threads in ONE pass (256 own frames + 3 halo took a
// second pass for 3 threads, i.e. the whole workgroup twice as long), then each thread overlap-adds its output
// samples.  Spectrum from the hardware transcendentals (v_exp / v_sin / v_cos, ~1e-6 relative; the libm forms' range
// reduction was most of the frame synthesis).  HBM-bound: reads n_fft + 2 floats per frame, writes hop_s samples.
#include "common.hpp"

namespace {

constexpr int NF = 256;  // frame signals per workgroup (its frames + the halo)

struct IstftJob {
    const float* post;     // row j = frame f0 + j
    const float* tail_in;  // [B][halo][ldt], row i = frame f0 - halo + i
    float* tail_out;       // [B][halo][ldt], row i = frame f0 + Fc - halo + i
    float* wav;            // wav[b * bsw + n - n0]
    long ldp, bsp, bsw, ldt, n0, m_end;  // m_end: exclusive padded-sample bound of the chunk
    int B, f0, Fc, hs;
};

STZS_DEV int halo_of(int nfft, int hs) { return (nfft + hs - 1) / hs - 1; }

template <int NFFT>
__global__ __launch_bounds__(256) void istft_kernel(const IstftJob a) {
    extern __shared__ float sm[];
    constexpr int nfft = NFFT, nb = NFFT / 2 + 1;
    const int hs = a.hs;
    const int halo = halo_of(nfft, hs);
    const int FB = NF - halo;        // frames of this workgroup
    float* fr = sm;                  // NF * nfft windowed frame signals
    float* twc = fr + NF * nfft;
    float* tws = twc + nfft;
    float* win = tws + nfft;
    const int b = blockIdx.y, tid = threadIdx.x;
    const int fb0 = a.f0 + blockIdx.x * FB;  // absolute first frame of this block
    const int flast = a.f0 + a.Fc - 1;       // last frame of the chunk
    if (tid < nfft) {
        const double ang = 2.0 * 3.141592653589793 * tid / nfft;
        twc[tid] = (float)cos(ang);
        tws[tid] = (float)sin(ang);
        win[tid] = (float)(0.5 - 0.5 * cos(ang));
    }
    const float* Pp = a.post + (long)b * a.bsp;
    const float* Tp = a.tail_in ? a.tail_in + (long)b * halo * a.ldt : nullptr;
    // carried tail for the next chunk: raw rows of the chunk's last `halo` frames (block 0 writes it)
    if (a.tail_out && blockIdx.x == 0) {
        float* To = a.tail_out + (long)b * halo * a.ldt;
        for (int e = tid; e < halo * (nfft + 2); e += 256) {
            const int i = e / (nfft + 2), c = e - i * (nfft + 2);
            const int f = a.f0 + a.Fc - halo + i;
            float v = 0.f;
            if (f >= a.f0) v = Pp[(long)(f - a.f0) * a.ldp + c];
            else if (f >= 0 && Tp) v = Tp[(long)(a.Fc + i) * a.ldt + c];
            To[(long)i * a.ldt + c] = v;
        }
    }
    __syncthreads();
    for (int q = tid; q < NF; q += 256) {
        const int f = fb0 - halo + q;
        float* o = fr + q * nfft;
        const float* row = nullptr;
        if (f >= a.f0 && f <= flast) row = Pp + (long)(f - a.f0) * a.ldp;
        else if (f >= 0 && f < a.f0 && Tp) row = Tp + (long)(f - (a.f0 - halo)) * a.ldt;
        if (!row) {
            for (int i = 0; i < nfft; ++i) o[i] = 0.f;
            continue;
        }
        float re[nb], im[nb];
#pragma unroll
        for (int k = 0; k < nb; ++k) {
            const float mag = __expf(row[k]);
            // phase = sin(x) for an unbounded conv_post output x: reduced to [-pi, pi] first (two-constant Cody-Waite,
            // exact k 2pi_hi for |x| < 2^17), since v_sin's accuracy falls off with |x|
            const float xv = row[nb + k];
            const float kq = rintf(xv * 0.159154943091895336f);
            const float xr = fmaf(-kq, -1.7484555e-7f, fmaf(-kq, 6.28318548202514648f, xv));
            const float ph = __sinf(xr);
            re[k] = mag * __cosf(ph);
            im[k] = mag * __sinf(ph);
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
    float* W = a.wav + (long)b * a.bsw;
    for (int s = tid; s < FB * hs; s += 256) {
        const long m = (long)fb0 * hs + s;  // padded sample index
        const long n = m - nfft / 2;        // output sample index (centre trim)
        if (n < a.n0 || m >= a.m_end) continue;
        float y = 0.f, env = 0.f;
        int fhi = (int)(m / hs);
        if (fhi > flast) fhi = flast;
        for (int f = fhi; f >= 0 && m - (long)f * hs < nfft; --f) {
            const int i = (int)(m - (long)f * hs);
            const int q = f - (fb0 - halo);
            y += fr[q * nfft + i];
            env += win[i] * win[i];
        }
        W[n - a.n0] = y / env;
    }
}

// output span [n0, n1) of a chunk and the padded-sample bound m_end
void chunk_span(long f0, long Fc, int fin, int nfft, int hs, long* n0, long* n1, long* m_end) {
    const long me = fin ? (f0 + Fc - 1) * hs + nfft / 2 : (f0 + Fc) * hs;
    long a0 = f0 * hs - nfft / 2;
    if (a0 < 0) a0 = 0;
    long a1 = me - nfft / 2;
    if (a1 < a0) a1 = a0;
    *n0 = a0;
    *n1 = a1;
    *m_end = me;
}

int launch(const IstftJob& j, int nfft, int B, long m_lo, hipStream_t s) {
    const int halo = (nfft + j.hs - 1) / j.hs - 1;
    const int FB = NF - halo;
    const size_t lds = (size_t)(NF * nfft + 3 * nfft) * 4;
    // blocks cover the chunk's frames and, on the final chunk, the samples past its last frame start
    const long span_frames = (j.m_end - m_lo + j.hs - 1) / j.hs;
    long nblk = (span_frames + FB - 1) / FB;
    const long nblk_f = ((long)j.Fc + FB - 1) / FB;
    if (nblk < nblk_f) nblk = nblk_f;
    dim3 g((unsigned)nblk, B);
    if (nfft == 20)
        hipLaunchKernelGGL(istft_kernel<20>, g, dim3(256), lds, s, j);
    else if (nfft == 16)
        hipLaunchKernelGGL(istft_kernel<16>, g, dim3(256), lds, s, j);
    else
        return STZS_ESHAPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

bool bad_geom(int nfft, int hs) { return nfft <= 0 || nfft > 64 || nfft % 2 || hs <= 0 || hs > nfft; }

}  // namespace

extern "C" int stzs_istft(const stzs_istft_args* a, void* stream) {
    if (!a || !a->post || !a->wav) return STZS_EINVAL;
    if (a->B <= 0 || a->Tf < 2 || bad_geom(a->n_fft, a->hop_s) || a->ldp < a->n_fft + 2) return STZS_ESHAPE;
    IstftJob j{};
    j.post = a->post;
    j.wav = a->wav;
    j.ldp = a->ldp;
    j.bsp = a->bsp;
    j.bsw = a->bsw;
    j.B = a->B;
    j.f0 = 0;
    j.Fc = a->Tf;
    j.hs = a->hop_s;
    long n1;
    chunk_span(0, a->Tf, 1, a->n_fft, a->hop_s, &j.n0, &n1, &j.m_end);
    return launch(j, a->n_fft, a->B, 0, reinterpret_cast<hipStream_t>(stream));
}

extern "C" int stzs_istft_stream_span(int f0, int Fc, int final_chunk, int n_fft, int hop_s, int64_t* n0,
                                      int64_t* n1) {
    if (!n0 || !n1) return STZS_EINVAL;
    if (f0 < 0 || Fc <= 0 || bad_geom(n_fft, hop_s)) return STZS_ESHAPE;
    long a0, a1, me;
    chunk_span(f0, Fc, final_chunk != 0, n_fft, hop_s, &a0, &a1, &me);
    *n0 = a0;
    *n1 = a1;
    return (n_fft + hop_s - 1) / hop_s - 1;
}

extern "C" int stzs_istft_stream(const stzs_istft_stream_args* a, void* stream) {
    if (!a || !a->post || !a->wav) return STZS_EINVAL;
    if (a->B <= 0 || a->f0 < 0 || a->Fc <= 0 || bad_geom(a->n_fft, a->hop_s) || a->ldp < a->n_fft + 2)
        return STZS_ESHAPE;
    if (a->f0 > 0 && !a->tail_in) return STZS_EINVAL;  // frames before the chunk reach its samples
    if ((a->tail_in || a->tail_out) && a->ldt < a->n_fft + 2) return STZS_ESHAPE;
    if (a->final_chunk && a->f0 + a->Fc < 2) return STZS_ESHAPE;
    if (a->tail_in && a->tail_in == a->tail_out) return STZS_EINVAL;  // block 0 writes while others read
    IstftJob j{};
    j.post = a->post;
    j.tail_in = a->f0 > 0 ? a->tail_in : nullptr;
    j.tail_out = a->tail_out;
    j.wav = a->wav;
    j.ldp = a->ldp;
    j.bsp = a->bsp;
    j.bsw = a->bsw;
    j.ldt = a->ldt;
    j.B = a->B;
    j.f0 = a->f0;
    j.Fc = a->Fc;
    j.hs = a->hop_s;
    long n1;
    chunk_span(a->f0, a->Fc, a->final_chunk != 0, a->n_fft, a->hop_s, &j.n0, &n1, &j.m_end);
    if (n1 == j.n0 && !a->tail_out) return STZS_OK;  // nothing to emit or carry
    return launch(j, a->n_fft, a->B, (long)a->f0 * a->hop_s, reinterpret_cast<hipStream_t>(stream));
}
