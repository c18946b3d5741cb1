// LSTM recurrence of the prosody predictor: the 3 DurationEncoder
// BiLSTMs, the duration LSTM and the shared F0/N LSTM — 520 dependent steps per 5-s utterance.
//
// The input projection x W_ih^T + b is one MFMA GEMM over all steps (stzs_conv1d, ks = 1); this
// kernel runs only the sequential part.  One workgroup (4 waves) per (direction, 16 utterances):
// per step gates[16 x 4H] = h_{t-1}[16 x H] W_hh^T on v_mfma_f32_16x16x32_bf16 — h_{t-1} from LDS
// (A fragments, loaded once per step), W_hh^T streamed from L2 in fragment order (one 1-KB fully
// coalesced load per 16x32 tile, prefetched one column tile ahead, bf16: 512 KB per step at H=256).
// Gates go through LDS; each thread updates 16 (utterance, unit) cells with c in registers and
// publishes h_t (bf16) to LDS and to the output.  Two barriers per step, no inter-workgroup traffic.
#include "common.hpp"

namespace {

constexpr int MB = 16;  // utterances per workgroup (MFMA M)

__global__ __launch_bounds__(256) void lstm_mfma(const stzs_lstm_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int H = a.H, G4 = 4 * a.H;
    const int hp = H + 8;                                    // bf16 pitch of the h tile
    bf16_t* hs = reinterpret_cast<bf16_t*>(smem);            // [MB][hp]
    float* gs = reinterpret_cast<float*>(smem + ((MB * hp * 2 + 15) & ~15));  // [MB][G4 + 4]
    const int gp = G4 + 4;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int dir = blockIdx.y;
    const int b0 = blockIdx.x * MB;
    const int nks = H / 32, nct = G4 / 16;
    const bf16_t* Wd = reinterpret_cast<const bf16_t*>(a.whhT) + (long)dir * nct * nks * 512;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);

    // cells owned by this thread: (row = e / H, unit = e % H) for e = tid + 256 * i
    const int ncell = MB * H;
    const int cpt = (ncell + 255) / 256;
    float c[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) c[i] = 0.f;
    for (int e = tid; e < MB * hp; e += 256) hs[e] = 0;
    __syncthreads();

    for (int s = 0; s < a.T; ++s) {
        const int t = dir == 0 ? s : a.T - 1 - s;
        // A fragments of h_{t-1}: row = lane & 15, k = ks*32 + 8*(lane>>4)
        bf16x8 af[8];
#pragma unroll
        for (int ks = 0; ks < 8; ++ks)
            if (ks < nks) af[ks] = *reinterpret_cast<const bf16x8*>(hs + (lane & 15) * hp + ks * 32 + 8 * (lane >> 4));
        // column tiles of this wave: ct = wave + 4 * i
        bf16x8 bcur[8], bnxt[8];
        int ct = wave;
        if (ct < nct) {
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
                if (ks < nks) bcur[ks] = *reinterpret_cast<const bf16x8*>(Wd + ((long)ct * nks + ks) * 512 + lane * 8);
        }
        for (; ct < nct; ct += 4) {
            const int cn = ct + 4;
            if (cn < nct) {
#pragma unroll
                for (int ks = 0; ks < 8; ++ks)
                    if (ks < nks) bnxt[ks] = *reinterpret_cast<const bf16x8*>(Wd + ((long)cn * nks + ks) * 512 + lane * 8);
            }
            f32x4 acc = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < 8; ++ks)
                if (ks < nks) acc = __builtin_amdgcn_mfma_f32_16x16x32_bf16(af[ks], bcur[ks], acc, 0, 0, 0);
#pragma unroll
            for (int r = 0; r < 4; ++r) gs[((lane >> 4) * 4 + r) * gp + ct * 16 + (lane & 15)] = acc[r];
#pragma unroll
            for (int ks = 0; ks < 8; ++ks) bcur[ks] = bnxt[ks];
        }
        __syncthreads();
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            if (i >= cpt) break;
            const int e = tid + 256 * i;
            if (e >= ncell) break;
            const int row = e / H, j = e - row * H;
            const int b = b0 + row;
            float gi = gs[row * gp + j], gf = gs[row * gp + H + j], gg = gs[row * gp + 2 * H + j],
                  go = gs[row * gp + 3 * H + j];
            if (b < a.B) {
                const float* gx = a.gx + (long)b * a.bsg + (long)t * a.ldg + dir * G4;
                gi += gx[j];
                gf += gx[H + j];
                gg += gx[2 * H + j];
                go += gx[3 * H + j];
            }
            const float ig = 1.f / (1.f + __expf(-gi));
            const float fg = 1.f / (1.f + __expf(-gf));
            const float cg = tanhf(gg);
            const float og = 1.f / (1.f + __expf(-go));
            c[i] = fg * c[i] + ig * cg;
            const float h = og * tanhf(c[i]);
            const bf16_t hb = f2bf(h);
            hs[row * hp + j] = hb;
            if (b < a.B) Y[(long)b * a.bsy + (long)t * a.ldy + dir * H + j] = hb;
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" int stzs_lstm(const stzs_lstm_args* a, void* stream) {
    if (!a || !a->gx || !a->whhT || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->H <= 0 || a->H > 256 || a->H % 32 || (a->ndir != 1 && a->ndir != 2))
        return STZS_ESHAPE;
    if (MB * a->H > 256 * 16) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int hp = a->H + 8;
    const size_t lds = ((MB * hp * 2 + 15) & ~15) + (size_t)MB * (4 * a->H + 4) * 4;
    auto k = lstm_mfma;
    if (lds > 64 * 1024) (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3((a->B + MB - 1) / MB, a->ndir), dim3(256), lds, s, *a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
