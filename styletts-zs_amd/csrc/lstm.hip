// LSTM recurrence of the prosody predictor: the 3 DurationEncoder
// BiLSTMs, the duration LSTM and the shared F0/N LSTM — 520 dependent steps per 5-s utterance.
//
// The input projection x W_ih^T + b is one MFMA GEMM over all steps (stzs_conv1d, ks = 1); this
// kernel runs only the sequential part.  One workgroup per (direction, BB-utterance group);
// thread j owns hidden unit j: it accumulates its 4 gate rows against h_{t-1} (broadcast from
// LDS) with the transposed recurrent weights W_hh^T[k][4H] read coalesced across units (the
// 1 MB fp32 matrix stays L2-resident across steps), updates c and h in registers and publishes
// h_t to LDS.  One barrier per step; no inter-workgroup traffic.
#include "common.hpp"

namespace {

template <int BB>
__global__ __launch_bounds__(256) void lstm_rec(const stzs_lstm_args a) {
    __shared__ float hs[2][BB][256];
    const int j = threadIdx.x;
    const int dir = blockIdx.y;
    const int b0 = blockIdx.x * BB;
    const int H = a.H, G4 = 4 * a.H;
    const bool unit = j < H;
    float c[BB];
#pragma unroll
    for (int bb = 0; bb < BB; ++bb) {
        c[bb] = 0.f;
        hs[0][bb][j] = 0.f;
    }
    const float* Wt = a.whhT + (long)dir * H * G4;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);
    __syncthreads();
    for (int s = 0; s < a.T; ++s) {
        const int t = dir == 0 ? s : a.T - 1 - s;
        const int cur = s & 1;
        float acc[4][BB];
#pragma unroll
        for (int bb = 0; bb < BB; ++bb) {
            const int b = b0 + bb;
#pragma unroll
            for (int g = 0; g < 4; ++g)
                acc[g][bb] = (unit && b < a.B) ? a.gx[(long)b * a.bsg + (long)t * a.ldg + dir * G4 + g * H + j] : 0.f;
        }
        if (unit) {
#pragma unroll 4
            for (int k = 0; k < H; ++k) {
                const float* wr = Wt + (long)k * G4 + j;
                const float w0 = wr[0], w1 = wr[H], w2 = wr[2 * H], w3 = wr[3 * H];
#pragma unroll
                for (int bb = 0; bb < BB; ++bb) {
                    const float hk = hs[cur][bb][k];
                    acc[0][bb] += w0 * hk;
                    acc[1][bb] += w1 * hk;
                    acc[2][bb] += w2 * hk;
                    acc[3][bb] += w3 * hk;
                }
            }
        }
#pragma unroll
        for (int bb = 0; bb < BB; ++bb) {
            const float ig = 1.f / (1.f + expf(-acc[0][bb]));
            const float fg = 1.f / (1.f + expf(-acc[1][bb]));
            const float gg = tanhf(acc[2][bb]);
            const float og = 1.f / (1.f + expf(-acc[3][bb]));
            c[bb] = fg * c[bb] + ig * gg;
            const float h = og * tanhf(c[bb]);
            hs[cur ^ 1][bb][j] = unit ? h : 0.f;
            const int b = b0 + bb;
            if (unit && b < a.B) Y[(long)b * a.bsy + (long)t * a.ldy + dir * H + j] = f2bf(h);
        }
        __syncthreads();
    }
}

}  // namespace

extern "C" int stzs_lstm(const stzs_lstm_args* a, void* stream) {
    if (!a || !a->gx || !a->whhT || !a->y) return STZS_EINVAL;
    if (a->B <= 0 || a->T <= 0 || a->H <= 0 || a->H > 256 || (a->ndir != 1 && a->ndir != 2)) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    const int thr = ((a->H + 63) / 64) * 64;
    if (a->B >= 8) {
        hipLaunchKernelGGL(lstm_rec<8>, dim3((a->B + 7) / 8, a->ndir), dim3(thr), 0, s, *a);
    } else if (a->B >= 4) {
        hipLaunchKernelGGL(lstm_rec<4>, dim3((a->B + 3) / 4, a->ndir), dim3(thr), 0, s, *a);
    } else {
        hipLaunchKernelGGL(lstm_rec<1>, dim3(a->B, a->ndir), dim3(thr), 0, s, *a);
    }
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
