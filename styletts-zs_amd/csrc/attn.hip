// Denoiser multi-head attention: self-attention over the L_s = 50 style
// codes and cross-attention to [text ; prompt] context (T_txt + 50 keys).  These are tiny
// (Lq = 50, Lk <= ~530, dh = 64) and latency-bound, so v1 is an fp32-FMA online-softmax kernel:
// one workgroup per (row, head, 16 queries); keys streamed through LDS in 128-key chunks
// (bf16, 16-B padded rows); one lane per key for QK^T, one lane per head-dim for PV.
#include "common.hpp"

namespace {

constexpr int KC = 128;  // keys per LDS chunk
constexpr int QB = 16;   // queries per workgroup (4 per wave)

template <int DH>
__global__ __launch_bounds__(256) void attn_fwd(const stzs_attn_args a) {
    constexpr int KP = DH + 8;
    __shared__ __attribute__((aligned(16))) bf16_t Ks[KC][KP];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[KC][KP];
    __shared__ float Qs[QB][DH];
    __shared__ float Ps[4][4][KC];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long r = blockIdx.x;
    const int h = blockIdx.y, q0 = blockIdx.z * QB;
    const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + r * a.bsq + h * DH;
    const bf16_t* K = reinterpret_cast<const bf16_t*>(a.k) + r * a.bsk + h * DH;
    const bf16_t* V = reinterpret_cast<const bf16_t*>(a.v) + r * a.bsv + h * DH;
    const float scale = 1.f / sqrtf((float)DH);
    for (int i = tid; i < QB * DH; i += 256) {
        const int qi = i / DH, d = i - qi * DH;
        Qs[qi][d] = (q0 + qi < a.Lq) ? bf2f(Q[(long)(q0 + qi) * a.ldq + d]) * scale : 0.f;
    }
    float m[4], l[4], o[4];
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
        m[qq] = -INFINITY;
        l[qq] = 0.f;
        o[qq] = 0.f;
    }
    constexpr int VPR = DH / 8;
    for (int c0 = 0; c0 < a.Lk; c0 += KC) {
        __syncthreads();
        for (int i = tid; i < KC * VPR; i += 256) {
            const int kr = i / VPR, cv = i - kr * VPR;
            uint4 kv = make_uint4(0, 0, 0, 0), vv = make_uint4(0, 0, 0, 0);
            if (c0 + kr < a.Lk) {
                kv = *reinterpret_cast<const uint4*>(K + (long)(c0 + kr) * a.ldk + cv * 8);
                vv = *reinterpret_cast<const uint4*>(V + (long)(c0 + kr) * a.ldv + cv * 8);
            }
            *reinterpret_cast<uint4*>(&Ks[kr][cv * 8]) = kv;
            *reinterpret_cast<uint4*>(&Vs[kr][cv * 8]) = vv;
        }
        __syncthreads();
        float s[4][2];
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) s[qq][0] = s[qq][1] = 0.f;
#pragma unroll
        for (int slot = 0; slot < 2; ++slot) {
            const int kr = lane + slot * 64;
#pragma unroll
            for (int cv = 0; cv < VPR; ++cv) {
                float kf[8];
                load8(&Ks[kr][cv * 8], kf);
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) {
                    const float* qp = &Qs[wave * 4 + qq][cv * 8];
#pragma unroll
                    for (int j = 0; j < 8; ++j) s[qq][slot] += qp[j] * kf[j];
                }
            }
        }
#pragma unroll
        for (int qq = 0; qq < 4; ++qq) {
            const float s0 = (c0 + lane < a.Lk) ? s[qq][0] : -INFINITY;
            const float s1 = (c0 + lane + 64 < a.Lk) ? s[qq][1] : -INFINITY;
            const float mn = fmaxf(m[qq], wave_max(fmaxf(s0, s1)));
            const float al = expf(m[qq] - mn);
            const float p0 = expf(s0 - mn), p1 = expf(s1 - mn);
            l[qq] = l[qq] * al + wave_sum(p0 + p1);
            o[qq] *= al;
            m[qq] = mn;
            Ps[wave][qq][lane] = p0;
            Ps[wave][qq][lane + 64] = p1;
        }
        __syncthreads();
        const int kmax = min(KC, a.Lk - c0);
        if (lane < DH) {
            for (int k = 0; k < kmax; ++k) {
                const float vk = bf2f(Vs[k][lane]);
#pragma unroll
                for (int qq = 0; qq < 4; ++qq) o[qq] += Ps[wave][qq][k] * vk;
            }
        }
    }
    bf16_t* O = reinterpret_cast<bf16_t*>(a.o) + r * a.bso + h * DH;
#pragma unroll
    for (int qq = 0; qq < 4; ++qq) {
        const int qi = q0 + wave * 4 + qq;
        if (qi < a.Lq && lane < DH) O[(long)qi * a.ldo + lane] = f2bf(o[qq] / l[qq]);
    }
}

}  // namespace

extern "C" int stzs_attention(const stzs_attn_args* a, void* stream) {
    if (!a || !a->q || !a->k || !a->v || !a->o) return STZS_EINVAL;
    if (a->R <= 0 || a->Lq <= 0 || a->Lk <= 0 || a->heads <= 0) return STZS_ESHAPE;
    if (a->ldk % 8 || a->ldv % 8 || a->bsk % 8 || a->bsv % 8) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    dim3 g((unsigned)a->R, a->heads, (a->Lq + QB - 1) / QB);
    if (a->dh == 64)
        hipLaunchKernelGGL(attn_fwd<64>, g, dim3(256), 0, s, *a);
    else if (a->dh == 32)
        hipLaunchKernelGGL(attn_fwd<32>, g, dim3(256), 0, s, *a);
    else
        return STZS_ESHAPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
