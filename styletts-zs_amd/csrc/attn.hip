// Denoiser multi-head attention: self-attention over the L_s = 50 style codes
// and cross-attention to [text ; prompt] context (T_txt + 50 keys), head dim 64.
//
// Flash-style on v_mfma_f32_16x16x32_bf16: one workgroup (4 waves) per (row, head, 64 queries), one
// wave per 16 queries.  Keys stream through LDS in 64-key chunks: K as rows (B operand of S = Q K^T),
// V transposed (B operand of O = P V), both 16-B padded.  Online softmax in fp32 on the accumulator
// layout (row max / sum by in-register max + 16-lane xor shuffles); P goes C-layout -> A-layout through
// a per-wave bf16 LDS tile.  Q fragments come straight from global memory (read once).
#include "common.hpp"

namespace {

constexpr int KC = 64;  // keys per chunk

template <int DH>
__global__ __launch_bounds__(256) void attn_mfma(const stzs_attn_args a) {
    constexpr int NKS = DH / 32;   // k-steps of S
    constexpr int NDT = DH / 16;   // d tiles of O
    constexpr int KP = DH + 8;     // K row pitch (bf16)
    constexpr int VP = KC + 8;     // V^T row pitch
    constexpr int PP = KC + 8;     // P row pitch
    __shared__ __attribute__((aligned(16))) bf16_t Ks[KC * KP];
    __shared__ __attribute__((aligned(16))) bf16_t Vt[DH * VP];
    __shared__ __attribute__((aligned(16))) bf16_t Ps[4][16 * PP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long r = blockIdx.x;
    const int h = blockIdx.y;
    const int qb = blockIdx.z * 64 + wave * 16;
    const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + r * a.bsq + h * DH;
    const bf16_t* K = reinterpret_cast<const bf16_t*>(a.k) + r * a.bsk + h * DH;
    const bf16_t* V = reinterpret_cast<const bf16_t*>(a.v) + r * a.bsv + h * DH;
    const float scale = 1.f / sqrtf((float)DH);

    bf16x8 qf[NKS];
    {
        const int qr = min(qb + (lane & 15), a.Lq - 1);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[ks] = *reinterpret_cast<const bf16x8*>(Q + (long)qr * a.ldq + ks * 32 + 8 * (lane >> 4));
    }
    f32x4 o[NDT];
#pragma unroll
    for (int i = 0; i < NDT; ++i) o[i] = f32x4{0.f, 0.f, 0.f, 0.f};
    float m[4], l[4];
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        m[i] = -INFINITY;
        l[i] = 0.f;
    }
    bf16_t* P = Ps[wave];

    for (int c0 = 0; c0 < a.Lk; c0 += KC) {
        __syncthreads();
        // stage K rows and V^T for keys [c0, c0 + KC)
        for (int i = tid; i < KC * (DH / 8); i += 256) {
            const int kr = i / (DH / 8), cv = i - kr * (DH / 8);
            const bool ok = c0 + kr < a.Lk;
            const int kk = ok ? c0 + kr : 0;
            uint4 kv = *reinterpret_cast<const uint4*>(K + (long)kk * a.ldk + cv * 8);
            uint4 vv = *reinterpret_cast<const uint4*>(V + (long)kk * a.ldv + cv * 8);
            if (!ok) kv = vv = make_uint4(0, 0, 0, 0);
            *reinterpret_cast<uint4*>(Ks + kr * KP + cv * 8) = kv;
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                Vt[(cv * 8 + 2 * j) * VP + kr] = (bf16_t)(w[j] & 0xFFFF);
                Vt[(cv * 8 + 2 * j + 1) * VP + kr] = (bf16_t)(w[j] >> 16);
            }
        }
        __syncthreads();
        // S = Q K^T for 16 queries x 64 keys
        f32x4 s[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const bf16x8 kf = *reinterpret_cast<const bf16x8*>(Ks + (nt * 16 + (lane & 15)) * KP + ks * 32 + 8 * (lane >> 4));
                s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qf[ks], kf, s[nt], 0, 0, 0);
            }
        }
        // online softmax; element (row = (lane>>4)*4 + i, key = nt*16 + (lane & 15))
        float alpha[4];
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            float mx = -INFINITY;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const bool ok = c0 + nt * 16 + (lane & 15) < a.Lk;
                s[nt][i] = ok ? s[nt][i] * scale : -INFINITY;
                mx = fmaxf(mx, s[nt][i]);
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) mx = fmaxf(mx, __shfl_xor(mx, off, 64));
            const float mn = fmaxf(m[i], mx);
            alpha[i] = __expf(m[i] - mn);
            float sum = 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float pv = __expf(s[nt][i] - mn);
                s[nt][i] = pv;
                sum += pv;
            }
#pragma unroll
            for (int off = 1; off < 16; off <<= 1) sum += __shfl_xor(sum, off, 64);
            l[i] = l[i] * alpha[i] + sum;
            m[i] = mn;
        }
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] *= alpha[i];
        // P -> LDS (C layout) -> A fragments
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) P[((lane >> 4) * 4 + i) * PP + nt * 16 + (lane & 15)] = f2bf(s[nt][i]);
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KC / 32; ++ks) {
            const bf16x8 pf = *reinterpret_cast<const bf16x8*>(P + (lane & 15) * PP + ks * 32 + 8 * (lane >> 4));
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const bf16x8 vf = *reinterpret_cast<const bf16x8*>(Vt + (dt * 16 + (lane & 15)) * VP + ks * 32 + 8 * (lane >> 4));
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pf, vf, o[dt], 0, 0, 0);
            }
        }
    }
    bf16_t* O = reinterpret_cast<bf16_t*>(a.o) + r * a.bso + h * DH;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = qb + (lane >> 4) * 4 + i;
        if (q < a.Lq) {
            const float inv = 1.f / l[i];
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) O[(long)q * a.ldo + dt * 16 + (lane & 15)] = f2bf(o[dt][i] * inv);
        }
    }
}

// PRECISE mode (stzs_attn_args.precise = 1): fp32 q / k / v / o, fp32 dot products and libm expf on the VALU,
// online softmax per 64-key chunk.  One thread per query, one workgroup per (row, head, 256 queries): the
// denoiser's 50 x (<= a few hundred) x 64 per head is small, this path exists for fp32-level parity.
constexpr int KC32 = 64;
template <int DH>
__global__ __launch_bounds__(256) void attn_f32(const stzs_attn_args a) {
    __shared__ float Ks[KC32][DH + 1];
    __shared__ float Vs[KC32][DH + 1];
    const int tid = threadIdx.x;
    const long r = blockIdx.x;
    const int h = blockIdx.y;
    const int qi = blockIdx.z * 256 + tid;
    const bool qok = qi < a.Lq;
    const float* Q = reinterpret_cast<const float*>(a.q) + r * a.bsq + h * DH;
    const float* K = reinterpret_cast<const float*>(a.k) + r * a.bsk + h * DH;
    const float* V = reinterpret_cast<const float*>(a.v) + r * a.bsv + h * DH;
    const float scale = 1.f / sqrtf((float)DH);
    float q[DH], o[DH];
#pragma unroll
    for (int d = 0; d < DH; ++d) {
        q[d] = qok ? Q[(long)qi * a.ldq + d] : 0.f;
        o[d] = 0.f;
    }
    float m = -INFINITY, l = 0.f;
    for (int c0 = 0; c0 < a.Lk; c0 += KC32) {
        const int nk = min(KC32, a.Lk - c0);
        __syncthreads();
        for (int i = tid; i < KC32 * DH; i += 256) {  // rows past nk zeroed (read, masked)
            const int kr = i / DH, d = i - kr * DH;
            const bool ok = kr < nk;
            Ks[kr][d] = ok ? K[(long)(c0 + kr) * a.ldk + d] : 0.f;
            Vs[kr][d] = ok ? V[(long)(c0 + kr) * a.ldv + d] : 0.f;
        }
        __syncthreads();
        if (!qok) continue;
        // (static key indices keep sv in registers; keys past nk are masked, not branched around)
        float sv[KC32];
        float mx = m;
#pragma unroll
        for (int j = 0; j < KC32; ++j) {
            float acc = 0.f;
#pragma unroll
            for (int d = 0; d < DH; ++d) acc = fmaf(q[d], Ks[j][d], acc);
            sv[j] = j < nk ? acc * scale : -INFINITY;
            mx = fmaxf(mx, sv[j]);
        }
        const float corr = expf(m - mx);
        l *= corr;
#pragma unroll
        for (int d = 0; d < DH; ++d) o[d] *= corr;
#pragma unroll
        for (int j = 0; j < KC32; ++j) {
            const float pj = j < nk ? expf(sv[j] - mx) : 0.f;
            l += pj;
#pragma unroll
            for (int d = 0; d < DH; ++d) o[d] = fmaf(pj, Vs[j][d], o[d]);
        }
        m = mx;
    }
    if (qok) {
        float* O = reinterpret_cast<float*>(a.o) + r * a.bso + h * DH + (long)qi * a.ldo;
        const float inv = 1.f / l;
#pragma unroll
        for (int d = 0; d < DH; ++d) O[d] = o[d] * inv;
    }
}

}  // namespace

extern "C" int stzs_attention(const stzs_attn_args* a, void* stream) {
    if (!a || !a->q || !a->k || !a->v || !a->o) return STZS_EINVAL;
    if (a->R <= 0 || a->Lq <= 0 || a->Lk <= 0 || a->heads <= 0) return STZS_ESHAPE;
    if (a->ldq % 8 || a->ldk % 8 || a->ldv % 8 || a->bsq % 8 || a->bsk % 8 || a->bsv % 8) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->precise == 1) {
        dim3 g((unsigned)a->R, a->heads, (a->Lq + 255) / 256);
        if (a->dh == 64)
            hipLaunchKernelGGL(attn_f32<64>, g, dim3(256), 0, s, *a);
        else if (a->dh == 32)
            hipLaunchKernelGGL(attn_f32<32>, g, dim3(256), 0, s, *a);
        else
            return STZS_ESHAPE;
        STZS_LAUNCH_CHECK();
        return STZS_OK;
    }
    if (a->precise != 0) return STZS_EINVAL;
    dim3 g((unsigned)a->R, a->heads, (a->Lq + 63) / 64);
    if (a->dh == 64)
        hipLaunchKernelGGL(attn_mfma<64>, g, dim3(256), 0, s, *a);
    else if (a->dh == 32)
        hipLaunchKernelGGL(attn_mfma<32>, g, dim3(256), 0, s, *a);
    else
        return STZS_ESHAPE;
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
