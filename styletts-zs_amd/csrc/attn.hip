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

    // K / V chunk loads run one chunk ahead in registers: chunk c + 1's global loads are in flight while chunk c
    // is computed (cross-attention: 3 chunks of 64 keys), the LDS images are written from the registers
    constexpr int NLD = KC * (DH / 8) / 256;  // 16-B K (and V) words per thread per chunk
    static_assert(KC * (DH / 8) % 256 == 0, "whole chunk per pass");
    uint4 pk[NLD], pv[NLD];
    auto load_chunk = [&](int c0) {
#pragma unroll
        for (int j = 0; j < NLD; ++j) {
            const int i = tid + j * 256;
            const int kr = i / (DH / 8), cv = i - kr * (DH / 8);
            const bool ok = c0 + kr < a.Lk;
            const int kk = ok ? c0 + kr : 0;
            pk[j] = *reinterpret_cast<const uint4*>(K + (long)kk * a.ldk + cv * 8);
            pv[j] = *reinterpret_cast<const uint4*>(V + (long)kk * a.ldv + cv * 8);
            if (!ok) pk[j] = pv[j] = make_uint4(0, 0, 0, 0);
        }
    };
    load_chunk(0);
    for (int c0 = 0; c0 < a.Lk; c0 += KC) {
        __syncthreads();
        // stage K rows and V^T for keys [c0, c0 + KC) from the registers, then start the next chunk's loads
#pragma unroll
        for (int j = 0; j < NLD; ++j) {
            const int i = tid + j * 256;
            const int kr = i / (DH / 8), cv = i - kr * (DH / 8);
            const uint4 kv = pk[j], vv = pv[j];
            *reinterpret_cast<uint4*>(Ks + kr * KP + cv * 8) = kv;
            const uint32_t w[4] = {vv.x, vv.y, vv.z, vv.w};
#pragma unroll
            for (int q = 0; q < 4; ++q) {
                Vt[(cv * 8 + 2 * q) * VP + kr] = (bf16_t)(w[q] & 0xFFFF);
                Vt[(cv * 8 + 2 * q + 1) * VP + kr] = (bf16_t)(w[q] >> 16);
            }
        }
        if (c0 + KC < a.Lk) load_chunk(c0 + KC);
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

// PRECISE mode (stzs_attn_args.precise = 1): fp32 q / k / v / o.  The same flash structure on the same MFMAs
// with split operands (hi = bf16(x), lo = bf16(x - hi)): S = Qh Kh + Qh Kl + Ql Kh and O += Ph Vh + Ph Vl + Pl Vh
// (fp32 accumulate, ~fp32 accuracy), the softmax exponentials with libm expf.
template <int DH>
__global__ __launch_bounds__(256) void attn_x3(const stzs_attn_args a) {
    constexpr int NKS = DH / 32;
    constexpr int NDT = DH / 16;
    constexpr int KP = DH + 8;
    constexpr int VP = KC + 8;
    constexpr int PP = KC + 8;
    __shared__ __attribute__((aligned(16))) bf16_t Ks[2][KC * KP];
    __shared__ __attribute__((aligned(16))) bf16_t Vt[2][DH * VP];
    __shared__ __attribute__((aligned(16))) bf16_t Ps[2][4][16 * PP];
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const long r = blockIdx.x;
    const int h = blockIdx.y;
    const int qb = blockIdx.z * 64 + wave * 16;
    const float* Q = reinterpret_cast<const float*>(a.q) + r * a.bsq + h * DH;
    const float* K = reinterpret_cast<const float*>(a.k) + r * a.bsk + h * DH;
    const float* V = reinterpret_cast<const float*>(a.v) + r * a.bsv + h * DH;
    const float scale = 1.f / sqrtf((float)DH);
    auto split8 = [](const float* f, bf16x8& hi, bf16x8& lo) {
        uint4 hp = pack8(f);
        float hf[8], lf[8];
        unpack8(hp, hf);
#pragma unroll
        for (int j = 0; j < 8; ++j) lf[j] = f[j] - hf[j];
        uint4 lp = pack8(lf);
        hi = __builtin_bit_cast(bf16x8, hp);
        lo = __builtin_bit_cast(bf16x8, lp);
    };
    bf16x8 qh[NKS], ql[NKS];
    {
        const int qr = min(qb + (lane & 15), a.Lq - 1);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks) {
            float f[8];
            load8(Q + (long)qr * a.ldq + ks * 32 + 8 * (lane >> 4), f);
            split8(f, qh[ks], ql[ks]);
        }
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
    for (int c0 = 0; c0 < a.Lk; c0 += KC) {
        __syncthreads();
        for (int i = tid; i < KC * (DH / 8); i += 256) {
            const int kr = i / (DH / 8), cv = i - kr * (DH / 8);
            const bool ok = c0 + kr < a.Lk;
            const int kk = ok ? c0 + kr : 0;
            float kf[8], vf[8];
            load8(K + (long)kk * a.ldk + cv * 8, kf);
            load8(V + (long)kk * a.ldv + cv * 8, vf);
            if (!ok) {
#pragma unroll
                for (int j = 0; j < 8; ++j) kf[j] = vf[j] = 0.f;
            }
            bf16x8 kh, kl, vh, vl;
            split8(kf, kh, kl);
            split8(vf, vh, vl);
            *reinterpret_cast<bf16x8*>(&Ks[0][kr * KP + cv * 8]) = kh;
            *reinterpret_cast<bf16x8*>(&Ks[1][kr * KP + cv * 8]) = kl;
            const uint4 uh = __builtin_bit_cast(uint4, vh), ul = __builtin_bit_cast(uint4, vl);
            const uint32_t wh[4] = {uh.x, uh.y, uh.z, uh.w}, wl[4] = {ul.x, ul.y, ul.z, ul.w};
#pragma unroll
            for (int j = 0; j < 4; ++j) {
                Vt[0][(cv * 8 + 2 * j) * VP + kr] = (bf16_t)(wh[j] & 0xFFFF);
                Vt[0][(cv * 8 + 2 * j + 1) * VP + kr] = (bf16_t)(wh[j] >> 16);
                Vt[1][(cv * 8 + 2 * j) * VP + kr] = (bf16_t)(wl[j] & 0xFFFF);
                Vt[1][(cv * 8 + 2 * j + 1) * VP + kr] = (bf16_t)(wl[j] >> 16);
            }
        }
        __syncthreads();
        f32x4 s[4];
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            s[nt] = f32x4{0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int ks = 0; ks < NKS; ++ks) {
                const int ko = (nt * 16 + (lane & 15)) * KP + ks * 32 + 8 * (lane >> 4);
                const bf16x8 kh = *reinterpret_cast<const bf16x8*>(&Ks[0][ko]);
                const bf16x8 kl = *reinterpret_cast<const bf16x8*>(&Ks[1][ko]);
                s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ql[ks], kh, s[nt], 0, 0, 0);
                s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[ks], kl, s[nt], 0, 0, 0);
                s[nt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(qh[ks], kh, s[nt], 0, 0, 0);
            }
        }
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
            alpha[i] = expf(m[i] - mn);
            float sum = 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float pv = expf(s[nt][i] - mn);
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
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                const int pi = ((lane >> 4) * 4 + i) * PP + nt * 16 + (lane & 15);
                const bf16_t ph = f2bf(s[nt][i]);
                Ps[0][wave][pi] = ph;
                Ps[1][wave][pi] = f2bf(s[nt][i] - bf2f(ph));
            }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KC / 32; ++ks) {
            const int po = (lane & 15) * PP + ks * 32 + 8 * (lane >> 4);
            const bf16x8 ph = *reinterpret_cast<const bf16x8*>(&Ps[0][wave][po]);
            const bf16x8 pl = *reinterpret_cast<const bf16x8*>(&Ps[1][wave][po]);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const int vo = (dt * 16 + (lane & 15)) * VP + ks * 32 + 8 * (lane >> 4);
                const bf16x8 vh = *reinterpret_cast<const bf16x8*>(&Vt[0][vo]);
                const bf16x8 vl = *reinterpret_cast<const bf16x8*>(&Vt[1][vo]);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(pl, vh, o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vl, o[dt], 0, 0, 0);
                o[dt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(ph, vh, o[dt], 0, 0, 0);
            }
        }
    }
    float* O = reinterpret_cast<float*>(a.o) + r * a.bso + h * DH;
#pragma unroll
    for (int i = 0; i < 4; ++i) {
        const int q = qb + (lane >> 4) * 4 + i;
        if (q < a.Lq) {
            const float inv = 1.f / l[i];
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) O[(long)q * a.ldo + dt * 16 + (lane & 15)] = o[dt][i] * inv;
        }
    }
}

}  // namespace

extern "C" int stzs_attention(const stzs_attn_args* a, void* stream) {
    if (!a || !a->q || !a->k || !a->v || !a->o) return STZS_EINVAL;
    if (a->R <= 0 || a->Lq <= 0 || a->Lk <= 0 || a->heads <= 0) return STZS_ESHAPE;
    if (a->ldq % 8 || a->ldk % 8 || a->ldv % 8 || a->bsq % 8 || a->bsk % 8 || a->bsv % 8) return STZS_ESHAPE;
    hipStream_t s = reinterpret_cast<hipStream_t>(stream);
    if (a->precise == 1) {
        dim3 g((unsigned)a->R, a->heads, (a->Lq + 63) / 64);
        if (a->dh == 64)
            hipLaunchKernelGGL(attn_x3<64>, g, dim3(256), 0, s, *a);
        else if (a->dh == 32)
            hipLaunchKernelGGL(attn_x3<32>, g, dim3(256), 0, s, *a);
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
