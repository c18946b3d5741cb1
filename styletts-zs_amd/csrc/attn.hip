// Denoiser multi-head attention: self-attention over the L_s = 50 style codes
// and cross-attention to [text ; prompt] context (T_txt + 50 keys), head dim 64.
//
// bf16: the flash unit of csrc/attn_body.hpp, one workgroup per (row, head, 64 queries).
#include "attn_body.hpp"

namespace {

constexpr int KC = stzs_attn::KC;  // keys per chunk

template <int DH>
__global__ __launch_bounds__(256) void attn_mfma(const stzs_attn_args a) {
    __shared__ __attribute__((aligned(16))) unsigned char lds[stzs_attn::Lds<DH>::BYTES];
    stzs_attn::attn_unit<DH, stzs_attn::LdPlain>(a, blockIdx.x, blockIdx.y, blockIdx.z * 64, lds);
}

// PRECISE mode (stzs_attn_args.precise = 1): fp32 q / k / v / o.  The same flash structure on the same MFMAs
// with split operands (hi = bf16(x), lo = bf16(x - hi)): S = Qh Kh + Qh Kl + Ql Kh and O += Ph Vh + Ph Vl + Pl Vh
// (fp32 accumulate, ~fp32 accuracy), the softmax exponentials with libm expf.
template <int DH>
__global__ __launch_bounds__(256) void attn_x3(const stzs_attn_args a) {
    constexpr int NKS = DH / 32;
    constexpr int NDT = DH / 16;
    constexpr int KP = DH + 8;
    constexpr int VP = DH + 8;  // V rows, row-major: the PV fragments by transposed reads (attn_body.hpp frag_tr)
    constexpr int PTP = 16 + 4;  // P^T [key][query] per wave
    __shared__ __attribute__((aligned(16))) bf16_t Ks[2][KC * KP];
    __shared__ __attribute__((aligned(16))) bf16_t Vs[2][KC * VP];
    __shared__ __attribute__((aligned(16))) bf16_t Ps[2][4][KC * PTP];
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
            *reinterpret_cast<bf16x8*>(&Vs[0][kr * VP + cv * 8]) = vh;
            *reinterpret_cast<bf16x8*>(&Vs[1][kr * VP + cv * 8]) = vl;
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
        float alpha[4], mx[4], sum[4];  // (the row reductions on DPP, as attn_body.hpp)
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            mx[i] = -INFINITY;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const bool ok = c0 + nt * 16 + (lane & 15) < a.Lk;
                s[nt][i] = ok ? s[nt][i] * scale : -INFINITY;
                mx[i] = fmaxf(mx[i], s[nt][i]);
            }
        }
        stzs_attn::row16_max4(mx);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mn = fmaxf(m[i], mx[i]);
            alpha[i] = expf(m[i] - mn);
            sum[i] = 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float pv = expf(s[nt][i] - mn);
                s[nt][i] = pv;
                sum[i] += pv;
            }
            m[i] = mn;
        }
        stzs_attn::row16_sum4(sum);
#pragma unroll
        for (int i = 0; i < 4; ++i) l[i] = l[i] * alpha[i] + sum[i];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] *= alpha[i];
        // P (split) -> P^T images, one 8-B store per key tile and image; A fragments by transposed reads
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            float hf[4], lf[4];
#pragma unroll
            for (int i = 0; i < 4; ++i) {
                hf[i] = bf2f(f2bf(s[nt][i]));
                lf[i] = s[nt][i] - hf[i];
            }
            const int pi = (nt * 16 + (lane & 15)) * PTP + 4 * (lane >> 4);
            *reinterpret_cast<uint2*>(&Ps[0][wave][pi]) = make_uint2(pack2bf(hf[0], hf[1]), pack2bf(hf[2], hf[3]));
            *reinterpret_cast<uint2*>(&Ps[1][wave][pi]) = make_uint2(pack2bf(lf[0], lf[1]), pack2bf(lf[2], lf[3]));
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KC / 32; ++ks) {
            const bf16x8 ph = stzs_attn::frag_tr(Ps[0][wave], PTP, ks * 32, 0, lane);
            const bf16x8 pl = stzs_attn::frag_tr(Ps[1][wave], PTP, ks * 32, 0, lane);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const bf16x8 vh = stzs_attn::frag_tr(Vs[0], VP, ks * 32, dt * 16, lane);
                const bf16x8 vl = stzs_attn::frag_tr(Vs[1], VP, ks * 32, dt * 16, lane);
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
