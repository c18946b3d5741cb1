// The bf16 flash-attention unit of the denoiser, shared by the attention kernel
// (csrc/attn.hip: one workgroup per (row, head, 64 queries)) and the fused small-M linear (csrc/rows.hip: the
// last-arriving workgroup of a head's column tiles runs that head's attention inside the linear's launch).
//
// One 256-thread workgroup, one wave per 16 queries, v_mfma_f32_16x16x32_bf16.  Keys stream through LDS in
// 64-key chunks: K as rows (B operand of S = Q K^T), V transposed (B operand of O = P V), both 16-B padded.
// Online softmax in fp32 on the accumulator layout (row max / sum by in-register max + 16-lane xor shuffles);
// P goes C-layout -> A-layout through a per-wave bf16 LDS tile.  Q fragments come straight from global memory.
// The loader LD decides how q / k / v are read: plain loads (operands written by earlier launches) or sc1 loads
// (operands stored write-through earlier in the SAME launch by workgroups on any XCD).  Same arithmetic either way.
#pragma once
#include "common.hpp"

namespace stzs_attn {

constexpr int KC = 64;  // keys per chunk

template <int DH>
struct Lds {
    static constexpr int KP = DH + 8;  // K row pitch (bf16)
    static constexpr int VP = KC + 8;  // V^T row pitch
    static constexpr int PP = KC + 8;  // P row pitch
    static constexpr int K_ELEMS = KC * KP, V_ELEMS = DH * VP, P_ELEMS = 4 * 16 * PP;
    static constexpr int BYTES = 2 * (K_ELEMS + V_ELEMS + P_ELEMS);
};

// operands written by earlier launches
struct LdPlain {
    static STZS_DEV uint4 ld(const bf16_t* base, long off) { return *reinterpret_cast<const uint4*>(base + off); }
};

// operands stored write-through (sc1) in this launch: every load of them sc1 (bypasses this CU's L1 and the
// XCD's L2 copy; MI355X guide Guideline 16, the sc1-load form of the hand-off).  base is wave-uniform.
// attention of queries [qb0, qb0 + 64) of row r, head h; lds >= Lds<DH>::BYTES, 16-B aligned
template <int DH, class LD>
STZS_DEV void attn_unit(const stzs_attn_args& a, long r, int h, int qb0, unsigned char* lds) {
    using LY = Lds<DH>;
    constexpr int NKS = DH / 32;  // k-steps of S
    constexpr int NDT = DH / 16;  // d tiles of O
    constexpr int KP = LY::KP, VP = LY::VP, PP = LY::PP;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Vt = Ks + LY::K_ELEMS;
    bf16_t* Ps = Vt + LY::V_ELEMS;
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int qb = qb0 + wave * 16;
    const bf16_t* Q = reinterpret_cast<const bf16_t*>(a.q) + r * a.bsq + h * DH;
    const bf16_t* K = reinterpret_cast<const bf16_t*>(a.k) + r * a.bsk + h * DH;
    const bf16_t* V = reinterpret_cast<const bf16_t*>(a.v) + r * a.bsv + h * DH;
    const float scale = 1.f / sqrtf((float)DH);

    bf16x8 qf[NKS];
    {
        const int qr = min(qb + (lane & 15), a.Lq - 1);
#pragma unroll
        for (int ks = 0; ks < NKS; ++ks)
            qf[ks] = __builtin_bit_cast(bf16x8, LD::ld(Q, (long)qr * a.ldq + ks * 32 + 8 * (lane >> 4)));
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
    bf16_t* P = Ps + wave * 16 * PP;

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
            pk[j] = LD::ld(K, (long)kk * a.ldk + cv * 8);
            pv[j] = LD::ld(V, (long)kk * a.ldv + cv * 8);
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

}  // namespace stzs_attn
