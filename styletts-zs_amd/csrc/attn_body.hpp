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

template <int CTRL>
STZS_DEV float dpp16(float x) {
    return __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), CTRL, 0xF, 0xF, true));
}
// x[i] reduced over the 16 lanes of each DPP row, the four values step-major (independent DPP reads between dependent
// ones); every lane of the row gets the result
STZS_DEV void row16_max4(float* x) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = fmaxf(x[i], dpp16<0xB1>(x[i]));  // quad_perm 1,0,3,2
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = fmaxf(x[i], dpp16<0x4E>(x[i]));  // quad_perm 2,3,0,1
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = fmaxf(x[i], dpp16<0x141>(x[i]));  // row_half_mirror
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] = fmaxf(x[i], dpp16<0x140>(x[i]));  // row_mirror
}
STZS_DEV void row16_sum4(float* x) {
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] += dpp16<0xB1>(x[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] += dpp16<0x4E>(x[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] += dpp16<0x141>(x[i]);
#pragma unroll
    for (int i = 0; i < 4; ++i) x[i] += dpp16<0x140>(x[i]);
}

template <int DH>
struct Lds {
    static constexpr int KP = DH + 8;  // K row pitch (bf16)
    static constexpr int VP = DH + 8;  // V row pitch (row-major: the PV B fragments by transposed reads)
    static constexpr int PTP = 16 + 4;  // P^T row pitch (a wave's [64 keys][16 queries], 8-B aligned rows)
    static constexpr int K_ELEMS = KC * KP, V_ELEMS = KC * VP, P_ELEMS = 4 * KC * PTP;
    static constexpr int BYTES = 2 * (K_ELEMS + V_ELEMS + P_ELEMS);
};

typedef short stzs_v4s __attribute__((ext_vector_type(4)));
// gfx950 ds_read_b64_tr_b16: per 16-lane group a 4-row x 16-column block of 16-bit elements, lane 4q+p addressing
// row q, columns 4p..4p+3; lane i receives column i of the 4 rows (row q in element q) -- cdna_hip_programming.md T10
STZS_DEV uint2 ld_tr16(const bf16_t* p) {
    const stzs_v4s v = __builtin_amdgcn_ds_read_tr16_b64_v4i16((__attribute__((address_space(3))) stzs_v4s*)(p));
    return __builtin_bit_cast(uint2, v);
}
// the 16x16x32 MFMA operand whose lane (n, g) holds elements [k0 + 8g + j][c0 + n], j < 8, of a row-major [k][c] LDS
// image with pitch `ld` (two transposed reads: rows k0 + 8g + 0..3 and + 4..7).  EXEC must be full.
STZS_DEV bf16x8 frag_tr(const bf16_t* img, int ld, int k0, int c0, int lane) {
    const int g = lane >> 4, q = (lane >> 2) & 3, p = lane & 3;
    const bf16_t* a = img + (k0 + 8 * g + q) * ld + c0 + 4 * p;
    const uint2 lo = ld_tr16(a), hi = ld_tr16(a + 4 * ld);
    return __builtin_bit_cast(bf16x8, make_uint4(lo.x, lo.y, hi.x, hi.y));
}

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
    constexpr int KP = LY::KP, VP = LY::VP, PTP = LY::PTP;
    bf16_t* Ks = reinterpret_cast<bf16_t*>(lds);
    bf16_t* Vs = Ks + LY::K_ELEMS;
    bf16_t* Ps = Vs + LY::V_ELEMS;
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
    bf16_t* Pt = Ps + wave * KC * PTP;  // this wave's P^T [key][query]

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
        // stage K and V rows for keys [c0, c0 + KC) from the registers (both row-major: V's PV fragments come from
        // transposed reads, r06 -- it was a scalar transposing store), then start the next chunk's loads
#pragma unroll
        for (int j = 0; j < NLD; ++j) {
            const int i = tid + j * 256;
            const int kr = i / (DH / 8), cv = i - kr * (DH / 8);
            *reinterpret_cast<uint4*>(Ks + kr * KP + cv * 8) = pk[j];
            *reinterpret_cast<uint4*>(Vs + kr * VP + cv * 8) = pv[j];
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
        // online softmax; element (row = (lane>>4)*4 + i, key = nt*16 + (lane & 15)).  The 16-lane row max / sum run
        // on DPP (quad_perm 1,0,3,2 / 2,3,0,1, row_half_mirror, row_mirror) instead of xor shuffles through
        // ds_bpermute: after the two quad steps every lane of a quad holds the same value, so the mirror partners
        // contribute exactly what the xor-4 / xor-8 partners did -- the same bits, at VALU latency (r06)
        float alpha[4], mx[4], sum[4];
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
        row16_max4(mx);
#pragma unroll
        for (int i = 0; i < 4; ++i) {
            const float mn = fmaxf(m[i], mx[i]);
            alpha[i] = __expf(m[i] - mn);
            sum[i] = 0.f;
#pragma unroll
            for (int nt = 0; nt < 4; ++nt) {
                const float pv = __expf(s[nt][i] - mn);
                s[nt][i] = pv;
                sum[i] += pv;
            }
            m[i] = mn;
        }
        row16_sum4(sum);
#pragma unroll
        for (int i = 0; i < 4; ++i) l[i] = l[i] * alpha[i] + sum[i];
#pragma unroll
        for (int dt = 0; dt < NDT; ++dt)
#pragma unroll
            for (int i = 0; i < 4; ++i) o[dt][i] *= alpha[i];
        // P -> LDS as P^T (lane (n, g) holds queries 4g..4g+3 of key nt*16 + n: one 8-B store per key tile) -> A
        // fragments by transposed reads (lane (n, g): query n, keys ks*32 + 8g + j); the same bf16 values as before
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) {
            const uint2 pq = make_uint2(pack2bf(s[nt][0], s[nt][1]), pack2bf(s[nt][2], s[nt][3]));
            *reinterpret_cast<uint2*>(Pt + (nt * 16 + (lane & 15)) * PTP + 4 * (lane >> 4)) = pq;
        }
        __syncthreads();
#pragma unroll
        for (int ks = 0; ks < KC / 32; ++ks) {
            const bf16x8 pf = frag_tr(Pt, PTP, ks * 32, 0, lane);
#pragma unroll
            for (int dt = 0; dt < NDT; ++dt) {
                const bf16x8 vf = frag_tr(Vs, VP, ks * 32, dt * 16, lane);
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
