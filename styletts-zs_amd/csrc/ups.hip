// The generator's up-sampling ConvTranspose1d as a polyphase conv, input staged ONCE.
//
// ConvTranspose1d(k = 2r, stride r) is a 2-tap conv over the input rows (pad 1) with r * Co output columns: column
// p * Co + co of GEMM row q lands at output time t = q r + p - pad_up (stzs/weights.py pack_conv(ups=r)).  The
// general MRF-family kernel gives every 128-column tile its own workgroup, and each of them stages (loads + LeakyReLU
// + bf16 LDS image) the same input rows again: the stage-1 ConvT (r = 6: 6 tiles) read its 131 MB input 6 times and
// ran at 0.25 of its HBM roofline (462 us for 917 MB of algorithmic traffic at batch 64).  Here one workgroup:
//   * stages the 129 input rows of its 128-row tile for EVERY 128-channel chunk once (LDS: chunks x 37 KB), and
//   * walks its column tiles (all of them, or a slice for very wide layers) over that resident tile, the
//     register-direct way of csrc/mrfv.hip: each wave owns 32 output columns, its weight fragments
//     (STZS_CONV_W_FRAG32 packing) come straight from global memory into VGPRs through a 4-deep register ring that
//     runs ahead ACROSS column tiles, the input fragments come from LDS, and there is no barrier in the K loop;
//   * the epilogue of each tile is straight from the accumulators (lane (g, n): 8 consecutive channels of one
//     input row q -> output row q r + p - pad_up): bias, the noise-conv residual at that row (loaded at the
//     start of the tile's K loop, its latency under the MFMAs), ReflectionPad(1,0) on the last stage.
// Same staged bf16 operands and the same K order per output element (chunk, tap, 32-wide k-step) as csrc/mrf.hip:
// bit-identical to the LANE16 form (tests/test_gpu_ops.py).
#include "common.hpp"

namespace {

constexpr int NTH = 256;
#ifndef STZS_UPS_P
#define STZS_UPS_P 288
#endif
constexpr int P = STZS_UPS_P;             // staged row pitch, bytes (288: conflict-free ds_read_b128, csrc/mrfv.hip)
// BT: q rows per tile, 128 or 64 (r06: the 512-channel first stage -- 4 chunks x 37 KB of staged rows held ONE
// workgroup per CU at 128 rows, and its 401-row utterances filled 4 x 128 tiles to 78 %); the same K order per output
// element either way: bit-identical
constexpr int rows_of(int bt) { return bt + 1; }  // a 2-tap conv at pad 1: rows q0 - 1 .. q0 + bt - 1
constexpr int tile_of(int bt) { return (rows_of(bt) * P + 15) & ~15; }
constexpr int RING = 4;                   // weight K-steps in flight (3 ahead); divides every NK (8 per chunk)

// NZ (STZS_CONV_UPS_NOISE): the 1x1 noise conv fused as one more K-step per column tile whose B operand is the
// harmonic-source rows of the tile's output rows (loaded at the tile's start, as the residual rows were) and whose
// weights follow the tile's ConvTranspose K-steps in the stream; there is then no residual operand.
template <int NCH, bool HR, bool NZ, int BT = 128>
__global__ __launch_bounds__(NTH, NCH * tile_of(BT) <= 80 * 1024 ? 2 : 1) void ups_conv(const stzs_conv_args a, int ctw) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int ROWS = rows_of(BT), TILE = tile_of(BT);
    constexpr int SB = (ROWS + 15) / 16;  // staged 16-B vectors per thread (16 row lanes)
    constexpr int MT = BT / 16;           // 16-row input fragments per wave
    constexpr int NK = NCH * 8;  // K-steps per column tile: chunks x 2 taps x 4
    constexpr int NKW = NK + (NZ ? 1 : 0);  // weight-stream K-steps per column tile
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int nx = gridDim.x;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * nx + blockIdx.x
                                                      : xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y);
    const int gy = lin / nx, bx = lin - gy * nx;
    const int bq = bx / tpb;
    const int q0 = (bx - bq * tpb) * BT;
    const int ncol = a.ups * a.Co;
    const int nct = (ncol + 127) / 128;
    const int ct0 = gy * ctw, ct1 = min(nct, ct0 + ctw);
    const int J = (ct1 - ct0) * NK;  // this workgroup's ConvTranspose K-steps over all its tiles
    const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + (long)ct0 * NKW * 512 + wave * 128 + lane;
    bf16x8 wf[RING][2];
    auto wload = [&](int j, int slot) {  // j >= J: a harmless re-load of the last K-step
        const int jj = j < J ? j : J - 1;
        const bf16x8* p = Wf + (long)(NZ ? (jj / NK) * NKW + jj % NK : jj) * 512;
        wf[slot][0] = p[0];
        wf[slot][1] = p[64];
    };
#pragma unroll
    for (int i = 0; i < RING - 1; ++i) wload(i, i);  // the first weights fly during the staging
    // ---- staging: every chunk's 129 rows, LeakyReLU, bf16, once ----
    const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (long)bq * a.bsx;
    const int cv = tid & 15, rsub = tid >> 4;
    const float slope = a.pro_slope;
    const bool lrelu = a.pro_act == STZS_ACT_LEAKY;
#pragma unroll
    for (int cc = 0; cc < NCH; ++cc) {
        const int c = cc * 128 + cv * 8;
        const bool c_ok = c < a.Ci;
        const int cl = c_ok ? c : 0;
        uint4 raw[SB];
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            int tin = q0 - 1 + rsub + 16 * i;
            tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
            raw[i] = *reinterpret_cast<const uint4*>(X + (long)tin * a.ldx + cl);
        }
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            const int r = rsub + 16 * i;
            const int tin = q0 - 1 + r;
            const bool ok = c_ok && tin >= 0 && tin < a.T_in;
            const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
            uint32_t o[4];
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                // x * 1 + 0 as the MRF-family staging computes it (fmaf(x, cscale, shift)): -0 becomes +0 there too
                float y0 = __uint_as_float(w[p] << 16) + 0.f, y1 = __uint_as_float(w[p] & 0xFFFF0000u) + 0.f;
                if (lrelu) {
                    y0 = y0 >= 0.f ? y0 : y0 * slope;
                    y1 = y1 >= 0.f ? y1 : y1 * slope;
                }
                o[p] = ok ? pack2bf(y0, y1) : 0u;
            }
            if (r < ROWS) *reinterpret_cast<uint4*>(smem + cc * TILE + r * P + cv * 16) = make_uint4(o[0], o[1], o[2], o[3]);
        }
    }
    __syncthreads();
    // ---- column tiles over the resident input ----
    const int g = lane >> 4, n = lane & 15;
    const int xoff0 = (lane & 15) * P + (lane >> 4) * 16;
    const int t_hi = a.T_final + a.refl - 1;
    const bf16_t* Rb = reinterpret_cast<const bf16_t*>(a.res) + (long)bq * a.bsr;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y) + (long)bq * a.bsy;
    f32x4 acc[2][MT];
    bf16x8 xf[MT];
    for (int ct = ct0; ct < ct1; ++ct) {
        const int jb = (ct - ct0) * NK;
        // this tile's output rows / channels and its residual rows, loaded now (consumed after the K loop)
        const int col0 = ct * 128 + wave * 32 + g * 8;
        const int ph = col0 / a.Co, cof = col0 - ph * a.Co;
        const bool col_ok = col0 < ncol;
        const int cofc = col_ok ? cof : 0;
        uint4 rr[MT];  // residual rows (HR) or, fused noise conv (NZ), the harmonic-source B fragments
        int trow[MT];
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int q = q0 + mt * 16 + n;
            const int t = q * a.ups + ph - a.ups_pad + a.refl;
            trow[mt] = t;
            const int tc = t < 0 ? 0 : (t > t_hi ? t_hi : t);
            if constexpr (NZ) rr[mt] = *reinterpret_cast<const uint4*>(Rb + (long)tc * a.ldr + g * 8);
            else if constexpr (HR) rr[mt] = *reinterpret_cast<const uint4*>(Rb + (long)tc * a.ldr + cofc);
        }
        bf16x8 wn[2];  // the noise conv's A fragments for this tile's 32 columns of the wave
        if constexpr (NZ) {
            const bf16x8* pn = Wf + (long)((ct - ct0) * NKW + NK) * 512;
            wn[0] = pn[0];
            wn[1] = pn[64];
        }
        float bias[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[cofc + i] : 0.f;
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(smem + xoff0 + mt * 16 * P);
        const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
        for (int s = 0; s < NK; ++s) {
            wload(jb + s + RING - 1, (s + RING - 1) % RING);
            const int sn = s + 1;  // next K-step's input fragments: chunk sn / 8, tap (sn / 4) & 1, kq sn & 3
            const int offn = (sn >> 3) * TILE + ((sn >> 2) & 1) * P + (sn & 3) * 64;
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s % RING][0], xf[mt], s == 0 ? zero : acc[0][mt], 0, 0, 0);
                acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s % RING][1], xf[mt], s == 0 ? zero : acc[1][mt], 0, 0, 0);
                if (sn < NK) xf[mt] = *reinterpret_cast<const bf16x8*>(smem + xoff0 + offn + mt * 16 * P);
            }
            __builtin_amdgcn_sched_group_barrier(0x020, 2, 0);  // the two weight loads first
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                if (sn < NK) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
            }
            __builtin_amdgcn_sched_barrier(0);
        }
        if constexpr (NZ) {  // the fused noise conv: one more K-step on the harmonic-source rows
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) {
                const bf16x8 hf = __builtin_bit_cast(bf16x8, rr[mt]);
                acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wn[0], hf, acc[0][mt], 0, 0, 0);
                acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wn[1], hf, acc[1][mt], 0, 0, 0);
            }
        }
        if (a.flags & 4) continue;  // diagnostic (tools/ups_bench.py): no epilogue
        // NZ, ReflectionPad(1,0): output row 0 takes row 2's ConvTranspose value (q = 0: the first row of the
        // workgroup's first 16-row tile) and row 0's noise term: the correction W_noise (har[0] - har[2]) in fp32,
        // computed once, outside the unrolled epilogue, by the lanes that hold q = 0
        float corr[8] = {0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f, 0.f};
        if constexpr (NZ) {
            if (a.refl && q0 == 0 && n == 0 && trow[0] == 2 && col_ok) {
#pragma unroll 1
                for (int j = 0; j < 32; ++j) {
                    const float d = bf2f(Rb[j]) - bf2f(Rb[2 * a.ldr + j]);
#pragma unroll
                    for (int i = 0; i < 8; ++i) corr[i] = fmaf(a.gate[(long)(cof + i) * 32 + j], d, corr[i]);
                }
            }
        }
        // epilogue: row q -> t = q ups + p - pad_up (+ refl), valid for q < T_out and t in [0, T_final)
#pragma unroll
        for (int mt = 0; mt < MT; ++mt) {
            const int q = q0 + mt * 16 + n;
            const int t = trow[mt];
            const int tp = t - a.refl;
            const bool ok = col_ok && q < a.T_out && tp >= 0 && tp < a.T_final;
            float v[8];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[nt][mt][r] + bias[nt * 4 + r];
            float w0[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) w0[i] = v[i];
            if constexpr (HR) {
                float f[8];
                unpack8(rr[mt], f);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] += f[i];
            }
#pragma unroll
            for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
            if (ok) *reinterpret_cast<uint4*>(Y + (long)t * a.ldy + cof) = pack8(v);
            if (a.refl && ok && t == 2) {  // ReflectionPad(1,0): row 0 mirrors source row 1 (+ row 0's residual)
                if constexpr (NZ) {  // the accumulator holds row 2's noise term: + W_noise (har[0] - har[2])
#pragma unroll
                    for (int i = 0; i < 8; ++i) w0[i] += corr[i];
                } else if constexpr (HR) {
                    float f[8];
                    load8(Rb + cof, f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) w0[i] += f[i];
                }
#pragma unroll
                for (int i = 0; i < 8; ++i) w0[i] *= a.alpha;
                *reinterpret_cast<uint4*>(Y + cof) = pack8(w0);
            }
        }
    }
}

}  // namespace

// internal entry (csrc/mrfv.hip routes FRAG32 weights with ups > 0 here)
__attribute__((visibility("hidden"))) int stzs_ups_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    const bool nz = (a.flags & STZS_CONV_UPS_NOISE) != 0;
    if (nz && (!a.res || !a.gate || a.Co % 128 || a.refl < 0 || a.refl > 1 || a.ldr < 32 || a.ldr % 8 || a.bsr % 8 ||
               (a.refl && a.T_final + a.refl < 3)))
        return STZS_EINVAL;  // fused noise conv: harmonic-source rows (>= 32 channels) + fp32 noise weights required
    if (a.ks != 2 || a.pad != 1 || a.dil != 1 || a.stride != 1 || a.cic != 128 || a.ci_pad % 128 || a.Co % 32 ||
        a.T_out != a.T_in + 1 || a.in_dtype != STZS_BF16 || a.out_dtype != STZS_BF16 || a.pro_mode != STZS_PRO_NONE ||
        (a.pro_act != STZS_ACT_LEAKY && a.pro_act != STZS_ACT_NONE) || a.pro_cscale != 1.f || (a.gate && !nz) || a.acc_in ||
        a.stat_part || a.epi_act != STZS_ACT_NONE || a.ldy % 8 || a.bsy % 8 ||
        (a.res && (a.ldr % 8 || a.bsr % 8 || a.res_tdiv != 1)) || a.co_pad < a.ups * a.Co)
        return STZS_ESHAPE;
    const int nch = a.ci_pad / 128;
    const int nct = (a.ups * a.Co + 127) / 128;
    // 64-row q tiles where the 128-row form's staged chunks hold one workgroup per CU (more than two chunks);
    // STZS_UPS_BT=128 / 64 forces a form (A/B)
    static const int bt_env = [] {
        const char* e = getenv("STZS_UPS_BT");
        return e ? atoi(e) : 0;
    }();
    const int BT = bt_env == 64 || bt_env == 128 ? bt_env : (nch > 2 ? 64 : 128);
    const int nqt = a.B * ((a.T_out + BT - 1) / BT);
    // column tiles per workgroup: all of them (input staged once), unless the q-tile grid alone leaves most of the
    // chip idle (the 40-fps first stage: 128 q tiles at batch 64) -- then slices, ~4 workgroups per CU in total
    const int target = 4 * stzs_cu_count();
    int groups = 1;
    while (groups < nct && (long)nqt * groups < target) ++groups;
    const int ctw = (nct + groups - 1) / groups;
    groups = (nct + ctw - 1) / ctw;
    const size_t lds = (size_t)nch * (BT == 64 ? tile_of(64) : tile_of(128));
    void (*k)(stzs_conv_args, int) = nullptr;
    const bool R = a.res != nullptr;
#define STZS_UPS_PICK(N, B_)                                                                                    \
    k = nz ? ups_conv<N, false, true, B_> : R ? ups_conv<N, true, false, B_> : ups_conv<N, false, false, B_>;
    switch (nch * (BT == 64 ? -1 : 1)) {
        case 1: STZS_UPS_PICK(1, 128) break;
        case 2: STZS_UPS_PICK(2, 128) break;
        case 3: STZS_UPS_PICK(3, 128) break;
        case 4: STZS_UPS_PICK(4, 128) break;
        case -1: STZS_UPS_PICK(1, 64) break;
        case -2: STZS_UPS_PICK(2, 64) break;
        case -3: STZS_UPS_PICK(3, 64) break;
        case -4: STZS_UPS_PICK(4, 64) break;
        default: return STZS_ESHAPE;
    }
#undef STZS_UPS_PICK
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, dim3((unsigned)nqt, (unsigned)groups), dim3(NTH), lds, s, a, ctw);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
