#pragma once
// mrfv_conv, the kernel template (csrc/mrfv.hip: launcher + multi-chunk / wide / AdaIN-block forms; csrc/mrfv_n1.hip:
// the single-chunk stage-1 forms).
// The MRF conv, register-direct weight form (SURVEY.md §8(a) a12 -- the generator's AdaINResBlock1
// convs -- and the k3 convs of the decoder / predictor AdaIN residual blocks, a9).
//
// Same arithmetic as csrc/mrf.hip (same K order per output element, same staged bf16 operands, so the
// two kernels are bit-identical), different data movement:
//  * the 4 waves of a 256-thread workgroup split the 128 OUTPUT CHANNELS (32 each) instead of a 2 x 2
//    grid, so every wave needs every time row of the staged input tile (8 B-fragments per K-step from
//    LDS, 50% of the LDS read rate at the MFMA rate) but only ITS 32 channels of the weights: 2
//    A-fragments per K-step, read straight into VGPRs with one coalesced 16-B load per lane each
//    (weights packed in fragment order, STZS_CONV_W_FRAG32) and prefetched two K-steps ahead;
//  * so the K loop has no weight ring, no LDS-DMA and no barrier at all -- the only barriers are the
//    two around the staging of each 128-channel input chunk;
//  * LDS = the staged input tile only (<= 51 KB at pitch 288), several workgroups per CU: one workgroup's staging
//    (HBM latency + the AdaIN / Snake VALU work) overlaps the others' MFMAs.
// Epilogue straight from the accumulators: lane (g, n) holds 8 consecutive channels (packed row
// w*32 + nt*16 + 4g + r <-> channel w*32 + g*8 + nt*4 + r) of one time row -> 16-B residual /
// accumulate loads and stores; fused InstanceNorm statistics per 64-row chunk as in mrf.hip.
#include "common.hpp"

#include <type_traits>

#ifndef STZS_MRFV_OCC
#define STZS_MRFV_OCC 2
#endif
#ifndef STZS_MRFV_OCC1
#define STZS_MRFV_OCC1 3
#endif

namespace {

constexpr int NTH = 256;
constexpr int BCO = 128;
// staged input row pitch, bytes.  A B fragment is read by lane (n = lane & 15, g = lane >> 4) at row rb + n, 16-B chunk
// g + 4 kq; ds_read_b128 serves 64 lanes in four 16-lane groups ({0-3, 12-15, 20-27}, {4-11, 16-19, 28-31}, +32) whose
// lanes conflict on a 16-B bank slot (a / 16) mod 16.  At pitch 272 the slot is (rb + n + c) mod 16 and every group has
// one 2-way collision (group 0: n = 12 at chunk g and n = 11 at chunk g + 1), i.e. 8 LDS cycles per read instead of 4
// (SQ: conflict share 0.505, profiles/r05_g_sq_k11_full.json) -- at the MFMA rate the B reads then need the whole LDS.
// At pitch 288 the slot is (2 (rb + n) + c) mod 16: within a group the chunk-g lanes land on slots of one parity and the
// chunk-(g + 1) lanes on the other, 8 distinct slots each for ANY row base rb (every tap / dilation): conflict-free.
#ifndef STZS_MRFV_P
#define STZS_MRFV_P 288
#endif
constexpr int P = STZS_MRFV_P;
// staged 16-B vectors per thread (16 rows each): rows_in = 128 + (KS - 1) dil <= 16 SB.  Sized per kernel width
// (k3: dil <= 8; k7 / k11: dil <= 5), not for the widest: every staged vector costs its transform (the cosines
// of the Snake) whether or not its row is used, and a k3 tile with SB = 12 transformed 192 rows for 130-138
// (ks 1, r06: the AdaIN blocks' 1x1 shortcut convs -- no halo)
constexpr int sb_rows(int ks) { return ks == 1 ? 8 : ks == 3 ? 9 : (ks == 7 ? 10 : 12); }
// the 64-row tiles (BT 64, small grids): 64 + (ks - 1) dil rows
constexpr int sb_rows64(int ks) { return ks == 1 ? 4 : ks == 3 ? 5 : (ks == 7 ? 6 : 8); }
constexpr int SB_MAX = 12;
constexpr int CS_BYTES = 5 * 128 * 4;  // per-channel prologue constants
// At pitch >= 288 the constants live in the rows' 32 pad bytes (bytes 256..287, never read or written by the tile's
// staging / K loop): float i at row i / 8, byte 256 + 4 (i % 8) -- 80 rows; the tile then costs rows x P bytes and
// the k11 d5 tile (178 rows, 51.3 KB) still fits three workgroups per CU (with the constants appended, 53.8 KB, it
// did not: 593 vs 555 us per stage-1 k11 launch, profiles/r06a_mrfv_*.log)
constexpr bool CS_IN_PAD = P >= 288;
constexpr int CS_ROWS = 5 * 128 / 8;
STZS_DEV float* cs_at(unsigned char* smem, int rows_in, int i) {
    if constexpr (CS_IN_PAD) return reinterpret_cast<float*>(smem + (i >> 3) * P + 256 + (i & 7) * 4);
    return reinterpret_cast<float*>(smem + ((rows_in * P + 15) & ~15)) + i;
}
// dynamic LDS bytes of a tile of `rows` staged rows
inline size_t mrfv_lds(int rows) {
    if (CS_IN_PAD) return (size_t)(rows > CS_ROWS ? rows : CS_ROWS) * P;
    return (((size_t)rows * P + 15) & ~(size_t)15) + CS_BYTES;
}

// x[0..N) summed over the 16 lanes of each DPP row, in place, VALU only.  Each step is ONE v_add_f32 with the DPP
// permutation on its first source (hipcc emitted a v_mov_b32_dpp + v_add_f32 pair per step); the N values go
// step-major, so a value's next step issues N instructions after the write it reads (DPP read-after-VALU-write
// needs 2 wait states; N >= 8 here).  Same additions in the same order as x += dpp(x): bit-identical.
template <int N>
STZS_DEV void row_sum16_n(float* x) {
    static_assert(N >= 4, "dependent DPP steps need >= 2 independent instructions between them");
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[1,0,3,2] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 quad_perm:[2,3,0,1] row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_half_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
#pragma unroll
    for (int i = 0; i < N; ++i) asm volatile("v_add_f32_dpp %0, %0, %0 row_mirror row_mask:0xf bank_mask:0xf" : "+v"(x[i]));
}

// STZS_MRFV_PROF probe build (tools/mrfv_phase.py --build; never in the library build): thread 0 of every workgroup
// stamps into g_mprof[workgroup][8]: s_memtime at entry (0), after the staging barrier (1), after the K loop (2), after
// the epilogue's stores issued (3) and drained (4); s_memrealtime (100 MHz) at entry (5) and exit (6); HW_ID | XCC_ID << 32
// (7).  Workgroup = dispatch index blockIdx.y * gridDim.x + blockIdx.x.  STZS_MRFV_DIAG=2 (probe only): no row loads.
#ifdef STZS_MRFV_PROF
__device__ unsigned long long g_mprof[8 * 16384];
#define MPROF(i, v)                                                                    \
    if (threadIdx.x == 0) {                                                            \
        const unsigned wg_ = blockIdx.y * gridDim.x + blockIdx.x;                     \
        if (wg_ < 16384) g_mprof[wg_ * 8 + (i)] = (v);                                 \
    }
#else
#define MPROF(i, v)
#endif

// NCH = 1: exactly one 128-channel input chunk (the stage-1 generator convs): the accumulators are not live
// during the staging, so the kernel fits 3 workgroups per CU; NCH = 0: any number of chunks, 2 per CU.
// AL: the epilogue scales by a.alpha (alpha != 1; a uniform runtime test was if-converted into a multiply + select
// per element)
// WPW: 32-channel weight groups per wave.  1: a workgroup owns 128 output channels; 2 (the wide form, multi-chunk
// inputs with co_pad % 256 == 0): 256, so a 256-channel layer stages (loads + AdaIN + Snake) each input row ONCE
// instead of once per 128-channel tile, and every B fragment read from LDS feeds 4 MFMAs instead of 2.  Same K
// order per output element either way (bit-identical).
// BT: time rows per tile, 128 or 64 (r05: small grids -- batch 1 -- where the 128-row tiles leave CUs idle).  The
// staged operands, the K order of every output element and the 64-row statistics chunks are the same: bit-identical.
// (r06) the body as an always-inlined device function: the kernel mrfv_conv below is this body alone (same code
// object), mrfv_trio runs three of them in one launch.
template <int PACT, bool HR, bool HA, int KS, int NCH, bool AL, int WPW = 1, int BT = 128>
STZS_DEV void mrfv_body(const stzs_conv_args a) {
    static_assert(WPW == 1 || (WPW == 2 && NCH != 1), "the wide form is for multi-chunk inputs");
    static_assert(BT == 128 || (BT == 64 && WPW == 1), "64-row tiles: narrow form");
    MPROF(5, __builtin_amdgcn_s_memrealtime())
    MPROF(0, __builtin_amdgcn_s_memtime())
    MPROF(7, (unsigned long long)__builtin_amdgcn_s_getreg(4 | (31 << 11)) |
                 ((unsigned long long)__builtin_amdgcn_s_getreg(0x14 | (3 << 11)) << 32))
    constexpr int NA = 2 * WPW;  // A fragments (16 output channels each) per wave and K-step
    constexpr int MT = BT / 16;  // 16-row B fragments per wave
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int NKC = KS * 4;  // 32-wide K-steps per 128-channel chunk
    const int dil = a.dil;
    const int rows_in = BT + (KS - 1) * dil;
    auto cs = [&](int i) { return cs_at(smem, rows_in, i); };
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int nx = gridDim.x;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * nx + blockIdx.x
                                                      : xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y);
    const int by = lin / nx, bx = lin - by * nx;  // (co tile, utterance x time tile)
    const int bq = bx / tpb;
    const int t0 = (bx - bq * tpb) * BT;
    const int nchunk = NCH ? NCH : a.ci_pad >> 7;
    constexpr int SB = BT == 128 ? sb_rows(KS) : sb_rows64(KS);
    // weights: [co tile][chunk][tap][kq][wave][nt][lane][8] bf16 -> 512 bf16x8 per K-step.  Wide form: wave w takes
    // the packed waves 2 (w & 1) and 2 (w & 1) + 1 of 128-channel tile 2 by + (w >> 1) -- consecutive in the stream
    const int ct = WPW == 1 ? by : by * 2 + (wave >> 1);
    const int ow0 = WPW == 1 ? wave : (wave & 1) * 2;
    const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + ((long)ct * nchunk * NKC) * 512 + ow0 * 128 + lane;
    auto wload = [&](bf16x8 (&w)[NA], int kk) {
        const bf16x8* p = Wf + (long)kk * 512;
#pragma unroll
        for (int j = 0; j < NA; ++j) w[j] = p[64 * j];
    };
    f32x4 acc[NA][MT];

    const int xoff0 = (lane & 15) * P + (lane >> 4) * 16;
    const int dP = dil * P;
    const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (long)bq * a.bsx;
    const int cv = tid & 15, rsub = tid >> 4;
#ifndef STZS_MRFV_PD
#define STZS_MRFV_PD 2
#endif
    // weight K-steps in flight ahead of the MFMAs (the wide form's K-step is twice as long: one is as far ahead in
    // time, and two spill its 256 VGPRs)
    constexpr int PD = WPW == 2 ? 1 : STZS_MRFV_PD;
    bf16x8 wf[PD + 1][NA];
    bf16x8 xf[MT];
    // PF (r05, the multi-chunk LeakyReLU / identity block convs): the NEXT input chunk's raw rows and AdaIN
    // constants are loaded into registers right after this chunk's staging, so they fly under this chunk's K loop
    // instead of being waited for at the next chunk's start (9 chunks per decoder conv: one staging latency each).
    // Same values staged, same K order: bit-identical to the in-place loads.
    constexpr bool PF = NCH == 0 && WPW == 1 && PACT != STZS_ACT_SNAKE;
    uint4 rawn[PF ? SB : 1];
    float pmu = 0.f, prs = 0.f, pgm = 0.f, pbe = 0.f;
    auto prefetch = [&](int cn) {  // chunk cn's rows (clamped addresses: the interior tiles' addresses unchanged)
        const int c = cn * 128 + cv * 8;
        const int cl = c < a.Ci ? c : 0;
#pragma unroll
        for (int i = 0; i < SB; ++i) {
            int tin = t0 - a.pad + rsub + 16 * i;
            tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
            rawn[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(X) + (unsigned)(tin * (int)a.ldx + cl) * 2u);
        }
        if (tid < 128 && a.pro_mode == STZS_PRO_ADAIN) {
            const int ch = cn * 128 + tid;
            const int chl = ch < a.Ci ? ch : 0;
            pmu = a.pro_mean[(long)bq * a.stat_bs + chl];
            prs = a.pro_rstd[(long)bq * a.stat_bs + chl];
            pgm = a.pro_gb[(long)bq * a.gb_bs + chl];
            pbe = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + chl];
        }
    };
    if constexpr (PF) {
        if (!(a.flags & 1)) prefetch(0);
    }

    for (int cc = 0; cc < nchunk; ++cc) {
        const int kb = cc * NKC;
#pragma unroll
        for (int i = 0; i < PD; ++i) wload(wf[i], kb + i);  // the chunk's first PD weight K-steps fly during the staging
        __syncthreads();  // every wave is done reading the previous chunk's tile and constants
#ifndef STZS_MRFV_NOSTAGE
        if (!(a.flags & 1)) {
#else
        if (0) {
#endif
            const int c = cc * 128 + cv * 8;
            const bool c_ok = c < a.Ci;  // vectors past Ci (ci_pad > Ci) are zero; weights there are 0
            const int cl = c_ok ? c : 0;
            // EARLY (r06, the single-chunk stage-1 forms): the tile's rows are loaded BEFORE the per-channel constants
            // below -- whose own global loads the constants block waits for -- instead of after them: one memory
            // latency per tile instead of two in series (tools/mrfv_phase.py: the staging phase is the longest phase of a
            // stage-1 workgroup).  Clamped addresses for every tile (an interior tile's are unchanged).  The multi-chunk
            // forms keep the old order: raw vectors live across the constants block spill the 256-VGPR wide form.
            constexpr bool EARLY = NCH == 1 && !PF;
            uint4 rawe[EARLY ? SB : 1];
            if constexpr (EARLY) {
#pragma unroll
                for (int i = 0; i < SB; ++i) {
                    int tin = t0 - a.pad + rsub + 16 * i;
                    tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                    const unsigned off = (unsigned)(tin * (int)a.ldx + cl) * 2u;
#if defined(STZS_MRFV_PROF) && STZS_MRFV_DIAG == 2
                    rawe[i] = make_uint4(off, off ^ 1u, off ^ 2u, off ^ 3u);  // (probe: no loads, same transform)
#else
                    rawe[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(X) + off);
#endif
                }
            }
            // per-channel constants (128 threads):  t = x*ka + kb (revolutions of cos(2 a y)),
            // out = cos(t) * km + (x*ksc + ksh)  [Snake]   or   out = act(x*ksc + ksh)
            if (tid < 128) {
                const int ch = cc * 128 + tid;
                const bool ok = ch < a.Ci;
                float sc = 0.f, sh = 0.f;
                if (ok && a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = PF ? pmu : a.pro_mean[(long)bq * a.stat_bs + ch];
                    const float rs = PF ? prs : a.pro_rstd[(long)bq * a.stat_bs + ch];
                    const float gm = PF ? pgm : a.pro_gb[(long)bq * a.gb_bs + ch];
                    const float be = PF ? pbe : a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + ch];
                    sc = (1.f + gm) * rs;
                    sh = be - mu * sc;
                } else if (ok) {
                    sc = a.pro_cscale;
                }
                if constexpr (PACT == STZS_ACT_SNAKE) {
                    const float al = ok ? a.pro_alpha[ch] : 1.f;
                    const float h = 0.5f / al;
                    const float w = al * 0.318309886183790672f;  // a / pi
                    *cs(tid) = sc * w;
                    *cs(128 + tid) = sh * w;
                    *cs(256 + tid) = sc;
                    *cs(384 + tid) = sh + h;
                    *cs(512 + tid) = -h;
                } else {
                    *cs(256 + tid) = sc;
                    *cs(384 + tid) = sh;
                }
            }
            // the tile's rows (+ dilation halo): SB 16-B loads per thread, then the transform in registers, then the
            // LDS stores.  Interior tiles (every staged row inside [0, T_in), every channel < Ci: all but the first
            // and last tile of an utterance) take a path without the clamps and the zero-padding masks.
            auto stage = [&](auto full_tag) {
                constexpr bool FULL = decltype(full_tag)::value;
                uint4 raw[SB];
#pragma unroll
                for (int i = 0; i < SB; ++i) {  // 32-bit offsets from the utterance base (SGPR): saddr loads
                    if constexpr (PF) {
                        raw[i] = rawn[i];  // (loaded under the previous chunk's K loop)
                    } else if constexpr (EARLY) {
                        raw[i] = rawe[i];  // (loaded ahead of the constants)
                    } else {
                        int tin = t0 - a.pad + rsub + 16 * i;
                        if constexpr (!FULL) tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                        const unsigned off = (unsigned)(tin * (int)a.ldx + cl) * 2u;
                        raw[i] = *reinterpret_cast<const uint4*>(reinterpret_cast<const char*>(X) + off);
                    }
                }
                __syncthreads();  // constants visible
                // pair-major: the constants of one channel pair (10 registers) at a time, each vector's
                // pair transformed in place (the staging holds only the raw vectors + one pair's constants)
                const float slope = a.pro_slope;
                uint32_t* rw = reinterpret_cast<uint32_t*>(raw);
#pragma unroll
                for (int p = 0; p < 4; ++p) {
                    __builtin_amdgcn_sched_barrier(0);  // keep one pair's constants live at a time
                    const int c0 = cv * 8 + 2 * p;
                    const f32x2 ksc = *reinterpret_cast<const f32x2*>(cs(256 + c0));
                    const f32x2 ksh = *reinterpret_cast<const f32x2*>(cs(384 + c0));
                    f32x2 ka = {0.f, 0.f}, kbv = {0.f, 0.f}, km = {0.f, 0.f};
                    if constexpr (PACT == STZS_ACT_SNAKE) {
                        ka = *reinterpret_cast<const f32x2*>(cs(c0));
                        kbv = *reinterpret_cast<const f32x2*>(cs(128 + c0));
                        km = *reinterpret_cast<const f32x2*>(cs(512 + c0));
                    }
#pragma unroll
                    for (int i = 0; i < SB; ++i) {
                        const uint32_t w = rw[4 * i + p];
                        const f32x2 x = f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
                        f32x2 y = x * ksc + ksh;  // v_pk_fma_f32
                        if constexpr (PACT == STZS_ACT_SNAKE) {
                            const f32x2 t = x * ka + kbv;
                            const f32x2 cz = f32x2{__builtin_amdgcn_cosf(t.x), __builtin_amdgcn_cosf(t.y)};
                            y = cz * km + y;
                        } else if constexpr (PACT == STZS_ACT_LEAKY) {
                            y.x = y.x >= 0.f ? y.x : y.x * slope;
                            y.y = y.y >= 0.f ? y.y : y.y * slope;
                        }
                        if constexpr (FULL) {
                            rw[4 * i + p] = pack2bf(y.x, y.y);
                        } else {
                            const int tin = t0 - a.pad + rsub + 16 * i;  // zero padding / channels past Ci
                            const bool ok = c_ok && tin >= 0 && tin < a.T_in;
                            rw[4 * i + p] = ok ? pack2bf(y.x, y.y) : 0u;
                        }
                    }
                }
#pragma unroll
                for (int i = 0; i < SB; ++i) {
                    const int r = rsub + 16 * i;
                    if (r < rows_in) *reinterpret_cast<uint4*>(smem + r * P + cv * 16) = raw[i];
                }
            };
            const bool interior = t0 - a.pad >= 0 && t0 - a.pad + 16 * SB <= a.T_in && cc * 128 + 128 <= a.Ci;
            if (interior)
                stage(std::integral_constant<bool, true>{});
            else
                stage(std::integral_constant<bool, false>{});
        }
        __syncthreads();
        MPROF(1, __builtin_amdgcn_s_memtime())
        if constexpr (PF) {
            if (cc + 1 < nchunk && !(a.flags & 1)) prefetch(cc + 1);  // the next chunk flies under this K loop
        }
        // K loop: no barrier.  K-step s = tap*4 + kq reads input rows t + tap*dil, channels kq*32 ..
        // FIRST (the first chunk): K-step 0 takes the MFMA's inline-constant 0 as its C operand instead of 64
        // v_mov zeroings of the accumulators (the same sums: 0 + products either way)
        auto kloop = [&](auto first_tag) {
            constexpr bool FIRST = decltype(first_tag)::value;
            const f32x4 zero = {0.f, 0.f, 0.f, 0.f};
#pragma unroll
            for (int mt = 0; mt < MT; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(smem + xoff0 + mt * 16 * P);
#pragma unroll
            for (int s = 0; s < NKC; ++s) {
                if (s + PD < NKC) wload(wf[(s + PD) % (PD + 1)], kb + s + PD);
                const int sn = s + 1;
                const int offn = (sn >> 2) * dP + (sn & 3) * 64;
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    const bool z = FIRST && s == 0;
#pragma unroll
                    for (int j = 0; j < NA; ++j)
                        acc[j][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(wf[s % (PD + 1)][j], xf[mt], z ? zero : acc[j][mt], 0, 0, 0);
                    if (sn < NKC) xf[mt] = *reinterpret_cast<const bf16x8*>(smem + xoff0 + offn + mt * 16 * P);
                }
                if (s + 2 < NKC) {
                    __builtin_amdgcn_sched_group_barrier(0x020, NA, 0);  // the weight loads first
                }
#pragma unroll
                for (int mt = 0; mt < MT; ++mt) {
                    __builtin_amdgcn_sched_group_barrier(0x008, NA, 0);
                    if (sn < NKC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        };
        if constexpr (NCH == 1) {
            kloop(std::integral_constant<bool, true>{});
        } else {  // (two K-loop bodies spill the multi-chunk forms: zero the accumulators once instead)
            if (cc == 0) {
#pragma unroll
                for (int i = 0; i < NA; ++i)
#pragma unroll
                    for (int j = 0; j < MT; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
            }
            kloop(std::integral_constant<bool, false>{});
        }
    }
    MPROF(2, __builtin_amdgcn_s_memtime())
    if (a.flags & 4) return;

    // ---------------- epilogue: lane (g, n): time t = t0 + mt*16 + n, channels co0 .. co0 + 7
    const int g = lane >> 4, n = lane & 15;
    const bool stat = a.stat_part != nullptr;
    // residual rows at t / res_tdiv; the Snake (MRF) forms always have res_tdiv 1 (checked by the launcher)
    constexpr bool TD1 = PACT == STZS_ACT_SNAKE;
    const char* Rq = reinterpret_cast<const char*>(a.res) + (long)bq * a.bsr * 2;
    const char* Aq = reinterpret_cast<const char*>(a.acc_in) + (long)bq * a.bsa * 2;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);
    const int nch = (a.T_out + 63) / 64;
#pragma unroll
    for (int sw = 0; sw < WPW; ++sw) {  // (wide form: the wave's two 32-channel groups one after the other)
    const int co0 = ct * BCO + (ow0 + sw) * 32 + g * 8;
    const bool col_ok = co0 < a.Co;
    const int coc = col_ok ? co0 : 0;
    float bias[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[coc + i] : 0.f;
    // the residual / accumulate rows of BOTH halves in flight at once (the second half's HBM latency hides
    // behind the first half's epilogue); uniform utterance bases + 32-bit per-lane offsets
    uint4 rr[MT], aa[MT];
#pragma unroll
    for (int mt = 0; mt < MT; ++mt) {
        const int t = t0 + mt * 16 + n;
        const int tc = t < a.T_out ? t : a.T_out - 1;
        if constexpr (HR) {
            const int tr = TD1 ? tc : tc / a.res_tdiv;
            rr[mt] = *reinterpret_cast<const uint4*>(Rq + (unsigned)(tr * (int)a.ldr + coc) * 2u);
        }
        if constexpr (HA) aa[mt] = *reinterpret_cast<const uint4*>(Aq + (unsigned)(tc * (int)a.lda + coc) * 2u);
    }
#pragma unroll
    for (int h = 0; h < MT / 4; ++h) {  // 64-row halves: one statistics partial each
        float ss[8], sq[8];
#pragma unroll
        for (int i = 0; i < 8; ++i) ss[i] = sq[i] = 0.f;
#pragma unroll
        for (int m = 0; m < 4; ++m) {
            const int mt = h * 4 + m;
            const int t = t0 + mt * 16 + n;
            const bool ok = col_ok && t < a.T_out;
            float v[8];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[sw * 2 + nt][mt][r] + bias[nt * 4 + r];
            if constexpr (HR) {
                float f[8];
                unpack8(rr[mt], f);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] += f[i];
            }
            if constexpr (AL) {  // (x * 1 == x: the alpha == 1 forms skip it without changing a bit)
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
            }
            if constexpr (HA) {
                float f[8];
                unpack8(aa[mt], f);
#pragma unroll
                for (int i = 0; i < 8; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
            }
            const uint4 o = pack8(v);
            if (ok) *reinterpret_cast<uint4*>(Y + (long)bq * a.bsy + (long)t * a.ldy + coc) = o;
            if (stat && ok) {  // statistics of the stored (bf16-rounded) values
                float f[8];
                unpack8(o, f);
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    ss[i] += f[i];
                    sq[i] = fmaf(f[i], f[i], sq[i]);
                }
            }
        }
        if (stat) {
            row_sum16_n<8>(ss);
            row_sum16_n<8>(sq);
            const int r0 = t0 + h * 64;
            if (n == 0 && col_ok && r0 < a.T_out) {
                float* Pp = reinterpret_cast<float*>(a.stat_part) + (((long)bq * nch + r0 / 64) * a.stat_ld + co0) * 2;
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    Pp[2 * i] = ss[i];
                    Pp[2 * i + 1] = sq[i];
                }
            }
        }
    }
    }
#ifdef STZS_MRFV_PROF
    MPROF(3, __builtin_amdgcn_s_memtime())
    asm volatile("s_waitcnt vmcnt(0)" ::: "memory");
    MPROF(4, __builtin_amdgcn_s_memtime())
    MPROF(6, __builtin_amdgcn_s_memrealtime())
#endif
}

template <int PACT, bool HR, bool HA, int KS, int NCH, bool AL, int WPW = 1, int BT = 128>
__global__ __launch_bounds__(NTH, NCH == 1 ? STZS_MRFV_OCC1 : STZS_MRFV_OCC) void mrfv_conv(const stzs_conv_args a) {
    mrfv_body<PACT, HR, HA, KS, NCH, AL, WPW, BT>(a);
}

// (r06) the three resblocks' convs of one MRF layer (k 3 / 7 / 11, same input, same shape and form) in ONE launch: grid
// z = 0, 1, 2 runs the k11, k7, k3 problem (the longest workgroups dispatched first), each with its own arguments --
// every workgroup executes exactly the body of the single-problem kernel, so the outputs are bit-identical.  At batch 1
// a single conv fills 63 (stage 0) or 376 (stage 1) workgroups of 256 CUs and its time is latency, not throughput:
// side by side the three take little more than the k11 alone.  Snake prologue, no accumulate input, alpha 1, the narrow
// 64-row tiles (the small-grid form); csrc/mrfv.hip stzs_mrfv_trio_launch checks the rest.
template <bool HR, int NCH, int BT>
__global__ __launch_bounds__(NTH, NCH == 1 ? STZS_MRFV_OCC1 : STZS_MRFV_OCC) void mrfv_trio(const stzs_conv_args a3,
                                                                                        const stzs_conv_args a7,
                                                                                        const stzs_conv_args a11) {
    if (blockIdx.z == 0)
        mrfv_body<STZS_ACT_SNAKE, HR, false, 11, NCH, false, 1, BT>(a11);
    else if (blockIdx.z == 1)
        mrfv_body<STZS_ACT_SNAKE, HR, false, 7, NCH, false, 1, BT>(a7);
    else
        mrfv_body<STZS_ACT_SNAKE, HR, false, 3, NCH, false, 1, BT>(a3);
}

template <int PACT, bool HR, bool HA, int NCH, bool AL, int WPW = 1, int BT = 128>
void (*pick_ks(int ks))(stzs_conv_args) {
    switch (ks) {
        case 3: return mrfv_conv<PACT, HR, HA, 3, NCH, AL, WPW, BT>;
        case 7: return mrfv_conv<PACT, HR, HA, 7, NCH, AL, WPW, BT>;
        case 11: return mrfv_conv<PACT, HR, HA, 11, NCH, AL, WPW, BT>;
        default: return nullptr;
    }
}

}  // namespace

// the narrow single-chunk Snake forms (the stage-1 generator convs, NCH = 1), compiled in csrc/mrfv_n1.hip without
// packed-fp32 VALU ops: beside the K loop's MFMAs a v_pk_fma_f32 costs more issue than two v_fma_f32
// (MI355X_MICROARCH.md constants table, "packed f32 VALU ... an anti-lever beside MFMAs"); stage-1 k7 / k11 2.5-5 %
// faster so built (profiles/r06e_mrfv_nopk.log), while the wide stage-0 forms (256 VGPRs) lose 7 % and keep them
using mrfv_kfn = void (*)(stzs_conv_args);
mrfv_kfn stzs_mrfv_pick_n1(int ks, bool hr, bool ha, bool al, bool t64);
using mrfv_trio_kfn = void (*)(stzs_conv_args, stzs_conv_args, stzs_conv_args);
mrfv_trio_kfn stzs_mrfv_trio_pick_n1(bool hr);  // (the single-chunk trio forms, 64-row tiles)
