// The MRF conv (the generator's AdaINResBlock1 convs, about half of all
// synthesis time) on gfx950 -- also the k3 convs of the decoder / prosody-predictor AdaIN residual
// blocks (a9, a11) with a LeakyReLU or identity prologue and the nearest-x2 residual (t / res_tdiv).
//
// y[b, t, co] = epi( sum_{tap, ci} W[tap, co, ci] * snake(adain(x))[b, t + tap*dil - pad, ci] ),
// 128-channel input chunks, bf16 in / out, stride 1; epi = ((v + bias + res) * alpha + beta * acc_in),
// optional fused InstanceNorm statistics of the stored output.
//
// One 256-thread workgroup (4 waves, 2 x 2) per 128-row x 128-channel output tile, two workgroups
// per CU (<= 80 KB LDS each):
//  * STAGING, per 128-channel input chunk: the tile's rows plus the dilation halo, one batch of 16-B
//    loads per thread, the AdaIN affine folded into per-channel constants that sit in the idle weight
//    ring slot, and the Snake in its cosine form  x + 1/(2a) - cos(2 a x)/(2a)  (three FMAs and one
//    v_cos_f32 per element) -> bf16 rows with a 272-B pitch (conflict-free ds_read_b128).
//  * K LOOP: one K-step = 32 input channels of one tap = 16 MFMAs (v_mfma_f32_16x16x32_bf16) per
//    wave.  Weights stream by LDS-DMA through a 4-slot ring, filled three K-steps ahead; each K-step
//    does one counted vmcnt + s_barrier, and the NEXT K-step's fragments are read (ds_read_b128)
//    between the current K-step's MFMAs.  The K-step body is branch-free (past the end a fill is a
//    harmless re-copy into a retired slot), so the compiler's lgkmcnt waits stay counted.
//  * EPILOGUE straight from the accumulators: the MFMA operands are swapped (weights = A, input = B,
//    so C is [channel][time]) and the packer permutes channels (STZS_CONV_W_LANE16) so that each lane
//    holds 16 consecutive channels of one time step -> 32-B vector residual / accumulate loads and
//    stores, no LDS round trip.  Statistics: per-lane sums, xor-reduced over the 16 time lanes, one
//    deterministic fp32 partial per (utterance, 64-row chunk, channel).
// (A persistent warp-specialised variant -- producer waves staging the next tile beside the MFMA
// waves -- measured 2x slower: see DESIGN.md, "MRF conv".)
#include "common.hpp"

namespace {

constexpr int NTH = 256;
constexpr int BT = 128, BCO = 128;
constexpr int P = 272;  // staged input row pitch, bytes
constexpr int NSL = 4, SLOT = 8192;
constexpr int SB = 12;  // staged 16-B vectors per thread: 16 row lanes x 12 = 192 >= rows_in

STZS_DEV int gswz(int r) { return (0x1320 >> (((r >> 2) & 3) * 4)) & 3; }

// sum over the 16 lanes of a DPP row, result in every lane: VALU-only (no ds_bpermute)
STZS_DEV float row_sum16(float x) {
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));   // quad_perm 1,0,3,2
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));   // quad_perm 2,3,0,1
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true));  // row_half_mirror
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, true));  // row_mirror
    return x;
}

// NR: weight-ring slots (power of 2), filled NR - 1 K-steps ahead.  NR = 4 at two workgroups per CU; NR = 8 (64 KB of
// ring) when the grid is smaller than the CU count (batch 1: 16-64 workgroups whose K loop is a serial chain of
// LDS-DMA round trips -- the bytes in flight per CU, not the MFMAs, set its pace).  Same K order: bit-identical.
template <int PACT, bool HR, bool HA, int NR>
__global__ __launch_bounds__(NTH, NR == 4 ? 2 : 1) void mrf_conv(const stzs_conv_args a) {
    constexpr int NSL = NR;
    constexpr int FD = NR - 1;  // fill distance
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = a.ks, dil = a.dil;
    const int rows_in = BT + (ks - 1) * dil;
    unsigned char* ring = smem + ((rows_in * P + 15) & ~15);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int wt = wave >> 1, wc = wave & 1;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int nx = gridDim.x;
    const int lin = (a.flags & STZS_CONV_LINEAR_IDS) ? blockIdx.y * nx + blockIdx.x
                                                      : xcd_remap(blockIdx.y * nx + blockIdx.x, nx * gridDim.y);
    const int by = lin / nx, bx = lin - by * nx;  // (co tile, utterance x time tile)
    const int bq = bx / tpb;
    const int t0 = (bx - bq * tpb) * BT;
    const int nchunk = a.ci_pad >> 7;
    const int NK = nchunk * ks * 4;
    const bf16_t* Wt = reinterpret_cast<const bf16_t*>(a.w) + (long)by * NK * (BCO * 32);
    auto fill = [&](int k) {  // k >= NK: a harmless re-copy (clamped source) into a retired slot
        const bf16_t* src = Wt + (long)(k < NK ? k : NK - 1) * (BCO * 32) + wave * 1024 + lane * 8;
        unsigned char* dst = ring + (k & (NSL - 1)) * SLOT + wave * 2048;
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                         (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)(src + 512),
                                         (__attribute__((address_space(3))) void*)(dst + 1024), 16, 0, 0);
    };
    f32x4 acc[4][4];  // [nt: channel tile][mt: time tile]
    auto gate_wait = [&]() {  // fill k+1 landed; fills k+2 .. k+FD-1 (2 LDS-DMA instructions each) may fly
        if constexpr (FD == 3)
            __builtin_amdgcn_s_waitcnt(0x0F72);
        else
            __builtin_amdgcn_s_waitcnt(0x0F70 | (2 * (FD - 2)));
    };
#pragma unroll
    for (int i = 0; i < 4; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};

    const int brow = wc * 64 + (lane & 15);
    const int boff0 = brow * 64 + (((lane >> 4) ^ gswz(brow)) << 4);
    const int arow0 = (wt * 64 + (lane & 15)) * P + (lane >> 4) * 16;
    bf16x8 fa0[4], fb0[4], fa1[4], fb1[4];
    auto readB = [&](bf16x8 (&fb)[4], int k) {
        const unsigned char* wl = ring + (k & (NSL - 1)) * SLOT + boff0;
#pragma unroll
        for (int nt = 0; nt < 4; ++nt) fb[nt] = *reinterpret_cast<const bf16x8*>(wl + nt * 1024);
    };
    auto readA = [&](bf16x8 (&fx)[4], int off) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) fx[mt] = *reinterpret_cast<const bf16x8*>(smem + off + mt * 16 * P);
    };
    auto mma = [&](const bf16x8 (&fx)[4], const bf16x8 (&fw)[4]) {
#pragma unroll
        for (int nt = 0; nt < 4; ++nt)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
                acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[nt], fx[mt], acc[nt][mt], 0, 0, 0);
    };

    const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (long)bq * a.bsx;
    const int cv = tid & 15, rsub = tid >> 4;
#pragma unroll
    for (int i = 0; i < FD - 1; ++i) fill(i);
    int k = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();  // every wave is done reading the previous chunk's input tile
        if (!(a.flags & 1)) {
            const int c = cc * 128 + cv * 8;
            const bool c_ok = c < a.Ci;  // vectors past Ci (ci_pad > Ci) are zero; weights there are 0
            const int cl = c_ok ? c : 0;
            uint4 raw[SB];
            bool okv[SB];
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                int tin = t0 - a.pad + rsub + 16 * i;
                okv[i] = c_ok && tin >= 0 && tin < a.T_in;
                tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                raw[i] = *reinterpret_cast<const uint4*>(X + (long)tin * a.ldx + cl);
            }
            // per-channel constants, computed once per channel by 128 threads into the ring slot that
            // stays idle until this chunk's first K-step fills it (slot (k + FD) & (NSL - 1)):
            //   t = x*ka + kb (revolutions of cos(2 a y)),  out = cos(t) * km + (x*ksc + ksh)
            float* cs = reinterpret_cast<float*>(ring + ((k + FD) & (NSL - 1)) * SLOT);
            if (tid < 128) {
                const int ch = cc * 128 + tid;
                const bool ok = ch < a.Ci;
                float sc = 0.f, sh = 0.f;
                if (ok && a.pro_mode == STZS_PRO_ADAIN) {
                    const float mu = a.pro_mean[(long)bq * a.stat_bs + ch];
                    const float rs = a.pro_rstd[(long)bq * a.stat_bs + ch];
                    const float gm = a.pro_gb[(long)bq * a.gb_bs + ch];
                    const float be = a.pro_gb[(long)bq * a.gb_bs + a.gb_beta_off + ch];
                    sc = (1.f + gm) * rs;
                    sh = be - mu * sc;
                } else if (ok) {
                    sc = a.pro_cscale;
                }
                if constexpr (PACT == STZS_ACT_SNAKE) {
                    const float al = ok ? a.pro_alpha[ch] : 1.f;
                    const float h = 0.5f / al;
                    const float w = al * 0.318309886183790672f;  // a / pi
                    cs[tid] = sc * w;
                    cs[128 + tid] = sh * w;
                    cs[256 + tid] = sc;
                    cs[384 + tid] = sh + h;
                    cs[512 + tid] = -h;
                } else {  // LeakyReLU / identity: y = x*sc + sh
                    cs[256 + tid] = sc;
                    cs[384 + tid] = sh;
                }
            }
            __syncthreads();
            float ka[8], kb[8], ksc[8], ksh[8], km[8];
#pragma unroll
            for (int j = 0; j < 8; ++j) {
                ksc[j] = cs[256 + cv * 8 + j];
                ksh[j] = cs[384 + cv * 8 + j];
                if constexpr (PACT == STZS_ACT_SNAKE) {
                    ka[j] = cs[cv * 8 + j];
                    kb[j] = cs[128 + cv * 8 + j];
                    km[j] = cs[512 + cv * 8 + j];
                }
            }
            const float slope = a.pro_slope;
#pragma unroll
            for (int i = 0; i < SB; ++i) {
                const int r = rsub + 16 * i;
                if (r < rows_in) {
                    const uint32_t w[4] = {raw[i].x, raw[i].y, raw[i].z, raw[i].w};
                    uint32_t o[4];
#pragma unroll
                    for (int p = 0; p < 4; ++p) {
                        const float x0 = __uint_as_float(w[p] << 16), x1 = __uint_as_float(w[p] & 0xFFFF0000u);
                        const int j0 = 2 * p, j1 = 2 * p + 1;
                        float y0 = fmaf(x0, ksc[j0], ksh[j0]), y1 = fmaf(x1, ksc[j1], ksh[j1]);
                        if constexpr (PACT == STZS_ACT_SNAKE) {
                            y0 = fmaf(__builtin_amdgcn_cosf(fmaf(x0, ka[j0], kb[j0])), km[j0], y0);
                            y1 = fmaf(__builtin_amdgcn_cosf(fmaf(x1, ka[j1], kb[j1])), km[j1], y1);
                        } else if constexpr (PACT == STZS_ACT_LEAKY) {
                            y0 = y0 >= 0.f ? y0 : y0 * slope;
                            y1 = y1 >= 0.f ? y1 : y1 * slope;
                        }
                        o[p] = okv[i] ? pack2bf(y0, y1) : 0u;
                    }
                    *reinterpret_cast<uint4*>(smem + r * P + cv * 16) = make_uint4(o[0], o[1], o[2], o[3]);
                }
            }
        }
        __syncthreads();
        if (cc == 0) {  // (the barrier above drained fills 0 .. FD-2)
            fill(FD - 1);
            readB(fb0, 0);
        }
        readA(fa0, arow0);
        const int ntap = (a.flags & 2) ? 1 : ks;
        // fill k+1 landed (fill k+2 may stay in flight) -> barrier -> fill k+3 into the retired
        // slot k-1 -> NEXT fragments read between the CURRENT K-step's 16 MFMAs
#define STZS_MRF_STEP(FX, FW, NX, NW, AOFF)                                     \
    {                                                                           \
        gate_wait();                                                            \
        __builtin_amdgcn_s_barrier();                                           \
        fill(k + FD);                                                           \
        __builtin_amdgcn_sched_barrier(0);                                      \
        readB(NW, k + 1);                                                       \
        readA(NX, AOFF);                                                        \
        mma(FX, FW);                                                            \
        _Pragma("unroll") for (int ii = 0; ii < 8; ++ii) {                      \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                  \
        }                                                                       \
        __builtin_amdgcn_sched_group_barrier(0x008, 8, 0);                      \
        __builtin_amdgcn_sched_barrier(0);                                      \
        ++k;                                                                    \
    }
        for (int tap = 0; tap + 1 < ntap; ++tap) {
            const int ab = arow0 + tap * dil * P;
            STZS_MRF_STEP(fa0, fb0, fa1, fb1, ab + 64)
            STZS_MRF_STEP(fa1, fb1, fa0, fb0, ab + 128)
            STZS_MRF_STEP(fa0, fb0, fa1, fb1, ab + 192)
            STZS_MRF_STEP(fa1, fb1, fa0, fb0, ab + dil * P)
        }
        {  // last tap of the chunk (peeled: the final K-step of the last chunk is special)
            const int ab = arow0 + (ntap - 1) * dil * P;
            STZS_MRF_STEP(fa0, fb0, fa1, fb1, ab + 64)
            STZS_MRF_STEP(fa1, fb1, fa0, fb0, ab + 128)
            STZS_MRF_STEP(fa0, fb0, fa1, fb1, ab + 192)
            if (cc + 1 < nchunk) STZS_MRF_STEP(fa1, fb1, fa0, fb0, arow0)  // next chunk re-reads A after staging
        }
#undef STZS_MRF_STEP
    }
    // The final K-step needs no wait, barrier, fill or prefetch: its fragments are in registers.  The
    // epilogue's residual / accumulate loads go out first so their latency hides under its MFMAs.
    // Output row of GEMM row q: t = q, or for the polyphase ConvTranspose (ups > 0) column n = phase p *
    // Co + channel (a 16-channel group never straddles phases, Co % 16 == 0): t = q*ups + p - ups_pad,
    // valid in [0, T_final), shifted by refl (ReflectionPad(1,0)).
    const int gq = lane >> 4, n = lane & 15;
    const int co0 = by * BCO + wc * 64 + gq * 16;
    const int ph = a.ups > 0 ? co0 / a.Co : 0;
    const bool col_ok = a.ups > 0 ? co0 < a.ups * a.Co : co0 < a.Co;
    const int cof = col_ok ? co0 - ph * a.Co : 0;  // channel of this lane group's first value
    const int t_hi = a.ups > 0 ? a.T_final + a.refl - 1 : a.T_out - 1;
    auto orow = [&](int mt, bool& ok) {
        const int q = t0 + wt * 64 + mt * 16 + n;
        if (a.ups > 0) {
            const int t = q * a.ups + ph - a.ups_pad;
            ok = col_ok && q < a.T_out && t >= 0 && t < a.T_final;
            return t + a.refl;
        }
        ok = col_ok && q < a.T_out;
        return q;
    };
    const int coc = cof;
    uint4 rr[4][2], aa[4][2];
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        bool okm;
        const int t = orow(mt, okm);
        const int tc = t < 0 ? 0 : (t > t_hi ? t_hi : t);
        if constexpr (HR) {  // (row t / res_tdiv: the nearest-x2 shortcut of an upsampling block)
            const bf16_t* p = reinterpret_cast<const bf16_t*>(a.res) + (long)bq * a.bsr + (long)(tc / a.res_tdiv) * a.ldr + coc;
            rr[mt][0] = *reinterpret_cast<const uint4*>(p);
            rr[mt][1] = *reinterpret_cast<const uint4*>(p + 8);
        }
        if constexpr (HA) {
            const bf16_t* p = reinterpret_cast<const bf16_t*>(a.acc_in) + (long)bq * a.bsa + (long)tc * a.lda + coc;
            aa[mt][0] = *reinterpret_cast<const uint4*>(p);
            aa[mt][1] = *reinterpret_cast<const uint4*>(p + 8);
        }
    }
    mma(fa1, fb1);
    if (a.flags & 4) return;

    // ---------------- epilogue straight from the accumulators
    // lane (gq = lane >> 4, n = lane & 15): time t = t0 + wt*64 + mt*16 + n, channels co0 .. co0+15
    // (packed row nt*16 + gq*4 + r of the wave's 64 columns  <->  channel co0 + nt*4 + r)
    float bias[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) bias[i] = a.bias ? a.bias[coc + i] : 0.f;
    const bool stat = a.stat_part != nullptr;
    float ss[16], sq[16];
#pragma unroll
    for (int i = 0; i < 16; ++i) ss[i] = sq[i] = 0.f;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);
    {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) {
            bool ok;
            const int t = orow(mt, ok);
            float v[16];
#pragma unroll
            for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[nt][mt][r] + bias[nt * 4 + r];
            if constexpr (HR) {
                float f[16];
                unpack8(rr[mt][0], f);
                unpack8(rr[mt][1], f + 8);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] += f[i];
            }
#pragma unroll
            for (int i = 0; i < 16; ++i) v[i] *= a.alpha;
            if constexpr (HA) {
                float f[16];
                unpack8(aa[mt][0], f);
                unpack8(aa[mt][1], f + 8);
#pragma unroll
                for (int i = 0; i < 16; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
            }
            const uint4 o0 = pack8(v), o1 = pack8(v + 8);
            if (ok) {
                bf16_t* p = Y + (long)bq * a.bsy + (long)t * a.ldy + cof;
                *reinterpret_cast<uint4*>(p) = o0;
                *reinterpret_cast<uint4*>(p + 8) = o1;
            }
            if (a.refl && ok && t == 2) {  // ReflectionPad(1,0): row 0 mirrors source row 1 (+ row 0's residual)
                float w[16];
#pragma unroll
                for (int nt = 0; nt < 4; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) w[nt * 4 + r] = acc[nt][mt][r] + bias[nt * 4 + r];
                if constexpr (HR) {
                    float f[16];
                    load8(reinterpret_cast<const bf16_t*>(a.res) + (long)bq * a.bsr + coc, f);
                    load8(reinterpret_cast<const bf16_t*>(a.res) + (long)bq * a.bsr + coc + 8, f + 8);
#pragma unroll
                    for (int i = 0; i < 16; ++i) w[i] += f[i];
                }
#pragma unroll
                for (int i = 0; i < 16; ++i) w[i] *= a.alpha;
                bf16_t* p = Y + (long)bq * a.bsy + cof;
                *reinterpret_cast<uint4*>(p) = pack8(w);
                *reinterpret_cast<uint4*>(p + 8) = pack8(w + 8);
            }
            if (stat && ok) {  // statistics of the stored (bf16-rounded) values
                float f[16];
                unpack8(o0, f);
                unpack8(o1, f + 8);
#pragma unroll
                for (int i = 0; i < 16; ++i) {
                    ss[i] += f[i];
                    sq[i] = fmaf(f[i], f[i], sq[i]);
                }
            }
        }
    }
    if (stat) {
        // the 16 time lanes (n) of a channel group: xor-reduce, one 64-row partial per wave
#pragma unroll
        for (int i = 0; i < 16; ++i) {
            ss[i] = row_sum16(ss[i]);
            sq[i] = row_sum16(sq[i]);
        }
        const int r0 = t0 + wt * 64;
        if (n == 0 && col_ok && r0 < a.T_out) {
            const int nch = (a.T_out + 63) / 64;
            float* Pp = reinterpret_cast<float*>(a.stat_part) + (((long)bq * nch + r0 / 64) * a.stat_ld + co0) * 2;
#pragma unroll
            for (int i = 0; i < 16; ++i) {
                Pp[2 * i] = ss[i];
                Pp[2 * i + 1] = sq[i];
            }
        }
    }
}

// ---------------------------------------------------------------------------------------------
// Narrow conv (Co <= 32): conv_post (128 -> 22 channels, k 7, LeakyReLU(0.01) prologue, fp32 out) at
// the full frame rate.  A 128-column tile would waste 5/6 of the MFMAs; here a workgroup owns 256
// time rows x 32 channels, each wave 64 rows x 32 channels = 4 x 2 accumulators, 8 MFMAs per K-step.
// Weights: [NK][32][32] bf16 K-steps (2 KB, packed with STZS_CONV_W_NARROW32: packed row
// nt*16 + g*4 + r holds channel g*8 + nt*4 + r, so each lane ends up with 8 consecutive channels)
// through a 4-slot LDS-DMA ring filled by waves 0-1; the staging / K-step / epilogue scheme is the
// MRF kernel's.
constexpr int NBT = 256;
constexpr int NSLOT_B = 2048;
constexpr int NSB = 9;  // staged vectors per thread per batch (two batches: 16 x 18 = 288 rows)

__global__ __launch_bounds__(NTH, 2) void narrow_conv(const stzs_conv_args a) {
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    const int ks = a.ks, dil = a.dil;
    const int rows_in = NBT + (ks - 1) * dil;
    unsigned char* ring = smem + ((rows_in * P + 15) & ~15);
    const int tid = threadIdx.x, lane = tid & 63, wave = tid >> 6;
    const int tpb = (a.T_out + NBT - 1) / NBT;
    const int bx = (a.flags & STZS_CONV_LINEAR_IDS) ? (int)blockIdx.x : xcd_remap(blockIdx.x, gridDim.x);
    const int bq = bx / tpb;
    const int t0 = (bx - bq * tpb) * NBT;
    const int nchunk = a.ci_pad >> 7;
    const int NK = nchunk * ks * 4;
    const bf16_t* Wt = reinterpret_cast<const bf16_t*>(a.w);
    auto fill = [&](int k) {  // 2 KB per K-step: one 1-KB piece from each of waves 0 and 1
        if (wave < 2) {
            const bf16_t* src = Wt + (long)(k < NK ? k : NK - 1) * 1024 + wave * 512 + lane * 8;
            unsigned char* dst = ring + (k & (NSL - 1)) * NSLOT_B + wave * 1024;
            __builtin_amdgcn_global_load_lds((const __attribute__((address_space(1))) void*)src,
                                             (__attribute__((address_space(3))) void*)dst, 16, 0, 0);
        }
    };
    f32x4 acc[2][4];
#pragma unroll
    for (int i = 0; i < 2; ++i)
#pragma unroll
        for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
    const int brow = lane & 15;
    const int boff0 = brow * 64 + (((lane >> 4) ^ gswz(brow)) << 4);
    const int arow0 = (wave * 64 + (lane & 15)) * P + (lane >> 4) * 16;
    bf16x8 fa0[4], fb0[2], fa1[4], fb1[2];
    auto readB = [&](bf16x8 (&fb)[2], int k) {
        const unsigned char* wl = ring + (k & (NSL - 1)) * NSLOT_B + boff0;
        fb[0] = *reinterpret_cast<const bf16x8*>(wl);
        fb[1] = *reinterpret_cast<const bf16x8*>(wl + 1024);
    };
    auto readA = [&](bf16x8 (&fx)[4], int off) {
#pragma unroll
        for (int mt = 0; mt < 4; ++mt) fx[mt] = *reinterpret_cast<const bf16x8*>(smem + off + mt * 16 * P);
    };
    auto mma = [&](const bf16x8 (&fx)[4], const bf16x8 (&fw)[2]) {
#pragma unroll
        for (int nt = 0; nt < 2; ++nt)
#pragma unroll
            for (int mt = 0; mt < 4; ++mt)
                acc[nt][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(fw[nt], fx[mt], acc[nt][mt], 0, 0, 0);
    };
    const bf16_t* X = reinterpret_cast<const bf16_t*>(a.x) + (long)bq * a.bsx;
    const int cv = tid & 15, rsub = tid >> 4;
    const float csc = a.pro_cscale, slope = a.pro_slope;
    const bool leaky = a.pro_act == STZS_ACT_LEAKY;
    fill(0);
    fill(1);
    int k = 0;
    for (int cc = 0; cc < nchunk; ++cc) {
        __syncthreads();
        const int c = cc * 128 + cv * 8;
        const bool c_ok = c < a.Ci;
        const int cl = c_ok ? c : 0;
#pragma unroll
        for (int bt = 0; bt < 2; ++bt) {  // two staging batches of NSB vectors per thread
            uint4 raw[NSB];
#pragma unroll
            for (int i = 0; i < NSB; ++i) {
                int tin = t0 - a.pad + rsub + 16 * (bt * NSB + i);
                tin = tin < 0 ? 0 : (tin >= a.T_in ? a.T_in - 1 : tin);
                raw[i] = *reinterpret_cast<const uint4*>(X + (long)tin * a.ldx + cl);
            }
#pragma unroll
            for (int i = 0; i < NSB; ++i) {
                const int r = rsub + 16 * (bt * NSB + i);
                if (r < rows_in) {
                    const int tin = t0 - a.pad + r;
                    const bool ok = c_ok && tin >= 0 && tin < a.T_in;
                    float f[8];
                    unpack8(raw[i], f);
#pragma unroll
                    for (int j = 0; j < 8; ++j) {
                        float y = f[j] * csc;
                        if (leaky) y = y >= 0.f ? y : y * slope;
                        f[j] = ok ? y : 0.f;
                    }
                    *reinterpret_cast<uint4*>(smem + r * P + cv * 16) = pack8(f);
                }
            }
        }
        __syncthreads();
        if (cc == 0) {
            fill(2);
            readB(fb0, 0);
        }
        readA(fa0, arow0);
        // one K-step: fill k+1 landed (waves 0-1 hold one piece of fill k+2 in flight) -> barrier ->
        // fill k+3 -> next fragments read between the current 8 MFMAs
#define STZS_NARROW_STEP(FX, FW, NX, NW, AOFF)                                  \
    {                                                                           \
        __builtin_amdgcn_s_waitcnt(0x0F71);                                     \
        __builtin_amdgcn_s_barrier();                                           \
        fill(k + 3);                                                            \
        __builtin_amdgcn_sched_barrier(0);                                      \
        readB(NW, k + 1);                                                       \
        readA(NX, AOFF);                                                        \
        mma(FX, FW);                                                            \
        _Pragma("unroll") for (int ii = 0; ii < 6; ++ii) {                      \
            __builtin_amdgcn_sched_group_barrier(0x008, 1, 0);                  \
            __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);                  \
        }                                                                       \
        __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);                      \
        __builtin_amdgcn_sched_barrier(0);                                      \
        ++k;                                                                    \
    }
        for (int tap = 0; tap + 1 < ks; ++tap) {
            const int ab = arow0 + tap * dil * P;
            STZS_NARROW_STEP(fa0, fb0, fa1, fb1, ab + 64)
            STZS_NARROW_STEP(fa1, fb1, fa0, fb0, ab + 128)
            STZS_NARROW_STEP(fa0, fb0, fa1, fb1, ab + 192)
            STZS_NARROW_STEP(fa1, fb1, fa0, fb0, ab + dil * P)
        }
        const int ab = arow0 + (ks - 1) * dil * P;
        STZS_NARROW_STEP(fa0, fb0, fa1, fb1, ab + 64)
        STZS_NARROW_STEP(fa1, fb1, fa0, fb0, ab + 128)
        STZS_NARROW_STEP(fa0, fb0, fa1, fb1, ab + 192)
        if (cc + 1 < nchunk) {
            STZS_NARROW_STEP(fa1, fb1, fa0, fb0, arow0)
        } else {
            mma(fa1, fb1);
        }
#undef STZS_NARROW_STEP
    }
    // epilogue: lane (g, n) holds time t = t0 + wave*64 + mt*16 + n, channels g*8 .. g*8+7 (fp32)
    const int g = lane >> 4, n = lane & 15;
    const int ch0 = g * 8;
    if (ch0 >= a.Co) return;
    float bias[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bias[i] = (a.bias && ch0 + i < a.Co) ? a.bias[ch0 + i] : 0.f;
    float* Y = reinterpret_cast<float*>(a.y);
#pragma unroll
    for (int mt = 0; mt < 4; ++mt) {
        const int t = t0 + wave * 64 + mt * 16 + n;
        if (t < a.T_out) {
            float v[8];
#pragma unroll
            for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                for (int r = 0; r < 4; ++r) v[nt * 4 + r] = (acc[nt][mt][r] + bias[nt * 4 + r]) * a.alpha;
            store8(Y + (long)bq * a.bsy + (long)t * a.ldy + ch0, v);
        }
    }
}

}  // namespace

// internal entry used by stzs_conv1d for STZS_CONV_W_LANE16 weights
__attribute__((visibility("hidden"))) int stzs_mrf_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    const int rows_in = BT + (a.ks - 1) * a.dil;
    if (a.stride != 1 || a.cic != 128 || a.ci_pad % 128 || a.Co % 16 || rows_in > 16 * SB ||
        a.in_dtype != STZS_BF16 || a.out_dtype != STZS_BF16 || a.gate || a.epi_act != STZS_ACT_NONE ||
        (a.ups && (a.acc_in || a.stat_part || a.res_tdiv != 1)) ||
        a.ldy % 8 || a.bsy % 8 || (a.res && (a.ldr % 8 || a.bsr % 8)) || (a.acc_in && (a.lda % 8 || a.bsa % 8)))
        return STZS_ESHAPE;
    if (a.pro_act == STZS_ACT_SNAKE && !a.pro_alpha) return STZS_EINVAL;
    dim3 grid((unsigned)a.B * (unsigned)((a.T_out + BT - 1) / BT), a.co_pad / BCO);
    // a grid below the CU count (batch 1) gets the deep ring: one workgroup per CU anyway, more bytes in flight
    const bool deep = (long)grid.x * grid.y < stzs_cu_count();
    const size_t lds = (((size_t)rows_in * P + 15) & ~(size_t)15) + (deep ? 8 : NSL) * SLOT;
    if (lds > 160 * 1024) return STZS_ESHAPE;
    void (*k)(stzs_conv_args) = nullptr;
#define STZS_MRF_PICK(NR)                                                                                        \
    if (a.pro_act == STZS_ACT_SNAKE) {                                                                           \
        if (a.res && a.acc_in)                                                                                   \
            k = mrf_conv<STZS_ACT_SNAKE, true, true, NR>;                                                        \
        else if (a.res)                                                                                          \
            k = mrf_conv<STZS_ACT_SNAKE, true, false, NR>;                                                       \
        else if (a.acc_in)                                                                                       \
            k = mrf_conv<STZS_ACT_SNAKE, false, true, NR>;                                                       \
        else                                                                                                     \
            k = mrf_conv<STZS_ACT_SNAKE, false, false, NR>;                                                      \
    } else if (!a.acc_in) { /* the AdaIN residual blocks of the decoder / prosody predictor */                   \
        if (a.pro_act == STZS_ACT_LEAKY)                                                                         \
            k = a.res ? mrf_conv<STZS_ACT_LEAKY, true, false, NR> : mrf_conv<STZS_ACT_LEAKY, false, false, NR>;  \
        else if (a.pro_act == STZS_ACT_NONE)                                                                     \
            k = a.res ? mrf_conv<STZS_ACT_NONE, true, false, NR> : mrf_conv<STZS_ACT_NONE, false, false, NR>;    \
    }
    if (deep) {
        STZS_MRF_PICK(8)
    } else {
        STZS_MRF_PICK(4)
    }
#undef STZS_MRF_PICK
    if (!k) return STZS_ESHAPE;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(k, grid, dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}

// internal entry used by stzs_conv1d for STZS_CONV_W_NARROW32 weights
__attribute__((visibility("hidden"))) int stzs_narrow_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    const int rows_in = NBT + (a.ks - 1) * a.dil;
    if (a.stride != 1 || a.cic != 128 || a.ci_pad % 128 || a.Co > 32 || a.co_pad != 128 || rows_in > 16 * 2 * NSB ||
        a.in_dtype != STZS_BF16 || a.out_dtype != STZS_F32 || a.ups || a.gate || a.res || a.acc_in ||
        a.pro_mode != STZS_PRO_NONE || (a.pro_act != STZS_ACT_LEAKY && a.pro_act != STZS_ACT_NONE) ||
        a.epi_act != STZS_ACT_NONE || a.stat_part || a.ldy % 8 || a.bsy % 8 || a.ldy < ((a.Co + 7) / 8) * 8)
        return STZS_ESHAPE;
    const size_t lds = (((size_t)rows_in * P + 15) & ~(size_t)15) + NSL * NSLOT_B;
    dim3 grid((unsigned)a.B * (unsigned)((a.T_out + NBT - 1) / NBT));
    (void)hipFuncSetAttribute((const void*)narrow_conv, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    hipLaunchKernelGGL(narrow_conv, grid, dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
