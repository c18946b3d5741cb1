// The HBM-bound MRF convs (the k3 convs of the generator's stage-1 AdaINResBlock1,
// 128 channels x 24 001 frames, intensity 192 flop/B < the bf16 ridge), as a PERSISTENT, software-pipelined
// kernel.  Same arithmetic as csrc/mrfv.hip (same staged bf16 operands, same K order per output, same
// epilogue and statistics grouping), so the two are bit-identical; different schedule:
//  * two 256-thread workgroups per CU (2 waves per SIMD: one workgroup's K loop overlaps the other's
//    transform / epilogue) walking 64-row x 128-channel tiles persistently -- an XCD-contiguous range per
//    XCD; each of the 4 waves owns 32 output channels;
//  * the raw input of the NEXT tile lands in LDS by LDS-DMA (global_load_lds, 16 B per lane) while this
//    tile's K loop runs: two tile buffers, so the HBM read of tile i+1 is in flight for a whole tile of
//    compute instead of the load -> transform -> MFMA sequence of a one-tile workgroup (whose staging
//    alone ran at 2.2 TB/s);
//  * LDS-DMA writes lane-linearly, so the tile keeps a 256-B row pitch and the bank spread comes from an XOR
//    swizzle of the 16-B chunk index instead of row padding: LDS position p of row r holds channel chunk
//    p ^ (r & 15) (each lane picks its GLOBAL source chunk accordingly); B-fragment reads and the in-place
//    transform are then conflict-free;
//  * the AdaIN + Snake (cosine form) transform runs IN PLACE on the landed tile (ds_read_b128 -> VALU ->
//    ds_write_b128);
//  * each wave's weights (3 taps x 128 ci x 32 co = 96 VGPRs) stay in registers for the workgroup's whole
//    life: the K loop issues no global load, so the in-order vmcnt never makes it wait on the in-flight DMA.
//  * the residual / accumulate-input rows of the epilogue come by LDS-DMA too (issued before the K loop), so
//    no VGPR load ever sits behind a pending DMA (the compiler would drain vmcnt there).
// Per iteration (tile u in buffer b, next tile un landing in buffer 1-b, unn the one after):
//   K loop(u) | cs(un) | vmcnt(0) | barrier | constant loads(unn) | transform(un) in place |
//   DMA(unn) -> buffer b | epilogue(u) (stores, statistics) | barrier | DMA residual rows(un)
#include "common.hpp"

namespace {

constexpr int NTH = 256;  // 4 waves: one group of 32 output channels each, all 64 rows of the tile
constexpr int BT = 64;    // time rows per tile (= one statistics chunk, STZS_CONV_STAT_ROWS)
constexpr int RB = 16;    // rows landed per DMA instruction round (4 waves x 4 rows of 256 B)
constexpr int RP = 256;  // LDS row pitch: 128 bf16 channels, 16 chunks of 16 B, XOR-swizzled
constexpr int NRB = 5;    // RB-row blocks per tile buffer (one DMA instruction per wave each): rows_in =
                          // 64 + 2 dil <= 80 (dil <= 8)
constexpr int BUF = NRB * RB * RP;
constexpr int RBUF = BT * RP;  // residual / accumulate-input tile (LDS-DMA, same swizzle)
constexpr int CS_BYTES = 5 * 128 * 4;

STZS_DEV float row_sum16p(float x) {  // sum over the 16 lanes of a DPP row (VALU only; as mrfv.hip)
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0xB1, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x4E, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x141, 0xF, 0xF, true));
    x += __int_as_float(__builtin_amdgcn_mov_dpp(__float_as_int(x), 0x140, 0xF, 0xF, true));
    return x;
}

template <int PACT, bool HR, bool HA>
__global__ __launch_bounds__(NTH, 2) void mrfp_conv(const stzs_conv_args a) {  // 2 workgroups per CU
    extern __shared__ __attribute__((aligned(16))) unsigned char smem[];
    constexpr int KS = 3, NKC = KS * 4;
    unsigned char* rbuf = smem + 2 * BUF;             // residual tile (HR)
    unsigned char* abuf = rbuf + (HR ? RBUF : 0);     // accumulate-input tile (HA)
    float* cs = reinterpret_cast<float*>(abuf + (HA ? RBUF : 0));
    const int tid = threadIdx.x, lane = tid & 63;
    const int wave = __builtin_amdgcn_readfirstlane(tid >> 6);  // wave-uniform (SGPR): uniform LDS-DMA bases
    const int cg = wave;  // output channel group (32 channels) of this wave
    const int dil = a.dil;
    const int tpb = (a.T_out + BT - 1) / BT;
    const int ntiles = a.B * tpb;
    const int G = gridDim.x;

    // ---- register-resident weights: this wave's 32 packed output rows, all 12 K-steps (frag32 layout)
    bf16x8 W[NKC][2];
    {
        const bf16x8* Wf = reinterpret_cast<const bf16x8*>(a.w) + cg * 128 + lane;
#pragma unroll
        for (int s = 0; s < NKC; ++s) {
            W[s][0] = Wf[s * 512];
            W[s][1] = Wf[s * 512 + 64];
        }
    }

    // ---- LDS-DMA of a raw tile: wave w, instruction j lands rows j*32 + 4w .. +3 (1 KB, lane-linear);
    // lane l -> row r = j*32 + 4w + (l >> 4), position p = l & 15 holding channel chunk p ^ (r & 15)
    const int dsw = (lane & 15) ^ ((wave * 4 + (lane >> 4)) & 15);
    // (uniform utterance base + 32-bit per-lane byte offsets: saddr loads, one v_med3 clamp + one mad per row)
    const unsigned ldx2 = (unsigned)a.ldx * 2u;
    auto dma = [&](int u, int b) {
        const int q = u / tpb, t0 = (u - q * tpb) * BT;
        const char* Xq = reinterpret_cast<const char*>(a.x) + (long)q * a.bsx * 2;
        unsigned char* dst = smem + b * BUF + wave * 4 * RP;
        const int r0 = t0 - a.pad + wave * 4 + (lane >> 4);
#pragma unroll
        for (int j = 0; j < NRB; ++j) {
            const int tin = min(max(r0 + j * RB, 0), a.T_in - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(Xq + ((unsigned)tin * ldx2 + (unsigned)dsw * 16u)),
                (__attribute__((address_space(3))) void*)(dst + j * RB * RP), 16, 0, 0);
        }
    };
    // ---- LDS-DMA of tile u's residual / accumulate-input rows (the epilogue then loads nothing into VGPRs:
    // a VGPR load behind a pending LDS-DMA makes the compiler drain vmcnt, i.e. wait for the next tile)
    auto dma_rows = [&](int u, const void* base, long bs, long ld, unsigned char* buf) {
        const int q = u / tpb, t0 = (u - q * tpb) * BT;
        const char* Rq = reinterpret_cast<const char*>(base) + (long)q * bs * 2;
        unsigned char* dst = buf + wave * 4 * RP;
        const int r0 = t0 + wave * 4 + (lane >> 4);
        const unsigned ld2 = (unsigned)ld * 2u;
#pragma unroll
        for (int j = 0; j < BT / RB; ++j) {
            const int t = min(r0 + j * RB, a.T_out - 1);
            __builtin_amdgcn_global_load_lds(
                (const __attribute__((address_space(1))) void*)(Rq + ((unsigned)t * ld2 + (unsigned)dsw * 16u)),
                (__attribute__((address_space(3))) void*)(dst + j * RB * RP), 16, 0, 0);
        }
    };
    auto dma_res = [&](int u) {
        if constexpr (HR) dma_rows(u, a.res, a.bsr, a.ldr, rbuf);
        if constexpr (HA) dma_rows(u, a.acc_in, a.bsa, a.lda, abuf);
    };
    // ---- per-channel prologue constants of tile u's utterance (128 threads): loads, then the LDS write
    float pm = 0.f, pr = 0.f, pg = 0.f, pb = 0.f;
    auto cload = [&](int u) {
        if (tid < 128 && a.pro_mode == STZS_PRO_ADAIN) {
            const int q = u / tpb;
            pm = a.pro_mean[(long)q * a.stat_bs + tid];
            pr = a.pro_rstd[(long)q * a.stat_bs + tid];
            pg = a.pro_gb[(long)q * a.gb_bs + tid];
            pb = a.pro_gb[(long)q * a.gb_bs + a.gb_beta_off + tid];
        }
    };
    const float alpha_c = (PACT == STZS_ACT_SNAKE && tid < 128) ? a.pro_alpha[tid] : 1.f;
    auto cwrite = [&]() {
        if (tid < 128) {
            float sc, sh;
            if (a.pro_mode == STZS_PRO_ADAIN) {
                sc = (1.f + pg) * pr;
                sh = pb - pm * sc;
            } else {
                sc = a.pro_cscale;
                sh = 0.f;
            }
            if constexpr (PACT == STZS_ACT_SNAKE) {
                const float h = 0.5f / alpha_c;
                const float w = alpha_c * 0.318309886183790672f;  // a / pi
                cs[tid] = sc * w;
                cs[128 + tid] = sh * w;
                cs[256 + tid] = sc;
                cs[384 + tid] = sh + h;
                cs[512 + tid] = -h;
            } else {
                cs[256 + tid] = sc;
                cs[384 + tid] = sh;
            }
        }
    };
    // ---- in-place transform of a landed tile: thread (rs, cv) owns position cv of rows rs + 16 i, i.e.
    // channel chunk c = cv ^ rs for every row it touches (one set of constants per thread)
    auto transform = [&](int u, int b) {
        if (a.flags & 1) return;  // diagnostic ablation (tools/mrfv_bench.py FLAGS=1)
        const int q = u / tpb, t0 = (u - q * tpb) * BT;
        const int rs = tid >> 4, cv = tid & 15;
        const int c0 = (cv ^ (rs & 15)) * 8;
        f32x2 ka[4], kb[4], ksc[4], ksh[4], km[4];
#pragma unroll
        for (int p = 0; p < 4; ++p) {
            ksc[p] = *reinterpret_cast<const f32x2*>(cs + 256 + c0 + 2 * p);
            ksh[p] = *reinterpret_cast<const f32x2*>(cs + 384 + c0 + 2 * p);
            if constexpr (PACT == STZS_ACT_SNAKE) {
                ka[p] = *reinterpret_cast<const f32x2*>(cs + c0 + 2 * p);
                kb[p] = *reinterpret_cast<const f32x2*>(cs + 128 + c0 + 2 * p);
                km[p] = *reinterpret_cast<const f32x2*>(cs + 512 + c0 + 2 * p);
            }
        }
        const float slope = a.pro_slope;
        unsigned char* base = smem + b * BUF + rs * RP + cv * 16;
        // every row of the buffer, branch-free (rows past rows_in hold clamped real rows, never read by the K
        // loop): all loads first, then the VALU work, then all stores -- no per-row latency chain
        uint4 v[NRB];
#pragma unroll
        for (int i = 0; i < NRB; ++i) v[i] = *reinterpret_cast<const uint4*>(base + i * RB * RP);
#pragma unroll
        for (int i = 0; i < NRB; ++i) {
            uint32_t* rw = reinterpret_cast<uint32_t*>(&v[i]);
            const int tin = t0 - a.pad + rs + RB * i;
            // zero padding of the ACTIVATED input, as a bit mask (a select lets the compiler branch around the
            // cosines per pair, with an exec-mask dance per pair)
            const uint32_t mk = (tin >= 0 && tin < a.T_in) ? 0xFFFFFFFFu : 0u;
#pragma unroll
            for (int p = 0; p < 4; ++p) {
                const uint32_t w = rw[p];
                const f32x2 x = f32x2{__uint_as_float(w << 16), __uint_as_float(w & 0xFFFF0000u)};
                f32x2 y = x * ksc[p] + ksh[p];  // v_pk_fma_f32
                if constexpr (PACT == STZS_ACT_SNAKE) {
                    const f32x2 t = x * ka[p] + kb[p];
                    const f32x2 cz = f32x2{__builtin_amdgcn_cosf(t.x), __builtin_amdgcn_cosf(t.y)};
                    y = cz * km[p] + y;
                } else if constexpr (PACT == STZS_ACT_LEAKY) {
                    y.x = y.x >= 0.f ? y.x : y.x * slope;
                    y.y = y.y >= 0.f ? y.y : y.y * slope;
                }
                rw[p] = pack2bf(y.x, y.y) & mk;
            }
        }
#pragma unroll
        for (int i = 0; i < NRB; ++i) *reinterpret_cast<uint4*>(base + i * RB * RP) = v[i];
    };

    // ---- K loop: K-step s = tap*4 + kq reads rows mt*16 + i16 + tap*dil, channels kq*32 + 8*qq .. +8
    const int i16 = lane & 15, qq = lane >> 4;
    auto xaddr = [&](int s) {
        const int rr = i16 + (s >> 2) * dil;
        return rr * RP + ((((s & 3) << 2) | qq) ^ (rr & 15)) * 16;
    };
    const int g = lane >> 4, n = lane & 15;
    const int co0 = cg * 32 + g * 8;
    const bool col_ok = co0 < a.Co;
    const int coc = col_ok ? co0 : 0;
    float bias[8];
#pragma unroll
    for (int i = 0; i < 8; ++i) bias[i] = a.bias ? a.bias[coc + i] : 0.f;
    const bool stat = a.stat_part != nullptr;
    const int nch = (a.T_out + 63) / 64;
    bf16_t* Y = reinterpret_cast<bf16_t*>(a.y);

    // XCD-aware walk: workgroup w runs on XCD w % 8 (the dispatcher deals ids round-robin over the XCDs), so give
    // every XCD a CONTIGUOUS range of tiles, walked by its workgroups with their count as stride: tiles being
    // processed at the same time on one XCD are neighbours, and their dilation halos are hits in its L2
    int u = blockIdx.x, st = G, uend = ntiles;
    if (G >= 8) {
        const int x = blockIdx.x & 7;
        u = (int)((long)x * ntiles / 8) + (blockIdx.x >> 3);
        st = (G - x + 7) >> 3;
        uend = (int)((long)(x + 1) * ntiles / 8);
    }
    if (u >= uend) return;  // (whole workgroup, before any barrier)
    int b = 0;
    // prologue: tile u landed and transformed in buffer 0, tile u + G in flight to buffer 1
    dma(u, 0);
    dma_res(u);
    cload(u);
    cwrite();
    __builtin_amdgcn_s_waitcnt(0);  // vmcnt(0) lgkmcnt(0): this thread's DMA rows + constant loads
    __syncthreads();
    transform(u, 0);
    if (u + st < uend) cload(u + st);
    dma(u + st < uend ? u + st : uend - 1, 1);
    asm volatile("" ::: "memory");
    __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only (see the loop's barrier)
    __builtin_amdgcn_s_barrier();
    asm volatile("" ::: "memory");

    // diagnostic phase timer (flags & 2048, tools/mrfv_bench.py FLAGS=2048): s_memtime deltas per phase of
    // wave 0 of workgroups 0..15, summed over the tiles, written as u64 [wg][8] into stat_part after the loop
    unsigned long long pacc[7] = {0, 0, 0, 0, 0, 0, 0}, ptl = __builtin_amdgcn_s_memtime();
#define PROFT(i)                                                        \
    if (a.flags & 2048) {                                               \
        const unsigned long long n_ = __builtin_amdgcn_s_memtime();     \
        pacc[i] += n_ - ptl;                                            \
        ptl = n_;                                                       \
    }
    while (true) {
        PROFT(6)
        const int un = u + st;
        f32x4 acc[2][4];
#pragma unroll
        for (int i = 0; i < 2; ++i)
#pragma unroll
            for (int j = 0; j < 4; ++j) acc[i][j] = f32x4{0.f, 0.f, 0.f, 0.f};
        {
            const unsigned char* Bb = smem + b * BUF;
            bf16x8 xf[4];
            const int a0 = xaddr(0);
#pragma unroll
            for (int mt = 0; mt < 4; ++mt) xf[mt] = *reinterpret_cast<const bf16x8*>(Bb + a0 + mt * 16 * RP);
#pragma unroll
            for (int s = 0; s < (a.flags & 2 ? 0 : NKC); ++s) {  // (FLAGS=2: no MFMAs, diagnostic)
                const int an = xaddr(s + 1 < NKC ? s + 1 : s);
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    acc[0][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W[s][0], xf[mt], acc[0][mt], 0, 0, 0);
                    acc[1][mt] = __builtin_amdgcn_mfma_f32_16x16x32_bf16(W[s][1], xf[mt], acc[1][mt], 0, 0, 0);
                    if (s + 1 < NKC) xf[mt] = *reinterpret_cast<const bf16x8*>(Bb + an + mt * 16 * RP);
                }
#pragma unroll
                for (int mt = 0; mt < 4; ++mt) {
                    __builtin_amdgcn_sched_group_barrier(0x008, 2, 0);
                    if (s + 1 < NKC) __builtin_amdgcn_sched_group_barrier(0x100, 1, 0);
                }
                __builtin_amdgcn_sched_barrier(0);
            }
        }
        PROFT(0)
        if (un < uend) cwrite();  // cs was last read by transform(u), finished before the last barrier
        __builtin_amdgcn_s_waitcnt(0);  // the DMA of tile un (issued a whole tile ago) has landed
        __syncthreads();                // every wave is done with buffer b; tile un + cs(un) visible
        PROFT(1)

        // ---- next tile: its constants' loads, then its in-place transform (no LDS-DMA is pending now: a
        // ds_write behind one would make the compiler drain vmcnt), then the DMA two tiles ahead
        const int q = u / tpb, t0 = (u - q * tpb) * BT;
        if (un + st < uend) cload(un + st);
        if (un < uend) transform(un, 1 - b);
        __builtin_amdgcn_sched_barrier(0);
        PROFT(2)
        dma(un + st < uend ? un + st : uend - 1, b);
        __builtin_amdgcn_sched_barrier(0);
        PROFT(3)

        if (!(a.flags & 4))  // (FLAGS=4: no epilogue, diagnostic)
        // ---- epilogue(u): lane (g, n): time t = t0 + m*16 + n, channels co0 .. co0 + 7; the tile is one
        // statistics partial
        {
            float ss[8], sq[8];
#pragma unroll
            for (int i = 0; i < 8; ++i) ss[i] = sq[i] = 0.f;
#pragma unroll
            for (int m = 0; m < 4; ++m) {
                const int t = t0 + m * 16 + n;
                const bool ok = col_ok && t < a.T_out;
                float v[8];
#pragma unroll
                for (int nt = 0; nt < 2; ++nt)
#pragma unroll
                    for (int r = 0; r < 4; ++r) v[nt * 4 + r] = acc[nt][m][r] + bias[nt * 4 + r];
                // residual / accumulate rows from their LDS tiles: row r's channel chunk c at position c ^ (r & 15)
                const int rrow = m * 16 + n;
                const int roff = rrow * RP + (((coc >> 3) ^ (rrow & 15)) << 4);
                if constexpr (HR) {
                    float f[8];
                    unpack8(*reinterpret_cast<const uint4*>(rbuf + roff), f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] += f[i];
                }
                if (a.alpha != 1.f) {  // (uniform; x * 1 == x, so skipping it changes no bit)
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] *= a.alpha;
                }
                if constexpr (HA) {
                    float f[8];
                    unpack8(*reinterpret_cast<const uint4*>(abuf + roff), f);
#pragma unroll
                    for (int i = 0; i < 8; ++i) v[i] = fmaf(a.beta, f[i], v[i]);
                }
                const uint4 o = pack8(v);
                if (ok) *reinterpret_cast<uint4*>(Y + (long)q * a.bsy + (long)t * a.ldy + coc) = o;
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
#pragma unroll
                for (int i = 0; i < 8; ++i) {
                    ss[i] = row_sum16p(ss[i]);
                    sq[i] = row_sum16p(sq[i]);
                }
                const int r0 = t0;
                if (n == 0 && col_ok && r0 < a.T_out) {
                    float* Pp = reinterpret_cast<float*>(a.stat_part) + (((long)q * nch + r0 / 64) * a.stat_ld + co0) * 2;
#pragma unroll
                    for (int i = 0; i < 8; ++i) {
                        Pp[2 * i] = ss[i];
                        Pp[2 * i + 1] = sq[i];
                    }
                }
            }
        }
        if (un >= uend) break;
        PROFT(4)
        // tile un transformed before its K loop: LDS writes complete + s_barrier, WITHOUT __syncthreads()'s
        // workgroup fence, which would also drain vmcnt -- i.e. wait for the DMA just issued
        asm volatile("" ::: "memory");
        __builtin_amdgcn_s_waitcnt(0xC07F);  // lgkmcnt(0) only
        __builtin_amdgcn_s_barrier();
        asm volatile("" ::: "memory");
        dma_res(un);  // every wave's epilogue(u) has read the residual tiles
        u = un;
        b = 1 - b;
        PROFT(5)
    }
#undef PROFT
    if ((a.flags & 2048) && a.stat_part && blockIdx.x < 16 && tid == 0) {
        unsigned long long* o = reinterpret_cast<unsigned long long*>(a.stat_part) + blockIdx.x * 8;
        for (int i = 0; i < 7; ++i) o[i] = pacc[i];
        o[7] = __builtin_amdgcn_s_getreg((31 << 11) | 4);  // HW_ID: wave / SIMD / CU / SE of this wave
    }
}

}  // namespace

// internal entry (csrc/mrfv.hip stzs_mrfv_conv_launch): the k3 FRAG32 residual convs with exactly one 128-channel
// input chunk and one 128-column output tile, when STZS_CONV_MRF_PIPE is set.  Returns 1 when not applicable
// (the caller falls back to mrfv_conv).
__attribute__((visibility("hidden"))) int stzs_mrfp_conv_launch(const stzs_conv_args& a, hipStream_t s) {
    if (a.ks != 3 || a.Ci != 128 || a.ci_pad != 128 || a.co_pad != 128 || a.ldx < 128 || a.dil > 8 ||
        !(a.flags & STZS_CONV_MRF_PIPE))
        return 1;
    if (a.pro_act != STZS_ACT_SNAKE && a.pro_act != STZS_ACT_LEAKY && a.pro_act != STZS_ACT_NONE) return 1;
    if (a.acc_in && a.pro_act != STZS_ACT_SNAKE) return 1;
    if (a.res && a.res_tdiv != 1) return 1;
    // only the residual forms: measured (tools/mrfv_bench.py, B 64, stage 1) c2 324 vs 352 us, c2 + accumulate 298
    // vs 351 us; without a residual both kernels sit at the same MFMA + VALU sum (~270 us), mrfv.hip keeps those
    if (!a.res) return 1;
    const int n_cu = stzs_cu_count();
    const bool R = a.res != nullptr, A = a.acc_in != nullptr;
    void (*k)(stzs_conv_args) = nullptr;
    if (a.pro_act == STZS_ACT_SNAKE)
        k = R ? (A ? mrfp_conv<STZS_ACT_SNAKE, true, true> : mrfp_conv<STZS_ACT_SNAKE, true, false>)
              : (A ? mrfp_conv<STZS_ACT_SNAKE, false, true> : mrfp_conv<STZS_ACT_SNAKE, false, false>);
    else if (a.pro_act == STZS_ACT_LEAKY)
        k = R ? mrfp_conv<STZS_ACT_LEAKY, true, false> : mrfp_conv<STZS_ACT_LEAKY, false, false>;
    else
        k = R ? mrfp_conv<STZS_ACT_NONE, true, false> : mrfp_conv<STZS_ACT_NONE, false, false>;
    const size_t lds = 2 * (size_t)BUF + (size_t)RBUF * ((a.res != nullptr) + (a.acc_in != nullptr)) + CS_BYTES;
    (void)hipFuncSetAttribute((const void*)k, hipFuncAttributeMaxDynamicSharedMemorySize, (int)lds);
    const long ntiles = (long)a.B * ((a.T_out + BT - 1) / BT);
    const long G = ntiles < 2L * n_cu ? ntiles : 2L * n_cu;  // two workgroups per CU
    hipLaunchKernelGGL(k, dim3((unsigned)G), dim3(NTH), lds, s, a);
    STZS_LAUNCH_CHECK();
    return STZS_OK;
}
